set -e
ROOT=$(pwd)
OUT=gpurun_out/r4n
mkdir -p $OUT
for pass in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_ACTIVE_INST_VALU"; do
  name=pmc_lm_$(echo $pass | cut -d' ' -f1)
  (cd /tmp && export TMPDIR=/tmp && MOPT_SYNC_CHECK=1 timeout -s KILL 150 rocprofv3 --output-format csv --pmc $pass -d "$ROOT/$OUT/$name" -o run -- python3 "$ROOT/scripts/bench_configs.py" --config lm-125m --steps 2 --warmup 1 > "$ROOT/$OUT/$name.log" 2>&1)
done
echo done
