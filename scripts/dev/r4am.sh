set -e
OUT=gpurun_out/r4am
mkdir -p $OUT
ROOT=$(pwd)
run() {  # run NAME COUNTERS...
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --output-format csv \
      --pmc "$@" -d "$ROOT/$OUT/$name" -o run -- \
      python3 "$ROOT/scripts/bench_configs.py" --config resnet20 --steps 3 --warmup 2 \
      > "$ROOT/$OUT/$name.log" 2>&1)
}
run mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run wait SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
run fetch FETCH_SIZE
run write WRITE_SIZE
echo done
