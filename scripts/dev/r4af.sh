set -e
OUT=gpurun_out/r4af
mkdir -p $OUT
ROOT=$(pwd)
run() {  # run NAME COUNTERS...
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --output-format csv \
      --pmc "$@" -d "$ROOT/$OUT/$name" -o run -- \
      python3 "$ROOT/scripts/gemm_bench.py" --shapes lm.qkv --no-torch --iters 5 \
      > "$ROOT/$OUT/$name.log" 2>&1)
}
run mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
run wait SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT
run lds SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAIT_ANY SQ_INSTS_SALU
run tcc TCC_HIT_sum TCC_MISS_sum
echo done
