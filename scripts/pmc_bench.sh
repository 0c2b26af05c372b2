#!/bin/bash
# PMC counters of the headline bench's kernels (one counter group per pass, short run)
set -e
OUT=${OUT:-gpurun_out/pmc_bench}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pmc() {
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --output-format csv --pmc "$@" -d "$ROOT/$OUT/$name" -o run -- \
      python3 "$ROOT/bench.py" --steps 32 --warmup 16 > "$ROOT/$OUT/$name.log" 2>&1
}
pmc wait SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES
pmc fetch FETCH_SIZE TCC_HIT_sum
echo done
