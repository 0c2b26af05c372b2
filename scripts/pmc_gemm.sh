#!/bin/bash
# PMC counters of the population GEMM kernel on the LM / ResNet shapes (one counter group per pass)
set -e
OUT=${OUT:-gpurun_out/pmc_gemm}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
pmc() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --output-format csv --pmc "$@" -d "$ROOT/$OUT/$name" -o run -- \
      python3 "$ROOT/scripts/gemm_bench.py" --no-torch --iters 2 > "$ROOT/$OUT/$name.log" 2>&1
}
pmc mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES
pmc lds SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU
pmc fetch FETCH_SIZE
echo done
