#!/bin/bash
# GPU measurement recipe (run on the box through gpurun from the repo root):
#   bench.py, per-kernel microbench, rocprofv3 kernel trace of the bench, PMC counters of the
#   kernels (own runs; counters never combined with trace domains).
set -e
OUT=${OUT:-gpurun_out/prof}
mkdir -p "$OUT"
ROOT=$(pwd)
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 python scripts/kernel_bench.py --out "$OUT/kbench.json" > "$OUT/kbench.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 64 --warmup 32 > "$ROOT/$OUT/trace.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE \
    -d "$ROOT/$OUT/pmc1" -o run -- python3 "$ROOT/scripts/kernel_bench.py" --iters 3 \
    > "$ROOT/$OUT/pmc1.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES \
    -d "$ROOT/$OUT/pmc2" -o run -- python3 "$ROOT/scripts/kernel_bench.py" --iters 3 \
    > "$ROOT/$OUT/pmc2.log" 2>&1
echo done
