#!/bin/bash
# GPU check recipe: kernel numerics tests, headline bench, per-kernel microbench.
set -e
OUT=${OUT:-gpurun_out/check}
mkdir -p "$OUT"
timeout -k 10 600 python -m pytest tests -m gpu -x -q > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 300 python bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 python scripts/kernel_bench.py --out "$OUT/kbench.json" > "$OUT/kbench.log" 2>&1
cat "$OUT/bench.json"
tail -3 "$OUT/pytest_gpu.log"
cat "$OUT/kbench.log"
