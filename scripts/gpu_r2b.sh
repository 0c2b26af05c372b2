#!/bin/bash
# Round-2 re-entry check: GPU test suite, headline bench (N=1) and rank-0 decision cost at 1 and
# 8 simulated ranks on the box CPU.
set -e
OUT=${OUT:-gpurun_out/r2b}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
MOPT_GPU_TIMELINE=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
WORLD=1 timeout -k 10 200 python scripts/profile_decide.py > "$OUT/decide_w1.log" 2>&1
WORLD=8 timeout -k 10 200 python scripts/profile_decide.py > "$OUT/decide_w8.log" 2>&1
echo done
