#!/bin/bash
# Rank-0 decision cost at 1/8 simulated ranks on the GPU box's CPU (no GPU use).
set -e
OUT=${OUT:-gpurun_out/decide}
mkdir -p "$OUT"
for w in 1 8; do
  WORLD=$w timeout -k 10 300 python scripts/profile_decide.py > "$OUT/world$w.log" 2>&1
done
echo done
