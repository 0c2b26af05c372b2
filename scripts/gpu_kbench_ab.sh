#!/bin/bash
# Per-kernel A/B: momentum dtype and stream groups (scripts/kernel_bench.py) + kernel trace.
set -e
OUT=${OUT:-gpurun_out/kbench_ab}
mkdir -p "$OUT"
for cfg in "fp32 1" "bf16 1" "fp32 2" "bf16 2"; do
  set -- $cfg
  timeout -k 10 120 python scripts/kernel_bench.py --momentum-dtype $1 --streams $2 --out "$OUT/k_$1_s$2.json" > "$OUT/k_$1_s$2.log" 2>&1
done
echo done
