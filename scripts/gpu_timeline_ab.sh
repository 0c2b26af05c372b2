#!/bin/bash
# Same box: kernel_bench (per-kernel) and the headline bench with GPU-event timelines,
# fp32 vs bf16 momentum.
set -e
OUT=${OUT:-gpurun_out/timeline_ab}
mkdir -p "$OUT"
for m in fp32 bf16; do
  timeout -k 10 120 python scripts/kernel_bench.py --momentum-dtype $m > "$OUT/k_$m.log" 2>&1
  MOPT_GPU_TIMELINE=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --momentum-dtype $m > "$OUT/b_$m.json" 2> "$OUT/b_$m.err"
done
echo done
