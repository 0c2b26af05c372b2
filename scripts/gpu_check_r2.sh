#!/bin/bash
# GPU test suite, per-kernel bench (bf16 / fp32 momentum) and the headline bench (N=1) with the
# GPU-event timeline.
set -e
OUT=${OUT:-gpurun_out/check_r2}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
for m in bf16 fp32; do
  timeout -k 10 120 python scripts/kernel_bench.py --momentum-dtype $m --out "$OUT/k_$m.json" > "$OUT/k_$m.log" 2>&1
done
MOPT_GPU_TIMELINE=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
echo done
