#!/bin/bash
# Re-entry check: GPU tests, headline bench (driver command), configs 3-5 throughput.
set -e
OUT=${OUT:-gpurun_out/r2c}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
OUT=$OUT bash scripts/gpu_configs.sh > /dev/null
echo done
