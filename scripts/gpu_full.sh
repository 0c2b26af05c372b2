#!/bin/bash
# Full round-end rehearsal: every GPU test, smoke(), the driver's bench command, configs 3-5.
set -e
OUT=${OUT:-gpurun_out/full}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
OUT=$OUT bash scripts/gpu_configs.sh > /dev/null
echo done
