#!/bin/bash
# K11: GPU numerics of the batched-tangent inner step and config-4 throughput.
set -e
OUT=${OUT:-gpurun_out/k11b}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_pgemm_ad.py tests/test_lm_gpu.py tests/test_hyper.py -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/pytest.log" 2>&1
timeout -k 10 300 python scripts/bench_configs.py --config hyper --steps 3 --warmup 1 > "$OUT/hyper.json" 2> "$OUT/hyper.err"
echo done
