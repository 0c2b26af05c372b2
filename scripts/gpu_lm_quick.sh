#!/bin/bash
# LM + ResNet GPU tests and the 125M-LM / ResNet-20 step times.
set -e
OUT=${OUT:-gpurun_out/lmq}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_lm_gpu.py tests/test_resnet_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
timeout -k 10 300 python scripts/bench_configs.py --config lm-125m --steps 20 --warmup 10 > "$OUT/lm.json" 2> "$OUT/lm.err"
timeout -k 10 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > "$OUT/resnet.json" 2> "$OUT/resnet.err"
echo done
