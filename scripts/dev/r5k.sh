#!/bin/bash
# Round 5: ResNet-20 weight-gradient offsets split into scalar + lane parts (round-4 patch): A/B.
set -e
OUT=gpurun_out/r5k; mkdir -p $OUT
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_resnet_gpu.py tests/test_conv_gpu.py > $OUT/pytest_resnet.log 2>&1 || $T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_resnet_gpu.py > $OUT/pytest_resnet.log 2>&1
echo tests ok
for rep in 1 2; do
  $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet_$rep.json 2> $OUT/resnet_$rep.err
  (cd ab_base && $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30) > $OUT/resnet_base_$rep.json 2> $OUT/resnet_base_$rep.err
done
echo done
