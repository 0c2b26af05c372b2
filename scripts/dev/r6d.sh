#!/bin/bash
# Round 5: stride-2 data gradients on 128-pixel bands (CI >= 32) -- ResNet tests, conv bench and
# ResNet-20 A/B against the previous commit (ab_base).
set -e
OUT=gpurun_out/r6d; mkdir -p $OUT
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_resnet_gpu.py > $OUT/pytest_resnet.log 2>&1
echo tests ok
$T 200 python scripts/conv_bench.py --out $OUT/conv_new.json > $OUT/conv_new.log 2>&1
(cd ab_base && $T 200 python scripts/conv_bench.py --out ../$OUT/conv_base.json > ../$OUT/conv_base.log 2>&1)
for rep in 1 2; do
  $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet_new_$rep.json 2> $OUT/resnet_new_$rep.err
  (cd ab_base && $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > ../$OUT/resnet_base_$rep.json 2> ../$OUT/resnet_base_$rep.err)
done
echo done
