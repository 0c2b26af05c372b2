#!/bin/bash
# Round 5: BatchNorm finalize folded into the apply pass (each block derives its channels'
# statistics from the sums; block (0, p) writes stat and the running update) -- ResNet GPU tests,
# 3 interleaved ResNet-20 repetitions against ab_base.
set -e
OUT=gpurun_out/r7c; mkdir -p $OUT
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_resnet_gpu.py tests/test_checked_build_gpu.py > $OUT/pytest.log 2>&1
echo tests ok
for rep in 1 2 3; do
  $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet_new_$rep.json 2> $OUT/resnet_new_$rep.err
  (cd ab_base && $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > ../$OUT/resnet_base_$rep.json 2> ../$OUT/resnet_base_$rep.err)
  echo rep $rep
done
echo done
