#!/bin/bash
# Round 5: batch-norm reduce/apply block counts (1024 / 2048 default / 4096 / 8192) on ResNet-20,
# 3 interleaved repetitions; ResNet/conv GPU tests of the 1024-workgroup weight gradient first.
set -e
OUT=gpurun_out/r6m; mkdir -p $OUT
T="timeout -k 10"
V=$GRAFT_REPO_ROOT/metaopt_amd/ops/lib/variants
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_resnet_gpu.py > $OUT/pytest.log 2>&1
echo tests ok
for rep in 1 2 3; do
  for v in bn1024 base bn4096 bn8192; do
    if [ $v = base ]; then L=""; else L=$V/$v/libmopt_kernels.so; fi
    MOPT_KERNEL_LIB=$L $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet_${v}_$rep.json 2> $OUT/resnet_${v}_$rep.err
  done
  echo rep $rep
done
echo done
