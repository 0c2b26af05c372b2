#!/bin/bash
# Round 5: weight-gradient workgroup count (1024 / 2048 default / 4096) on ResNet-20,
# 3 interleaved repetitions, plus a kernel-trace profile of each.
set -e
OUT=gpurun_out/r6k; mkdir -p $OUT
T="timeout -k 10"
V=$GRAFT_REPO_ROOT/metaopt_amd/ops/lib/variants
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_resnet_gpu.py > $OUT/pytest.log 2>&1
echo tests ok
for rep in 1 2 3; do
  for v in wg1024 base wg4096; do
    if [ $v = base ]; then L=""; else L=$V/$v/libmopt_kernels.so; fi
    MOPT_KERNEL_LIB=$L $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet_${v}_$rep.json 2> $OUT/resnet_${v}_$rep.err
  done
  echo rep $rep
done
echo done
