#!/bin/bash
# Round 5: residual-BN relu' bit mask, BatchNorm unroll 4 (this tree) / 8 (variant u8) vs ab_base
# (no mask, unroll 4) -- ResNet GPU tests on both libraries, 3 interleaved ResNet-20 repetitions.
set -e
OUT=gpurun_out/r6r; mkdir -p $OUT
T="timeout -k 10"
U8=$GRAFT_REPO_ROOT/metaopt_amd/ops/lib/variants/u8/libmopt_kernels.so
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_resnet_gpu.py > $OUT/pytest.log 2>&1
MOPT_KERNEL_LIB=$U8 $T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_resnet_gpu.py > $OUT/pytest_u8.log 2>&1
echo tests ok
for rep in 1 2 3; do
  $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet_new_$rep.json 2> $OUT/resnet_new_$rep.err
  MOPT_KERNEL_LIB=$U8 $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet_u8_$rep.json 2> $OUT/resnet_u8_$rep.err
  (cd ab_base && $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > ../$OUT/resnet_base_$rep.json 2> ../$OUT/resnet_base_$rep.err)
  echo rep $rep
done
echo done
