#!/bin/bash
# Round 5: fused first layer (bwd0 of step t + fwd0 of step t+1) -- equality tests, headline A/B
# (MOPT_FUSE0 0/1, 2- vs 3-wave variant); conv 64-channel prefetch fix -- ResNet A/B.
set -e
OUT=gpurun_out/r5p; mkdir -p $OUT
T="timeout -k 10"
$T 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_resnet_gpu.py > $OUT/pytest.log 2>&1
echo tests ok
for rep in 1 2; do
  MOPT_FUSE0=0 $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_f0_$rep.json 2> $OUT/bench_f0_$rep.err
  MOPT_FUSE0=1 $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_f1_$rep.json 2> $OUT/bench_f1_$rep.err
  MOPT_FUSE0=1 MOPT_B0F_WAVES=2 $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_f1w2_$rep.json 2> $OUT/bench_f1w2_$rep.err
  $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet_$rep.json 2> $OUT/resnet_$rep.err
  echo rep $rep
done
(cd /tmp && export TMPDIR=/tmp && $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1)
echo done
