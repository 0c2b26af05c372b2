#!/bin/bash
# Round 5: residual BatchNorm backward reads a thread-mapped relu bit mask instead of y -- ResNet GPU tests,
# 3 interleaved ResNet-20 repetitions against ab_base, then the LM-125M kernel-trace profile.
set -e
OUT=gpurun_out/r6q; mkdir -p $OUT
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_resnet_gpu.py > $OUT/pytest.log 2>&1
echo tests ok
for rep in 1 2 3; do
  $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet_new_$rep.json 2> $OUT/resnet_new_$rep.err
  (cd ab_base && $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > ../$OUT/resnet_base_$rep.json 2> ../$OUT/resnet_base_$rep.err)
  echo rep $rep
done
(cd /tmp && export TMPDIR=/tmp && $T 400 rocprofv3 --kernel-trace --stats --output-format csv \
   -d $GRAFT_REPO_ROOT/$OUT/lm -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py --config lm-125m --sync-every 10 --steps 20 --warmup 10 > $GRAFT_REPO_ROOT/$OUT/lm.log 2>&1)
echo done
