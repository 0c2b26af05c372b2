#!/bin/bash
# Round 5: pipelined halo staging of the direct convolutions (next band's halo / dy tile loaded
# into registers during the current band's MFMAs, output tile copy-out one band behind):
# correctness, conv microbench and ResNet-20 step A/B against the previous commit (ab_base/).
set -e
OUT=gpurun_out/r5o; mkdir -p $OUT
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_resnet_gpu.py > $OUT/pytest_resnet.log 2>&1
echo resnet tests ok
$T 200 python scripts/conv_bench.py --out $OUT/conv_new.json > $OUT/conv_new.log 2>&1
(cd ab_base && $T 200 python scripts/conv_bench.py --out ../$OUT/conv_base.json > ../$OUT/conv_base.log 2>&1)
echo conv bench ok
for rep in 1 2; do
  $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet_new_$rep.json 2> $OUT/resnet_new_$rep.err
  (cd ab_base && $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > ../$OUT/resnet_base_$rep.json 2> ../$OUT/resnet_base_$rep.err)
  echo rep $rep
done
(cd /tmp && export TMPDIR=/tmp && $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py --config resnet20 --sync-every 10 --steps 20 --warmup 10 > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1)
echo done
