#!/bin/bash
# Round 5: fused first layer, 16-byte state layout -- equality, in-situ times (DIAG 0/1, 1 and 3
# streams), headline A/B.
set -e
OUT=gpurun_out/r5s; mkdir -p $OUT
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py > $OUT/pytest.log 2>&1
echo tests ok
for d in 0 1; do
  (cd /tmp && export TMPDIR=/tmp && MOPT_STREAMS=1 MOPT_B0F_DIAG=$d $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_s1_d$d -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 > $GRAFT_REPO_ROOT/$OUT/trace_s1_d$d.log 2>&1)
done
for rep in 1 2; do
  MOPT_FUSE0=0 $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_f0_$rep.json 2> $OUT/bench_f0_$rep.err
  MOPT_FUSE0=1 $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_f1_$rep.json 2> $OUT/bench_f1_$rep.err
  echo rep $rep
done
echo done
