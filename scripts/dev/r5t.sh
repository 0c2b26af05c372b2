#!/bin/bash
# Round 5: fused first layer, strips in pairs with alternating register sets -- equality, A/B
# against the copy-based prefetch (ab_base = previous commit), in-situ time.
set -e
OUT=gpurun_out/r5t; mkdir -p $OUT
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py > $OUT/pytest.log 2>&1
echo tests ok
for rep in 1 2; do
  $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_new_$rep.json 2> $OUT/bench_new_$rep.err
  (cd ab_base && $T 240 python bench.py --steps 20 --warmup 5 > ../$OUT/bench_base_$rep.json 2> ../$OUT/bench_base_$rep.err)
  echo rep $rep
done
(cd /tmp && export TMPDIR=/tmp && MOPT_STREAMS=1 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_s1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 > $GRAFT_REPO_ROOT/$OUT/trace_s1.log 2>&1)
echo done
