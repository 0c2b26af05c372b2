#!/bin/bash
# Round 5: the stream groups' steps queued round-robin in runs of MOPT_STEP_CHUNK steps (default
# 4; 0 = each group's whole interval in turn, the previous behaviour) -- kernel GPU tests, then
# the headline bench at chunk 0 / 1 / 2 / 4 / 8, 2 interleaved repetitions, then a kernel trace
# of the default for the stream-overlap timeline.
set -e
OUT=gpurun_out/r6u; mkdir -p $OUT
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py > $OUT/pytest.log 2>&1
echo tests ok
for rep in 1 2; do
  for c in 0 4 1 8 2; do
    MOPT_STEP_CHUNK=$c $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_c${c}_$rep.json 2> $OUT/bench_c${c}_$rep.err
  done
  echo rep $rep
done
for c in 0 4; do
  (cd /tmp && export TMPDIR=/tmp && MOPT_STEP_CHUNK=$c $T 300 rocprofv3 --kernel-trace --output-format csv \
     -d $GRAFT_REPO_ROOT/$OUT/trace_c$c -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 3 > $GRAFT_REPO_ROOT/$OUT/trace_c$c.log 2>&1)
done
echo done
