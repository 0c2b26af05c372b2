#!/bin/bash
# Round 5: fused first layer diagnostics -- in-situ kernel times with the forward part removed
# (DIAG 1), without the state prefetch (DIAG 2), and the full kernel.
set -e
OUT=gpurun_out/r5r; mkdir -p $OUT
T="timeout -k 10"
for d in 0 1 2; do
  (cd /tmp && export TMPDIR=/tmp && MOPT_B0F_DIAG=$d $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof$d -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 > $GRAFT_REPO_ROOT/$OUT/trace$d.log 2>&1)
  echo diag $d
done
(cd /tmp && export TMPDIR=/tmp && MOPT_STREAMS=1 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_s1 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 > $GRAFT_REPO_ROOT/$OUT/trace_s1.log 2>&1)
(cd /tmp && export TMPDIR=/tmp && MOPT_STREAMS=1 MOPT_FUSE0=0 $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_s1f0 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 6 --warmup 2 > $GRAFT_REPO_ROOT/$OUT/trace_s1f0.log 2>&1)
echo done
