#!/bin/bash
# Round 5 final tree: attention occupancy targets re-swept after the dK/dV changes (MOPT_ATTN_WAVES
# "fwd, dq, dkdv" variant builds), 2 interleaved repetitions of scripts/attn_bench.py.
set -e
OUT=gpurun_out/r7a; mkdir -p $OUT
T="timeout -k 10"
V=$GRAFT_REPO_ROOT/metaopt_amd/ops/lib/variants
for rep in 1 2; do
  for v in aw443 aw442 aw433 aw444 aw453; do
    MOPT_KERNEL_LIB=$V/$v/libmopt_kernels.so $T 120 python scripts/attn_bench.py --iters 40 > $OUT/attn_${v}_$rep.json 2> $OUT/attn_${v}_$rep.err
  done
  echo rep $rep
done
echo done
