#!/bin/bash
# Round 5: SLP A/B repeated (the first box was noisy: +-15 % between identical kernels) --
# 3 interleaved repetitions of attention, LM-125M, headline; new / noslp / base.
set -e
OUT=gpurun_out/r6i; mkdir -p $OUT
T="timeout -k 10"
NOSLP=$GRAFT_REPO_ROOT/metaopt_amd/ops/lib/variants/noslp/libmopt_kernels.so
run() {
  local tag=$1; shift
  "$@" > $OUT/${tag}_new.json 2> $OUT/${tag}_new.err
  MOPT_KERNEL_LIB=$NOSLP "$@" > $OUT/${tag}_noslp.json 2> $OUT/${tag}_noslp.err
  (cd ab_base && "$@" > ../$OUT/${tag}_base.json 2> ../$OUT/${tag}_base.err)
}
for rep in 1 2 3; do
  run attn$rep $T 120 python scripts/attn_bench.py --iters 40
  run lm$rep $T 300 python scripts/bench_configs.py --config lm-125m --steps 200 --warmup 0
  run bench$rep $T 240 python bench.py --steps 20 --warmup 5
  echo rep $rep
done
echo done
