#!/bin/bash
# Round 5: SLP vectorisation off -- (a) the attention file only (default build of this tree),
# (b) every kernel file (variant noslp), against (c) the previous commit (ab_base, SLP on).
set -e
OUT=gpurun_out/r6h; mkdir -p $OUT
T="timeout -k 10"
NOSLP=$GRAFT_REPO_ROOT/metaopt_amd/ops/lib/variants/noslp/libmopt_kernels.so
$T 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lm_gpu.py tests/test_kernels_gpu.py tests/test_resnet_gpu.py > $OUT/pytest.log 2>&1
echo tests ok
run() {  # run TAG CMD...: in this tree (new), with the noslp library, in ab_base (base)
  local tag=$1; shift
  "$@" > $OUT/${tag}_new.json 2> $OUT/${tag}_new.err
  MOPT_KERNEL_LIB=$NOSLP "$@" > $OUT/${tag}_noslp.json 2> $OUT/${tag}_noslp.err
  (cd ab_base && "$@" > ../$OUT/${tag}_base.json 2> ../$OUT/${tag}_base.err)
}
for rep in 1 2; do
  run attn$rep $T 120 python scripts/attn_bench.py
  run bench$rep $T 240 python bench.py --steps 20 --warmup 5
done
run lm $T 300 python scripts/bench_configs.py --config lm-125m --steps 200 --warmup 0
run resnet $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30
echo done
