#!/bin/bash
# Round 5: attention forward with two 64-query blocks per workgroup sharing the K / V tiles (this
# tree, MOPT_ATTN_FWD_QB=2) vs one (variant qb1) -- LM GPU tests, 3 interleaved attention / LM-125M
# repetitions.
set -e
OUT=gpurun_out/r6t; mkdir -p $OUT
T="timeout -k 10"
QB1=$GRAFT_REPO_ROOT/metaopt_amd/ops/lib/variants/qb1/libmopt_kernels.so
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lm_gpu.py > $OUT/pytest.log 2>&1
echo tests ok
for rep in 1 2 3; do
  $T 120 python scripts/attn_bench.py --iters 40 > $OUT/attn_qb2_$rep.json 2> $OUT/attn_qb2_$rep.err
  MOPT_KERNEL_LIB=$QB1 $T 120 python scripts/attn_bench.py --iters 40 > $OUT/attn_qb1_$rep.json 2> $OUT/attn_qb1_$rep.err
  $T 300 python scripts/bench_configs.py --config lm-125m --steps 200 --warmup 0 > $OUT/lm_qb2_$rep.json 2> $OUT/lm_qb2_$rep.err
  MOPT_KERNEL_LIB=$QB1 $T 300 python scripts/bench_configs.py --config lm-125m --steps 200 --warmup 0 > $OUT/lm_qb1_$rep.json 2> $OUT/lm_qb1_$rep.err
  echo rep $rep
done
echo done
