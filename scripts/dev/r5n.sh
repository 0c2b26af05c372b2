#!/bin/bash
# Round 5: 4-stage 32-deep ring GEMM at 256 x 256 (cfg 12): correctness, shapes A/B, LM step A/B.
set -e
OUT=gpurun_out/r5n; mkdir -p $OUT
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pgemm_gpu.py > $OUT/pytest_gemm.log 2>&1
echo gemm tests ok
$T 300 python scripts/gemm_bench.py --no-torch --shapes lm --cfgs 5,11,12 --splits 12:2 --out $OUT/gemm.json > $OUT/gemm.log 2>&1
echo gemm bench ok
for r in 0 1; do
  MOPT_GEMM_RING4=$r $T 300 python scripts/bench_configs.py --config lm-125m --steps 400 --warmup 0 > $OUT/lm_ring4_$r.json 2> $OUT/lm_ring4_$r.err
done
echo done
