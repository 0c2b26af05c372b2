#!/bin/bash
# Round 5: big GEMM with the next stage's LDS-DMA pieces interleaved with the first half-step's
# MFMAs -- correctness, LM shapes, LM-125M A/B against the previous commit (ab_base).
set -e
OUT=gpurun_out/r5z; mkdir -p $OUT
T="timeout -k 10"
$T 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pgemm_gpu.py tests/test_lm_gpu.py > $OUT/pytest.log 2>&1
echo tests ok
$T 300 python scripts/gemm_bench.py --no-torch --shapes lm --cfgs 5,6,7,11 --out $OUT/gemm_new.json > $OUT/gemm_new.log 2>&1
(cd ab_base && $T 300 python scripts/gemm_bench.py --no-torch --shapes lm --cfgs 5,6,7,11 --out ../$OUT/gemm_base.json > ../$OUT/gemm_base.log 2>&1)
echo gemm ok
for rep in 1 2; do
  $T 300 python scripts/bench_configs.py --config lm-125m --steps 200 --warmup 0 > $OUT/lm_new_$rep.json 2> $OUT/lm_new_$rep.err
  (cd ab_base && $T 300 python scripts/bench_configs.py --config lm-125m --steps 200 --warmup 0 > ../$OUT/lm_base_$rep.json 2> ../$OUT/lm_base_$rep.err)
done
echo done
