#!/bin/bash
# Round 5: attention forward row max on raw scores (scale folded into the exponent fma) --
# LM tests, 3 interleaved attention / LM-125M repetitions against ab_base.
set -e
OUT=gpurun_out/r6j; mkdir -p $OUT
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lm_gpu.py > $OUT/pytest.log 2>&1
echo tests ok
for rep in 1 2 3; do
  $T 120 python scripts/attn_bench.py --iters 40 > $OUT/attn_new_$rep.json 2> $OUT/attn_new_$rep.err
  (cd ab_base && $T 120 python scripts/attn_bench.py --iters 40 > ../$OUT/attn_base_$rep.json 2> ../$OUT/attn_base_$rep.err)
  $T 300 python scripts/bench_configs.py --config lm-125m --steps 200 --warmup 0 > $OUT/lm_new_$rep.json 2> $OUT/lm_new_$rep.err
  (cd ab_base && $T 300 python scripts/bench_configs.py --config lm-125m --steps 200 --warmup 0 > ../$OUT/lm_base_$rep.json 2> ../$OUT/lm_base_$rep.err)
  echo rep $rep
done
echo done
