#!/bin/bash
# Round 5: pack2bf as one two-source v_cvt_pk_bf16_f32 -- GPU suite, then A/B against the
# previous commit (ab_base) on the headline, LM-125M, ResNet-20 and the attention bench.
set -e
OUT=gpurun_out/r6g; mkdir -p $OUT
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1
echo tests ok
for rep in 1 2; do
  $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_new_$rep.json 2> $OUT/bench_new_$rep.err
  (cd ab_base && $T 240 python bench.py --steps 20 --warmup 5 > ../$OUT/bench_base_$rep.json 2> ../$OUT/bench_base_$rep.err)
  $T 120 python scripts/attn_bench.py --out $OUT/attn_new_$rep.json > $OUT/attn_new_$rep.log 2>&1
  (cd ab_base && $T 120 python scripts/attn_bench.py --out ../$OUT/attn_base_$rep.json > ../$OUT/attn_base_$rep.log 2>&1)
done
$T 300 python scripts/bench_configs.py --config lm-125m --steps 200 --warmup 0 > $OUT/lm_new.json 2> $OUT/lm_new.err
(cd ab_base && $T 300 python scripts/bench_configs.py --config lm-125m --steps 200 --warmup 0 > ../$OUT/lm_base.json 2> ../$OUT/lm_base.err)
$T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet_new.json 2> $OUT/resnet_new.err
(cd ab_base && $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > ../$OUT/resnet_base.json 2> ../$OUT/resnet_base.err)
echo done
