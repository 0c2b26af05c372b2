#!/bin/bash
# Round 5 north-star algorithm evidence on the final kernels: config 5 (PBT vs random search over
# the same 8 slots and 2000 steps, 2 seeds each) and config 3 (TPE vs random over ResNet-20,
# 3120 steps = 2 TPE generations of 96 trials, 3 seeds each).
set -e
OUT=gpurun_out/r6f; mkdir -p $OUT
T="timeout -k 10"
for seed in 1 2; do
  $T 600 python scripts/bench_configs.py --config lm-125m --steps 2000 --warmup 0 --seed $seed > $OUT/lm_pbt_s$seed.json 2> $OUT/lm_pbt_s$seed.err
  $T 600 python scripts/bench_configs.py --config lm-125m --steps 2000 --warmup 0 --seed $seed --algo random > $OUT/lm_random_s$seed.json 2> $OUT/lm_random_s$seed.err
  echo lm seed $seed
done
for seed in 0 1 2; do
  $T 400 python scripts/bench_configs.py --config resnet20 --steps 3120 --warmup 0 --seed $seed > $OUT/resnet_tpe_s$seed.json 2> $OUT/resnet_tpe_s$seed.err
  $T 400 python scripts/bench_configs.py --config resnet20 --steps 3120 --warmup 0 --seed $seed --algo random > $OUT/resnet_random_s$seed.json 2> $OUT/resnet_random_s$seed.err
  echo resnet seed $seed
done
echo done
