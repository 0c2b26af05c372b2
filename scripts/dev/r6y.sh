#!/bin/bash
# Round 5 final tree: headline at 43 timed intervals (best loss at 12 / 24 / 48), seeds 0 / 1 / 2,
# and config 5 over ten PBT generations (2000 steps).
set -e
OUT=gpurun_out/r6y; mkdir -p $OUT
T="timeout -k 10"
for seed in 0 1 2; do
  $T 300 python bench.py --steps 43 --warmup 5 --seed $seed > $OUT/bench48_s$seed.json 2> $OUT/bench48_s$seed.err
  echo seed $seed
done
$T 600 python scripts/bench_configs.py --config lm-125m --steps 2000 --warmup 0 > $OUT/lm125m_pbt2000.json 2> $OUT/lm125m_pbt2000.err
echo done
