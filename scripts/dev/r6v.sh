#!/bin/bash
# Round 5: round-robin step queueing, MOPT_STEP_CHUNK 0 (previous) vs 4 (default) -- headline
# bench, 5 interleaved repetitions.
set -e
OUT=gpurun_out/r6v; mkdir -p $OUT
T="timeout -k 10"
for rep in 1 2 3 4 5; do
  for c in 0 4; do
    MOPT_STEP_CHUNK=$c $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_c${c}_$rep.json 2> $OUT/bench_c${c}_$rep.err
  done
  echo rep $rep
done
echo done
