#!/bin/bash
# Round 5 final tree: 3 vs 4 stream groups (round-robin queueing), headline bench, 5 interleaved
# repetitions.
set -e
OUT=gpurun_out/r7b; mkdir -p $OUT
T="timeout -k 10"
for rep in 1 2 3 4 5; do
  for s in 3 4; do
    MOPT_STREAMS=$s $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_s${s}_$rep.json 2> $OUT/bench_s${s}_$rep.err
  done
  echo rep $rep
done
echo done
