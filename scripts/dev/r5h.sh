#!/bin/bash
# Round 5: stream-group count sweep of the headline bench (two repetitions each), one box.
set -e
OUT=gpurun_out/r5h; mkdir -p $OUT
T="timeout -k 10"
for rep in 1 2; do
  for s in 1 3 4 6 8; do
    MOPT_STREAMS=$s $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_s${s}_$rep.json 2> $OUT/bench_s${s}_$rep.err
  done
  MOPT_STREAMS=4 MOPT_FWD_TN=128 $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_s4_tn128_$rep.json 2> $OUT/bench_s4_tn128_$rep.err
  echo rep $rep
done
echo done
