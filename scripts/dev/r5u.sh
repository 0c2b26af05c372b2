#!/bin/bash
# Round 5: stream-group sweep with the fused first layer; PMC passes of the MLP kernels.
set -e
OUT=gpurun_out/r5u; mkdir -p $OUT
T="timeout -k 10"
for rep in 1 2; do
  for s in 2 3 4 5; do
    MOPT_STREAMS=$s $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_s${s}_$rep.json 2> $OUT/bench_s${s}_$rep.err
  done
  echo rep $rep
done
OUT=$OUT/pmc bash scripts/gpu.sh pmc_kbench
echo done
