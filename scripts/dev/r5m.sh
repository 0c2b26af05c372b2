#!/bin/bash
# Round 5: stream groups beyond 4 with more hardware queues (GPU_MAX_HW_QUEUES), one box;
# multi-rank rehearsal (gloo ranks sharing the GPU) with the stream groups.
set -e
OUT=gpurun_out/r5m; mkdir -p $OUT
T="timeout -k 10"
for rep in 1 2; do
  MOPT_STREAMS=3 $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_s3_q4_$rep.json 2> $OUT/bench_s3_q4_$rep.err
  for q in 8; do
    for s in 3 4 6 8; do
      GPU_MAX_HW_QUEUES=$q MOPT_STREAMS=$s $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_s${s}_q${q}_$rep.json 2> $OUT/bench_s${s}_q${q}_$rep.err
    done
  done
  echo rep $rep
done
$T 400 python bench.py --gpus 2 --steps 10 --warmup 3 --population 64 > $OUT/rehearsal_n2.json 2> $OUT/rehearsal_n2.err
echo done
