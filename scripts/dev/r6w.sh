#!/bin/bash
# Round 5: stream groups 2 / 3 / 4 with round-robin queueing (chunk 4), and chunk 2 at 3 groups
# -- headline bench, 3 interleaved repetitions.
set -e
OUT=gpurun_out/r6w; mkdir -p $OUT
T="timeout -k 10"
for rep in 1 2 3; do
  for v in s3 s2 s4 s3c2; do
    case $v in
      s3) E="MOPT_STREAMS=3";; s2) E="MOPT_STREAMS=2";; s4) E="MOPT_STREAMS=4";;
      s3c2) E="MOPT_STREAMS=3 MOPT_STEP_CHUNK=2";;
    esac
    env $E $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_${v}_$rep.json 2> $OUT/bench_${v}_$rep.err
  done
  echo rep $rep
done
echo done
