#!/bin/bash
# Round 5: search quality at 12 / 24 / 48 intervals on the final kernels, 3 seeds x (async ASHA
# default grace 4 intervals eta 4, async ASHA eta 2 from 2 intervals, random search); gloo rank
# rehearsals sharing the GPU; a 10-generation PBT run of config 5.
set -e
OUT=gpurun_out/r6b; mkdir -p $OUT
T="timeout -k 10"
for seed in 0 1 2; do
  for v in "async:--asha-mode async" "async_eta2:--asha-mode async --fidelity 2,16,2" "random:--algo random"; do
    $T 300 python bench.py --steps 43 --warmup 5 --seed $seed ${v#*:} > "$OUT/algo_${v%%:*}_s$seed.json" 2> "$OUT/algo_${v%%:*}_s$seed.err"
  done
  echo seed $seed
done
for n in 2 4; do
  $T 400 python bench.py --gpus $n --steps 10 --warmup 3 --population 64 > $OUT/rehearsal_n$n.json 2> $OUT/rehearsal_n$n.err
done
echo rehearsal ok
$T 600 python scripts/bench_configs.py --config lm-125m --steps 2000 --warmup 0 > $OUT/lm125m_pbt2000.json 2> $OUT/lm125m_pbt2000.err
echo done
