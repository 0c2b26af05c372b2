set -e
OUT=gpurun_out/r4ac
mkdir -p $OUT
for seed in 1 2 3 4; do
  for v in "random:--algo random" "async:--asha-mode async"; do
    timeout -k 10 240 python bench.py --steps 43 --warmup 5 --seed $seed ${v#*:} > "$OUT/algo_${v%%:*}_s$seed.json" 2> "$OUT/algo_${v%%:*}_s$seed.err"
    echo "seed $seed ${v%%:*} done"
  done
done
echo done
WORLD=8 PRIORS=headline N_SYNCS=60 timeout -k 10 300 python scripts/profile_decide.py > gpurun_out/r4ac/decide_world8_headline.log 2>&1
WORLD=8 timeout -k 10 300 python scripts/profile_decide.py > gpurun_out/r4ac/decide_world8_stress.log 2>&1
echo done2
