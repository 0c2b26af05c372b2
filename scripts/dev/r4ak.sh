set -e
OUT=gpurun_out/r4ak
mkdir -p $OUT
for seed in 0 1 2; do
  timeout -k 10 300 python scripts/bench_configs.py --config resnet20 --steps 1560 --warmup 0 --seed $seed > $OUT/resnet_tpe_s$seed.json 2> $OUT/resnet_tpe_s$seed.err
  timeout -k 10 300 python scripts/bench_configs.py --config resnet20 --steps 1560 --warmup 0 --seed $seed --algo random > $OUT/resnet_random_s$seed.json 2> $OUT/resnet_random_s$seed.err
  echo "seed $seed done"
done
echo done
