set -e
OUT=gpurun_out/r4ah
mkdir -p $OUT
V=metaopt_amd/ops/lib/variants
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lm_gpu.py > $OUT/pytest_lm.log 2>&1
for rep in 1 2 3; do
  timeout -k 10 120 python scripts/attn_bench.py >> $OUT/attn_sb1.log 2>&1
  MOPT_KERNEL_LIB=$V/attnsb0/libmopt_kernels.so timeout -k 10 120 python scripts/attn_bench.py >> $OUT/attn_sb0.log 2>&1
done
for rep in 1 2; do
  timeout -k 10 300 python scripts/bench_configs.py --config lm-125m --steps 20 --warmup 10 > $OUT/lm_sb1_$rep.json 2> $OUT/lm_sb1.err
  MOPT_KERNEL_LIB=$V/attnsb0/libmopt_kernels.so timeout -k 10 300 python scripts/bench_configs.py --config lm-125m --steps 20 --warmup 10 > $OUT/lm_sb0_$rep.json 2> $OUT/lm_sb0.err
done
echo done
