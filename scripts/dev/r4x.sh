set -e
OUT=gpurun_out/r4x
mkdir -p $OUT
V=metaopt_amd/ops/lib/variants
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py > $OUT/pytest_kernels.log 2>&1
for rep in 1 2; do
  timeout -k 10 200 python scripts/kernel_bench.py --momentum-dtype bf16 > $OUT/kbench_p1w3_$rep.log 2>&1
  for n in p0w4 p1w4; do
    MOPT_KERNEL_LIB=$V/$n/libmopt_kernels.so timeout -k 10 200 python scripts/kernel_bench.py --momentum-dtype bf16 > $OUT/kbench_${n}_$rep.log 2>&1
  done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
MOPT_KERNEL_LIB=$V/p0w4/libmopt_kernels.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_p0w4.json 2> $OUT/bench_p0w4.err
echo done
