set -e
OUT=gpurun_out/r4w
mkdir -p $OUT
V=metaopt_amd/ops/lib/variants
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py > $OUT/pytest_kernels.log 2>&1
for rep in 1 2; do
  timeout -k 10 200 python scripts/kernel_bench.py --momentum-dtype bf16 > $OUT/kbench_ts80_$rep.log 2>&1
  MOPT_KERNEL_LIB=$V/fts72/libmopt_kernels.so timeout -k 10 200 python scripts/kernel_bench.py --momentum-dtype bf16 > $OUT/kbench_ts72_$rep.log 2>&1
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
echo done
