set -e
OUT=gpurun_out/r4ag
mkdir -p $OUT
V=metaopt_amd/ops/lib/variants
for rep in 1 2 3; do
  timeout -k 10 200 python scripts/kernel_bench.py --momentum-dtype bf16 > $OUT/kbench_n2w4_$rep.log 2>&1
  MOPT_KERNEL_LIB=$V/n3w3/libmopt_kernels.so timeout -k 10 200 python scripts/kernel_bench.py --momentum-dtype bf16 > $OUT/kbench_n3w3_$rep.log 2>&1
done
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_n2w4_$rep.json 2> $OUT/bench.err
  MOPT_KERNEL_LIB=$V/n3w3/libmopt_kernels.so timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench_n3w3_$rep.json 2> $OUT/bench_n3w3.err
done
OUT=gpurun_out/r4ag bash scripts/gpu.sh tests
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4ag/smoke.log 2>&1
echo done
