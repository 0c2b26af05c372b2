set -e
mkdir -p gpurun_out/ab1
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab1/pytest.log 2>&1
tail -2 gpurun_out/ab1/pytest.log
for i in 1 2; do
  MOPT_KERNEL_LIB=$PWD/metaopt_amd/ops/lib/libmopt_kernels_base.so timeout -k 10 300 python bench.py --steps 256 --warmup 64 2>/dev/null | tail -1 | cut -c1-120
  timeout -k 10 300 python bench.py --steps 256 --warmup 64 2>/dev/null | tail -1 | cut -c1-120
done
