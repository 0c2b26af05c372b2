# A/B of the MLP weight layout (k-strip-major default vs row-major variant build), one box
set -e
mkdir -p gpurun_out/ab2
K="timeout -k 10 200 python scripts/kernel_bench.py --momentum-dtype bf16 --iters 30"
RM=$PWD/metaopt_amd/ops/lib/variants/rowmajor/libmopt_kernels.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py > gpurun_out/ab2/pytest.log 2>&1
$K > gpurun_out/ab2/strip.log 2>&1
MOPT_KERNEL_LIB=$RM $K > gpurun_out/ab2/rowmajor.log 2>&1
$K > gpurun_out/ab2/strip_again.log 2>&1
MOPT_BWD_PREFETCH=0 $K > gpurun_out/ab2/strip_pf0.log 2>&1
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > gpurun_out/ab2/bench.json 2> gpurun_out/ab2/bench.err
