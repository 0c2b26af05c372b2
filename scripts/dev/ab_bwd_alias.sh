set -e
mkdir -p gpurun_out/ab1
K="timeout -k 10 200 python scripts/kernel_bench.py --momentum-dtype bf16 --iters 30"
NA=$PWD/metaopt_amd/ops/lib/variants/noalias/libmopt_kernels.so
MOPT_BWD_PREFETCH=1 $K > gpurun_out/ab1/alias_pf1.log 2>&1
MOPT_BWD_PREFETCH=0 $K > gpurun_out/ab1/alias_pf0.log 2>&1
MOPT_KERNEL_LIB=$NA MOPT_BWD_PREFETCH=1 $K > gpurun_out/ab1/noalias_pf1.log 2>&1
MOPT_KERNEL_LIB=$NA MOPT_BWD_PREFETCH=0 $K > gpurun_out/ab1/noalias_pf0.log 2>&1
MOPT_BWD_PREFETCH=0 $K > gpurun_out/ab1/alias_pf0_again.log 2>&1
