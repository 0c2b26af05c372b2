#!/bin/bash
# A/B: LDS-free forward (default build) vs the LDS-staged forward (variant fwdlds).
set -e
OUT=${OUT:-gpurun_out/ab_fwd}
mkdir -p "$OUT"
V=$PWD/metaopt_amd/ops/lib/variants/fwdlds/libmopt_kernels.so
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
for i in 1 2; do
  timeout -k 10 120 python scripts/kernel_bench.py --momentum-dtype bf16 > "$OUT/k_direct_$i.log" 2>&1
  MOPT_KERNEL_LIB=$V timeout -k 10 120 python scripts/kernel_bench.py --momentum-dtype bf16 > "$OUT/k_lds_$i.log" 2>&1
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > "$OUT/b_direct.json" 2>/dev/null
MOPT_KERNEL_LIB=$V timeout -k 10 200 python bench.py --steps 20 --warmup 5 > "$OUT/b_lds.json" 2>/dev/null
echo done
