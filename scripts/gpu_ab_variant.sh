#!/bin/bash
# A/B of a kernel variant build (VARIANT=name under ops/lib/variants) against the default
# library: kernel_bench twice each, then the headline bench once each.
set -e
OUT=${OUT:-gpurun_out/ab_$VARIANT}
mkdir -p "$OUT"
V=$PWD/metaopt_amd/ops/lib/variants/$VARIANT/libmopt_kernels.so
MOPT_KERNEL_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_variant.log" 2>&1
for i in 1 2; do
  timeout -k 10 120 python scripts/kernel_bench.py --momentum-dtype bf16 > "$OUT/k_default_$i.log" 2>&1
  MOPT_KERNEL_LIB=$V timeout -k 10 120 python scripts/kernel_bench.py --momentum-dtype bf16 > "$OUT/k_variant_$i.log" 2>&1
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > "$OUT/b_default.json" 2>/dev/null
MOPT_KERNEL_LIB=$V timeout -k 10 200 python bench.py --steps 20 --warmup 5 > "$OUT/b_variant.json" 2>/dev/null
echo done
