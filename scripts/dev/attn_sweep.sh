set -e
OUT=gpurun_out/r4q
mkdir -p $OUT
V=metaopt_amd/ops/lib/variants
for rep in 1 2; do
  timeout -k 10 120 python scripts/attn_bench.py >> $OUT/attn_sweep.log 2>&1
  for n in w343 w443 w053 w033 w042 w044 w243; do
    MOPT_KERNEL_LIB=$V/$n/libmopt_kernels.so timeout -k 10 120 python scripts/attn_bench.py >> $OUT/attn_sweep.log 2>&1
  done
done
echo done
