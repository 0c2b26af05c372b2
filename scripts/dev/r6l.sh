#!/bin/bash
# Round 5: conv workgroup counts: weight gradient 512 / 768 / 1024, and with wgrad 1024 the
# forward/data-gradient total 2048 or 512 (default 1024); 3 interleaved ResNet-20 repetitions.
set -e
OUT=gpurun_out/r6l; mkdir -p $OUT
T="timeout -k 10"
V=$GRAFT_REPO_ROOT/metaopt_amd/ops/lib/variants
for rep in 1 2 3; do
  for v in wg512 wg768 wg1024 f2048 f512; do
    if [ $v = base ]; then L=""; else L=$V/$v/libmopt_kernels.so; fi
    MOPT_KERNEL_LIB=$L $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet_${v}_$rep.json 2> $OUT/resnet_${v}_$rep.err
  done
  echo rep $rep
done
echo done
