set -e
OUT=gpurun_out/r4ao
mkdir -p $OUT
V=metaopt_amd/ops/lib/variants
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_resnet_gpu.py > $OUT/pytest_resnet.log 2>&1
for rep in 1 2; do
  timeout -k 10 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet_new_$rep.json 2> $OUT/resnet_new.err
  MOPT_KERNEL_LIB=$V/wgold/libmopt_kernels.so timeout -k 10 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet_old_$rep.json 2> $OUT/resnet_old.err
done
OUT=gpurun_out/r4ao bash scripts/gpu.sh trace_resnet
echo done
