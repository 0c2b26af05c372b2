set -e
OUT=gpurun_out/r4ad
mkdir -p $OUT
V=metaopt_amd/ops/lib/variants
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lm_gpu.py > $OUT/pytest_lm.log 2>&1
for rep in 1 2; do
  timeout -k 10 300 python scripts/bench_configs.py --config lm-125m --steps 20 --warmup 10 > $OUT/lm_new_$rep.json 2> $OUT/lm_new.err
  MOPT_KERNEL_LIB=$V/epi3old/libmopt_kernels.so timeout -k 10 300 python scripts/bench_configs.py --config lm-125m --steps 20 --warmup 10 > $OUT/lm_old_$rep.json 2> $OUT/lm_old.err
done
OUT=gpurun_out/r4ad bash scripts/gpu.sh trace_lm
WORLD=8 PRIORS=headline N_SYNCS=60 timeout -k 10 300 python scripts/profile_decide.py > $OUT/decide_world8_headline_stagger.log 2>&1
echo done
