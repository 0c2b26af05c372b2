set -e
OUT=gpurun_out/r4r
mkdir -p $OUT
MOPT_GEMM_RP=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pgemm_gpu.py > $OUT/pytest_rp.log 2>&1
for v in 0 1 0 1; do
  MOPT_GEMM_RP=$v timeout -k 10 300 python scripts/gemm_bench.py --no-torch --shapes lm --out $OUT/gemm_rp$v.json > $OUT/gemm_rp$v.log 2>&1
done
for v in 0 1; do
  MOPT_GEMM_RP=$v timeout -k 10 300 python scripts/bench_configs.py --config lm-125m --steps 20 --warmup 10 > $OUT/lm_rp$v.json 2> $OUT/lm_rp$v.err
done
echo done
