set -e
OUT=gpurun_out/r4ae
mkdir -p $OUT
timeout -k 10 400 python scripts/gemm_bench.py --shapes lm. --no-torch --cfgs 5,6,7,11 --splits 5:2,6:2,7:2,11:2,5:4,6:4,7:4,11:4 --out $OUT/gemm_lm.json > $OUT/gemm_lm.log 2>&1
echo done
