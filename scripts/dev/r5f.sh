#!/bin/bash
# Round 5: MLP forward A/B (64-column vs W-direct 128-column), ring GEMM correctness + A/B, one box.
set -e
OUT=gpurun_out/r5f; mkdir -p $OUT
T="timeout -k 10"
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"
$T 300 $PYT tests/test_kernels_gpu.py tests/test_hyper.py > $OUT/pytest_mlp.log 2>&1
echo mlp tests ok
$T 400 $PYT tests/test_pgemm_gpu.py tests/test_lm_gpu.py > $OUT/pytest_gemm.log 2>&1
echo gemm tests ok
for rep in 1 2; do
  MOPT_FWD_TN=64 $T 200 python scripts/kernel_bench.py --momentum-dtype bf16 > $OUT/kb_tn64_$rep.log 2>&1
  MOPT_FWD_TN=64 MOPT_NARROW=0 $T 200 python scripts/kernel_bench.py --momentum-dtype bf16 > $OUT/kb_tn64_wide_$rep.log 2>&1
  MOPT_FWD_TN=128 $T 200 python scripts/kernel_bench.py --momentum-dtype bf16 > $OUT/kb_tn128_w3_$rep.log 2>&1
  MOPT_FWD_TN=128 MOPT_KERNEL_LIB=metaopt_amd/ops/lib/variants/fwdw2/libmopt_kernels.so $T 200 python scripts/kernel_bench.py --momentum-dtype bf16 > $OUT/kb_tn128_w2_$rep.log 2>&1
  echo kb rep $rep
done
$T 300 python scripts/gemm_bench.py --no-torch --shapes lm --cfgs 5,6,7,11,12,13 --splits 12:2,13:2,5:2 --out $OUT/gemm.json > $OUT/gemm.log 2>&1
echo gemm bench ok
MOPT_FWD_TN=128 $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_tn128.json 2> $OUT/bench_tn128.err
MOPT_FWD_TN=64 $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_tn64.json 2> $OUT/bench_tn64.err
for r in 0 1; do
  MOPT_GEMM_RING=$r $T 300 python scripts/bench_configs.py --config lm-125m --steps 400 --warmup 0 > $OUT/lm_ring$r.json 2> $OUT/lm_ring$r.err
done
echo done
