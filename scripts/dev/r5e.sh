#!/bin/bash
# Round 5: narrow loss layer + W-direct 128-column forward (MOPT_FWD_TN=128) A/B, one box.
set -e
OUT=gpurun_out/r5e; mkdir -p $OUT
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_hyper.py tests/test_checked_build_gpu.py > $OUT/pytest.log 2>&1
echo tests ok
for rep in 1 2; do
  MOPT_FWD_TN=64 $T 200 python scripts/kernel_bench.py --momentum-dtype bf16 > $OUT/kb_tn64_$rep.log 2>&1
  MOPT_FWD_TN=64 MOPT_NARROW=0 $T 200 python scripts/kernel_bench.py --momentum-dtype bf16 > $OUT/kb_tn64_wide_$rep.log 2>&1
  MOPT_FWD_TN=128 $T 200 python scripts/kernel_bench.py --momentum-dtype bf16 > $OUT/kb_tn128_w3_$rep.log 2>&1
  MOPT_FWD_TN=128 MOPT_KERNEL_LIB=metaopt_amd/ops/lib/variants/fwdw2/libmopt_kernels.so $T 200 python scripts/kernel_bench.py --momentum-dtype bf16 > $OUT/kb_tn128_w2_$rep.log 2>&1
  echo rep $rep
done
MOPT_FWD_TN=128 $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_tn128.json 2> $OUT/bench_tn128.err
MOPT_FWD_TN=64 $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_tn64.json 2> $OUT/bench_tn64.err
echo done
