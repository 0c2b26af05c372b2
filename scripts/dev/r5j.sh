#!/bin/bash
# Round 5: live extents in the MLP kernels (buffer loads/stores skip the padding): tests, A/B.
set -e
OUT=gpurun_out/r5j; mkdir -p $OUT
T="timeout -k 10"
$T 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py tests/test_checked_build_gpu.py tests/test_resume.py > $OUT/pytest_mlp.log 2>&1
echo tests ok
$T 200 python scripts/kernel_bench.py --momentum-dtype bf16 > $OUT/kb.log 2>&1
for rep in 1 2; do
  $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err
  (cd ab_base && $T 240 python bench.py --steps 20 --warmup 5) > $OUT/bench_base_$rep.json 2> $OUT/bench_base_$rep.err
done
echo done
