#!/bin/bash
# A/B of the population train step: HIP streams per population and the momentum buffer dtype
# (bench.py, N=1), after the GPU test suite.
set -e
OUT=${OUT:-gpurun_out/ab_streams}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
for cfg in "1 fp32" "2 fp32" "3 fp32" "1 bf16" "2 bf16"; do
  set -- $cfg
  MOPT_STREAMS=$1 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --momentum-dtype $2 > "$OUT/bench_s$1_$2.json" 2> "$OUT/bench_s$1_$2.err"
done
echo done
