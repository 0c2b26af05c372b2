#!/bin/bash
# Population GEMM: numerics of every tile configuration, then throughput per configuration on the
# LM / ResNet shapes against hipBLASLt.
set -e
OUT=${OUT:-gpurun_out/gemm}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_pgemm_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
timeout -k 10 300 python scripts/gemm_bench.py --cfgs ${CFGS:-0,5,6,7} --out "$OUT/gemm.json" > "$OUT/gemm.log" 2>&1
echo done
