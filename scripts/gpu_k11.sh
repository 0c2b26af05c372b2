#!/bin/bash
# K11 on the MFMA GEMM: GPU numerics, config-4 throughput, kernel trace of the outer steps.
set -e
OUT=${OUT:-gpurun_out/k11}
mkdir -p "$OUT"
ROOT=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_pgemm_ad.py tests/test_lm_gpu.py -m gpu -q -k "hyper or forward_over" --timeout 120 --timeout-method thread -rA > "$OUT/pytest.log" 2>&1 || true
timeout -k 10 300 python scripts/bench_configs.py --config hyper --steps 3 --warmup 1 > "$OUT/bench_hyper.json" 2> "$OUT/bench_hyper.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace" -o run -- \
    python3 "$ROOT/scripts/bench_configs.py" --config hyper --steps 1 --warmup 0 > "$ROOT/$OUT/trace.log" 2>&1
echo done
