#!/bin/bash
# ResNet-20 (config 3): conv/BN numerics tests, step time with the direct conv kernels vs the
# implicit GEMM (MOPT_CONV_IMPLICIT=1), kernel-time table of the direct path.
set -e
OUT=${OUT:-gpurun_out/resnet}
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_resnet_gpu.py -x -v --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
timeout -k 10 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > "$OUT/resnet20.json" 2> "$OUT/resnet20.err"
MOPT_CONV_IMPLICIT=1 timeout -k 10 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > "$OUT/resnet20_implicit.json" 2> "$OUT/resnet20_implicit.err"
timeout -k 10 200 python scripts/conv_bench.py --implicit --out "$OUT/conv_bench.json" > "$OUT/conv_bench.log" 2>&1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- python scripts/bench_configs.py --config resnet20 --steps 20 --warmup 10 > "$OUT/prof.log" 2>&1
echo done
