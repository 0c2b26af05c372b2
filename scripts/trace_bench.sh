#!/bin/bash
# Kernel trace of the headline bench (rocprofv3 --kernel-trace --stats) for the per-kernel split
# and the GPU idle share of the timed window.
set -e
OUT=${OUT:-gpurun_out/trace_bench}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 128 --warmup 64 > "$ROOT/$OUT/bench.json" 2> "$ROOT/$OUT/bench.err"
echo done
