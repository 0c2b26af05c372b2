#!/bin/bash
# Kernel trace of the headline bench (one configuration per call: ARGS), for gap analysis.
set -e
OUT=${OUT:-gpurun_out/trace_bench}
mkdir -p "$OUT"
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 5 $ARGS > "$ROOT/$OUT/bench.json" 2> "$ROOT/$OUT/bench.err"
echo done
