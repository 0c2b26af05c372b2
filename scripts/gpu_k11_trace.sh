#!/bin/bash
# Kernel trace of config 4 (one outer step after one warm-up).
set -e
OUT=${OUT:-gpurun_out/k11t}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/k11" -o k11 -- python3 "$ROOT/scripts/bench_configs.py" --config hyper --steps 1 --warmup 1 > "$ROOT/$OUT/k11.log" 2>&1
echo done
