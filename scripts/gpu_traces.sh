#!/bin/bash
# Kernel traces (timestamps) of the 125M-LM step and of one config-4 outer step.
set -e
OUT=${OUT:-gpurun_out/traces}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/lm" -o lm -- python3 "$ROOT/scripts/bench_configs.py" --config lm-125m --steps 4 --warmup 3 > "$ROOT/$OUT/lm.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/k11" -o k11 -- python3 "$ROOT/scripts/bench_configs.py" --config hyper --steps 1 --warmup 1 > "$ROOT/$OUT/k11.log" 2>&1
echo done
