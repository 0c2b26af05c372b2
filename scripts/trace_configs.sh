#!/bin/bash
# Kernel traces (rocprofv3 --kernel-trace --stats) of BASELINE configs 3 and 5 on one GPU.
set -e
OUT=${OUT:-gpurun_out/trace_cfg}
ROOT=$(pwd)
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/resnet20" -o run -- \
    python3 "$ROOT/scripts/bench_configs.py" --config resnet20 --steps 30 --warmup 30 > "$ROOT/$OUT/resnet20.log" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/lm125m" -o run -- \
    python3 "$ROOT/scripts/bench_configs.py" --config lm-125m --steps 20 --warmup 10 > "$ROOT/$OUT/lm125m.log" 2>&1
echo done
