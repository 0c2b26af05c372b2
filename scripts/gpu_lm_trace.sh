#!/bin/bash
# 125M-LM step time (two runs) and a kernel trace of a few steps.
set -e
OUT=${OUT:-gpurun_out/lmt}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 300 python scripts/bench_configs.py --config lm-125m --steps 20 --warmup 10 > "$OUT/lm1.json" 2> "$OUT/lm1.err"
timeout -k 10 300 python scripts/bench_configs.py --config lm-125m --steps 20 --warmup 10 > "$OUT/lm2.json" 2> "$OUT/lm2.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/lm" -o lm -- python3 "$ROOT/scripts/bench_configs.py" --config lm-125m --steps 4 --warmup 3 > "$ROOT/$OUT/lm.log" 2>&1
echo done
