#!/bin/bash
# Round 5: steady-state LM-125M kernel trace; rank-0 decide at W = 8 on the box CPU.
set -e
OUT=gpurun_out/r5l; mkdir -p $OUT
ROOT=$(pwd)
T="timeout -k 10"
(cd /tmp && export TMPDIR=/tmp && $T 300 rocprofv3 --kernel-trace --stats --output-format csv \
   -d "$ROOT/$OUT/trace_lm" -o run -- python3 "$ROOT/scripts/bench_configs.py" --config lm-125m \
   --sync-every 10 --steps 20 --warmup 10 > "$ROOT/$OUT/trace_lm.log" 2>&1)
echo trace ok
WORLD=8 $T 300 python scripts/profile_decide.py > $OUT/decide_world8_stress.log 2>&1
WORLD=8 PRIORS=headline $T 300 python scripts/profile_decide.py > $OUT/decide_world8_headline.log 2>&1
echo done
