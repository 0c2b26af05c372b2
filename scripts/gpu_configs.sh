#!/bin/bash
# Throughput of BASELINE configs 3, 4, 5 on one GPU (each step under its own time limit).
set -e
OUT=${OUT:-gpurun_out/configs}
mkdir -p "$OUT"
timeout -k 10 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > "$OUT/resnet20.json" 2> "$OUT/resnet20.err"
timeout -k 10 300 python scripts/bench_configs.py --config lm-tiny --steps 100 --warmup 50 > "$OUT/lm_tiny.json" 2> "$OUT/lm_tiny.err"
timeout -k 10 400 python scripts/bench_configs.py --config lm-125m --steps 50 --warmup 50 > "$OUT/lm_125m.json" 2> "$OUT/lm_125m.err"
timeout -k 10 300 python scripts/bench_configs.py --config hyper --steps 3 --warmup 1 > "$OUT/hyper.json" 2> "$OUT/hyper.err"
cat "$OUT"/*.json
