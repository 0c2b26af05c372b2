#!/bin/bash
# Headline bench at N=1 and multi-rank rehearsals (ranks share the one GPU over gloo) with the
# child-process storage writer; GPU-event timeline at N=1.
set -e
OUT=${OUT:-gpurun_out/r2_scale}
mkdir -p "$OUT"
MOPT_GPU_TIMELINE=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > "$OUT/n1.json" 2> "$OUT/n1.err"
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > "$OUT/n2.json" 2> "$OUT/n2.err"
timeout -k 10 300 python bench.py --gpus 4 --steps 10 --warmup 3 > "$OUT/n4.json" 2> "$OUT/n4.err"
echo done
