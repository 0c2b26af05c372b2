#!/bin/bash
# Round 5: headline bench run-to-run variance on one box (back to back, then after a pause) with
# the card's temperature / power / clocks around each run (rocm-smi, read-only).
OUT=gpurun_out/r6e; mkdir -p $OUT
T="timeout -k 10"
smi() { timeout 20 rocm-smi --showtemp --showpower --showclocks --showuse > "$OUT/smi_$1.txt" 2>&1 || true; }
smi start
for rep in 1 2 3 4; do
  $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err || exit 1
  smi after_$rep
done
sleep 60
smi pause
$T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_5.json 2> $OUT/bench_5.err || exit 1
smi after_5
echo done
