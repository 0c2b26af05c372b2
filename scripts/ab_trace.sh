#!/bin/bash
# Kernel-time A/B of two kernel-library builds inside the headline bench:
#   bash scripts/ab_trace.sh <variant.so>   (B = the in-tree library)
set -e
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/ab_trace
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
MOPT_KERNEL_LIB=$1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/a" -o run -- \
    python3 "$ROOT/bench.py" --steps 128 --warmup 32 > "$OUT/a.json" 2> "$OUT/a.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/b" -o run -- \
    python3 "$ROOT/bench.py" --steps 128 --warmup 32 > "$OUT/b.json" 2> "$OUT/b.err"
for v in a b; do
  echo "== $v"; tail -1 "$OUT/$v.json" | cut -c1-100
  python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$OUT/$v/run_kernel_stats.csv')))
for r in rows[:6]: print(r['Name'][:60], r['Calls'], r['AverageNs'], r['Percentage'])
"
done
