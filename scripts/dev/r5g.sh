#!/bin/bash
# Round 5: in-situ per-kernel trace of the headline bench (64 vs 128 forward) + stream groups A/B.
set -e
OUT=gpurun_out/r5g; mkdir -p $OUT
ROOT=$(pwd)
T="timeout -k 10"
prof() {   # prof NAME -- cmd...
  local name=$1; shift 2
  (cd /tmp && export TMPDIR=/tmp && $T 300 rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$ROOT/$OUT/$name" -o run -- "$@" > "$ROOT/$OUT/$name.log" 2>&1)
}
MOPT_FWD_TN=64 prof trace_tn64 -- python3 "$ROOT/bench.py" --steps 10 --warmup 3
MOPT_FWD_TN=128 prof trace_tn128 -- python3 "$ROOT/bench.py" --steps 10 --warmup 3
echo traces ok
for s in 1 2 3; do MOPT_STREAMS=$s $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_streams$s.json 2> $OUT/bench_streams$s.err; done
echo done
