#!/bin/bash
# Round-2 headline measurement on one MI355X (run from the repo root through gpurun):
#   driver-shaped bench (N=1, --steps 20 --warmup 5), a longer run, random vs ASHA at the same
#   budget, the 2-rank launcher as a gloo rehearsal, and a rocprofv3 kernel trace of the bench.
set -e
OUT=${OUT:-gpurun_out/r2}
mkdir -p "$OUT"
ROOT=$(pwd)
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > "$OUT/pytest_gpu.log" 2>&1
fi
timeout -k 10 240 python bench.py --steps 20 --warmup 5 > "$OUT/bench_n1.json" 2> "$OUT/bench_n1.err"
timeout -k 10 240 python bench.py --steps 60 --warmup 5 > "$OUT/bench_n1_long.json" 2> "$OUT/bench_n1_long.err"
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --algo random > "$OUT/bench_random.json" 2> "$OUT/bench_random.err"
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > "$OUT/bench_n2_rehearsal.json" 2> "$OUT/bench_n2.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 20 --warmup 5 > "$ROOT/$OUT/trace.log" 2>&1
echo done
