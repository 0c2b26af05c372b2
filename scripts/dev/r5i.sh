#!/bin/bash
# Round 5: validation of the 3-stream default (GPU suite, smoke, bench, GPU timeline), one box.
set -e
OUT=gpurun_out/r5i; mkdir -p $OUT
T="timeout -k 10"
$T 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1
echo tests ok
$T 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
$T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
MOPT_GPU_TIMELINE=1 $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_timeline.json 2> $OUT/bench_timeline.err
$T 300 python bench.py --steps 43 --warmup 5 > $OUT/bench_43.json 2> $OUT/bench_43.err
echo done
