#!/bin/bash
# Round 5 validation of the current tree: GPU suite, smoke, headline bench (20 and 43 intervals,
# GPU timeline), config benches (PBT LM-125M 600 steps, ResNet-20, hyper), in-situ trace.
set -e
OUT=gpurun_out/r5y; mkdir -p $OUT
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1
echo tests ok
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
echo smoke ok
$T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err
MOPT_GPU_TIMELINE=1 $T 400 python bench.py --steps 43 --warmup 5 > $OUT/bench_48.json 2> $OUT/bench_48.err
echo bench ok
$T 400 python scripts/bench_configs.py --config lm-125m --steps 600 --warmup 0 > $OUT/lm125m_pbt600.json 2> $OUT/lm125m_pbt600.err
$T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet20.json 2> $OUT/resnet20.err
$T 300 python scripts/bench_configs.py --config hyper --steps 3 --warmup 1 > $OUT/hyper.json 2> $OUT/hyper.err
echo configs ok
(cd /tmp && export TMPDIR=/tmp && $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_bench -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 8 --warmup 3 > $GRAFT_REPO_ROOT/$OUT/trace_bench.log 2>&1)
(cd /tmp && export TMPDIR=/tmp && $T 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof_resnet -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py --config resnet20 --sync-every 10 --steps 20 --warmup 10 > $GRAFT_REPO_ROOT/$OUT/trace_resnet.log 2>&1)
echo done
