#!/bin/bash
# Round 5 final-tree validation (after the round-robin step queueing): GPU suite, smoke, headline bench
# x3, ResNet-20, LM-125M (PBT, 600 steps: three whole generations), conv microbench, hyper.
set -e
OUT=gpurun_out/r6x; mkdir -p $OUT
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1
echo tests ok
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
for rep in 1 2 3; do
  $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err
done
echo bench ok
$T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet20.json 2> $OUT/resnet20.err
$T 500 python scripts/bench_configs.py --config lm-125m --steps 600 --warmup 0 > $OUT/lm125m_pbt600.json 2> $OUT/lm125m_pbt600.err
echo lm ok
$T 200 python scripts/conv_bench.py --out $OUT/conv.json > $OUT/conv.log 2>&1
$T 300 python scripts/bench_configs.py --config hyper --steps 3 > $OUT/hyper.json 2> $OUT/hyper.err
echo done
