#!/bin/bash
# Round 5 final-tree validation: GPU suite, smoke, headline bench x2, ResNet-20, LM-125M (PBT,
# 400 steps), conv microbench with HBM PMC passes (FETCH_SIZE / WRITE_SIZE).
set -e
OUT=gpurun_out/r6c; mkdir -p $OUT
T="timeout -k 10"
$T 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests > $OUT/pytest_gpu.log 2>&1
echo tests ok
$T 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
for rep in 1 2; do
  $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_$rep.json 2> $OUT/bench_$rep.err
done
echo bench ok
$T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > $OUT/resnet20.json 2> $OUT/resnet20.err
$T 400 python scripts/bench_configs.py --config lm-125m --steps 400 --warmup 0 > $OUT/lm125m_pbt400.json 2> $OUT/lm125m_pbt400.err
$T 200 python scripts/conv_bench.py --out $OUT/conv.json > $OUT/conv.log 2>&1
for c in FETCH_SIZE WRITE_SIZE; do
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --output-format csv --pmc $c -d $GRAFT_REPO_ROOT/$OUT/pmc_conv_$c -o run -- python3 $GRAFT_REPO_ROOT/scripts/conv_bench.py --iters 3 > $GRAFT_REPO_ROOT/$OUT/pmc_conv_$c.log 2>&1)
done
echo done
