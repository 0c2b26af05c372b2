#!/bin/bash
# Round 5: XOR-swizzled backward LDS tiles (conflict-free fragment reads) -- tests, kernel bench,
# PMC LDS pass and headline A/B against the previous commit (ab_base).
set -e
OUT=gpurun_out/r5v; mkdir -p $OUT
T="timeout -k 10"
$T 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_kernels_gpu.py > $OUT/pytest.log 2>&1
echo tests ok
$T 120 python scripts/kernel_bench.py --momentum-dtype bf16 --out $OUT/kb_new.json > $OUT/kb_new.log 2>&1
(cd ab_base && $T 120 python scripts/kernel_bench.py --momentum-dtype bf16 --out ../$OUT/kb_base.json > ../$OUT/kb_base.log 2>&1)
for rep in 1 2; do
  $T 240 python bench.py --steps 20 --warmup 5 > $OUT/bench_new_$rep.json 2> $OUT/bench_new_$rep.err
  (cd ab_base && $T 240 python bench.py --steps 20 --warmup 5 > ../$OUT/bench_base_$rep.json 2> ../$OUT/bench_base_$rep.err)
  echo rep $rep
done
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $GRAFT_REPO_ROOT/$OUT/pmc_lds -o run -- python3 $GRAFT_REPO_ROOT/scripts/kernel_bench.py --iters 3 --momentum-dtype bf16 > $GRAFT_REPO_ROOT/$OUT/pmc_lds.log 2>&1)
echo done
