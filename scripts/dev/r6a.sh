#!/bin/bash
# Round 5: swizzled attention LDS tiles (common.h soff) with dQ / dK-dV at 3 / 2 waves --
# correctness, attention bench and LM-125M A/B against the previous commit (ab_base): dK/dV: vectorised LSE / Dsum LDS reads, 32-bit query-block offsets.
set -e
OUT=gpurun_out/r6a; mkdir -p $OUT
T="timeout -k 10"
$T 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_lm_gpu.py tests/test_kernels_gpu.py > $OUT/pytest.log 2>&1
echo tests ok
for rep in 1 2 3; do
  $T 120 python scripts/attn_bench.py --out $OUT/attn_new_$rep.json > $OUT/attn_new_$rep.log 2>&1
  (cd ab_base && $T 120 python scripts/attn_bench.py --out ../$OUT/attn_base_$rep.json > ../$OUT/attn_base_$rep.log 2>&1)
done
echo attn ok
$T 300 python scripts/bench_configs.py --config lm-125m --steps 200 --warmup 0 > $OUT/lm_new.json 2> $OUT/lm_new.err
(cd ab_base && $T 300 python scripts/bench_configs.py --config lm-125m --steps 200 --warmup 0 > ../$OUT/lm_base.json 2> ../$OUT/lm_base.err)
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --output-format csv --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES -d $GRAFT_REPO_ROOT/$OUT/pmc_lds -o run -- python3 $GRAFT_REPO_ROOT/scripts/attn_bench.py --iters 2 > $GRAFT_REPO_ROOT/$OUT/pmc_lds.log 2>&1)
echo done
