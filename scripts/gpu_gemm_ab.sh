#!/bin/bash
# Population GEMM A/B: default library vs a variant build (VARIANT), LM shapes, interleaved runs;
# then PMC counters of the default build (LDS, L2, HBM, MFMA) on the same shapes.
set -e
OUT=${OUT:-gpurun_out/gemm_ab}
ROOT=$(pwd)
mkdir -p "$OUT"
V=$ROOT/metaopt_amd/ops/lib/variants/$VARIANT/libmopt_kernels.so
timeout -k 10 300 python -u -m pytest tests/test_pgemm_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
MOPT_KERNEL_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_pgemm_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_variant.log" 2>&1
for i in 1 2; do
  timeout -k 10 200 python scripts/gemm_bench.py --shapes lm --no-torch > "$OUT/default_$i.log" 2>&1
  MOPT_KERNEL_LIB=$V timeout -k 10 200 python scripts/gemm_bench.py --shapes lm --no-torch > "$OUT/variant_$i.log" 2>&1
done
if [ -n "$PMC" ]; then
  cd /tmp && export TMPDIR=/tmp
  pmc() {
    local name=$1; shift
    timeout -s KILL 120 rocprofv3 --output-format csv --pmc "$@" -d "$ROOT/$OUT/pmc_$name" -o run -- \
        python3 "$ROOT/scripts/gemm_bench.py" --shapes lm --no-torch --iters 2 > "$ROOT/$OUT/pmc_$name.log" 2>&1
  }
  pmc lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS
  pmc l2 TCC_HIT_sum TCC_MISS_sum
  pmc fetch FETCH_SIZE
  pmc mfma SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVES
fi
echo done
