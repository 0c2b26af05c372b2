#!/bin/bash
# GPU measurement recipe (run on the box through gpurun from the repo root):
#   bench.py, per-kernel microbench, rocprofv3 kernel trace of the bench, PMC counters of the
#   kernels (own runs; counters never combined with trace domains).
set -e
OUT=${OUT:-gpurun_out/prof}
mkdir -p "$OUT"
ROOT=$(pwd)
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
timeout -k 10 300 python scripts/kernel_bench.py --momentum-dtype bf16 --out "$OUT/kbench.json" > "$OUT/kbench.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 3 > "$ROOT/$OUT/trace.log" 2>&1
# derived counters expand to many hardware counters: one derived counter per pass
pmc() {
  local name=$1; shift
  timeout -k 10 180 rocprofv3 --output-format csv --pmc "$@" -d "$ROOT/$OUT/$name" -o run -- \
      python3 "$ROOT/scripts/kernel_bench.py" --iters 3 --momentum-dtype bf16 > "$ROOT/$OUT/$name.log" 2>&1
}
if [ -z "$NO_PMC" ]; then
  pmc pmc_fetch FETCH_SIZE
  pmc pmc_write WRITE_SIZE
  pmc pmc_mfma SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES
  pmc pmc_lds SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES
fi
echo done
