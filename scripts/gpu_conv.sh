#!/bin/bash
# Conv kernel microbench (direct vs implicit GEMM), ResNet-20 step time, LDS PMC pass.
set -e
OUT=${OUT:-gpurun_out/conv}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 200 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
timeout -k 10 200 python scripts/conv_bench.py --implicit --out "$OUT/conv_bench.json" > "$OUT/conv_bench.log" 2>&1
timeout -k 10 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > "$OUT/resnet20.json" 2> "$OUT/resnet20.err"
cd /tmp && export TMPDIR=/tmp
pmc() {
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --output-format csv --pmc "$@" -d "$ROOT/$OUT/$name" -o run -- \
      python3 "$ROOT/scripts/conv_bench.py" --iters 1 > "$ROOT/$OUT/$name.log" 2>&1
}
pmc sq SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_WAIT_INST_LDS
echo done
