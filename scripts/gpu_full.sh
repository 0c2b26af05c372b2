#!/bin/bash
# Full round-end rehearsal: every GPU test, smoke(), the driver's bench command, configs 3-5.
set -e
OUT=${OUT:-gpurun_out/full}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
OUT=$OUT bash scripts/gpu_configs.sh > /dev/null
echo tests-and-benches done
# kernel tables of the final state (LM 125M, ResNet-20, config 4)
ROOT=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/lm" -o lm -- python3 "$ROOT/scripts/bench_configs.py" --config lm-125m --steps 6 --warmup 4 > "$ROOT/$OUT/lm_prof.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/k11" -o k11 -- python3 "$ROOT/scripts/bench_configs.py" --config hyper --steps 1 --warmup 1 > "$ROOT/$OUT/k11_prof.log" 2>&1
echo traces done
