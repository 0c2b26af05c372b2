#!/bin/bash
# LM / ResNet / hypergradient configs: GPU tests of the model families, then the config benches
# (lm-125m with the library NN forward on and off) and a kernel trace of the LM step.
set -e
OUT=${OUT:-gpurun_out/lm}
ROOT=$(pwd)
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests/test_lm_gpu.py tests/test_resnet_gpu.py tests/test_hyper.py tests/test_pgemm_ad.py -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1
timeout -k 10 300 python scripts/bench_configs.py --config lm-125m --steps 20 --warmup 10 > "$OUT/lm.json" 2> "$OUT/lm.err"
MOPT_LIBRARY_NN=1 timeout -k 10 300 python scripts/bench_configs.py --config lm-125m --steps 20 --warmup 10 > "$OUT/lm_lib.json" 2> "$OUT/lm_lib.err"
timeout -k 10 300 python scripts/bench_configs.py --config resnet20 --steps 40 --warmup 10 > "$OUT/resnet.json" 2> "$OUT/resnet.err"
timeout -k 10 300 python scripts/bench_configs.py --config hyper --steps 3 > "$OUT/hyper.json" 2> "$OUT/hyper.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$ROOT/$OUT/trace" -o lm -- python3 "$ROOT/scripts/bench_configs.py" --config lm-125m --steps 6 --warmup 4 > "$ROOT/$OUT/trace.log" 2>&1
echo done
