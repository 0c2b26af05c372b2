#!/bin/bash
# A/B of build-free MLP kernel switches on one box: OUT=dir bash scripts/dev/kb_ab.sh
set -e
OUT=${OUT:-gpurun_out/kb_ab}
mkdir -p "$OUT"
T="timeout -k 10 200"
$T python scripts/kernel_bench.py --momentum-dtype bf16 > "$OUT/kb_default.log" 2>&1
MOPT_BWD_PREFETCH=0 $T python scripts/kernel_bench.py --momentum-dtype bf16 > "$OUT/kb_nopf.log" 2>&1
MOPT_FWD_TN=128 $T python scripts/kernel_bench.py --momentum-dtype bf16 > "$OUT/kb_tn128.log" 2>&1
$T python scripts/kernel_bench.py --momentum-dtype bf16 > "$OUT/kb_default2.log" 2>&1
