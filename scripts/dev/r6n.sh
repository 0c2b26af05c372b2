#!/bin/bash
# Round 5: kernel-trace profiles of ResNet-20 and LM-125M on the current tree (per-kernel shares).
set -e
OUT=gpurun_out/r6n; mkdir -p $OUT
T="timeout -k 10"
prof() {
  local name=$1 lim=$2; shift 2
  (cd /tmp && export TMPDIR=/tmp && $T $lim rocprofv3 --kernel-trace --stats --output-format csv \
     -d $GRAFT_REPO_ROOT/$OUT/$name -o run -- python3 "$@" > $GRAFT_REPO_ROOT/$OUT/$name.log 2>&1)
}
prof resnet 300 $GRAFT_REPO_ROOT/scripts/bench_configs.py --config resnet20 --steps 30 --warmup 30
prof lm 400 $GRAFT_REPO_ROOT/scripts/bench_configs.py --config lm-125m --steps 60 --warmup 0
echo done
