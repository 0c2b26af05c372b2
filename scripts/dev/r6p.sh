#!/bin/bash
# Round 5: per-kernel times of the bit-mask BatchNorm (this tree) vs ab_base, ResNet-20.
set -e
OUT=gpurun_out/r6p; mkdir -p $OUT
T="timeout -k 10"
prof() {
  local name=$1 root=$2
  (cd /tmp && export TMPDIR=/tmp && $T 300 rocprofv3 --kernel-trace --stats --output-format csv \
     -d $GRAFT_REPO_ROOT/$OUT/$name -o run -- python3 $root/scripts/bench_configs.py --config resnet20 --steps 30 --warmup 30 > $GRAFT_REPO_ROOT/$OUT/$name.log 2>&1)
}
prof new $GRAFT_REPO_ROOT
prof base $GRAFT_REPO_ROOT/ab_base
echo done
