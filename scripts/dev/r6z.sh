#!/bin/bash
# Round 5 final tree: HBM bytes (FETCH_SIZE / WRITE_SIZE) and MFMA / LDS counters of the ResNet-20
# step's kernels (BatchNorm passes against their byte model), one counter set per run.
set -e
OUT=gpurun_out/r6z; mkdir -p $OUT
pass() {
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --output-format csv --pmc "$@" \
     -d $GRAFT_REPO_ROOT/$OUT/pmc_$name -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_configs.py \
     --config resnet20 --steps 30 --warmup 30 > $GRAFT_REPO_ROOT/$OUT/pmc_$name.log 2>&1)
  echo pass $name
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass busy GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVES
echo done
