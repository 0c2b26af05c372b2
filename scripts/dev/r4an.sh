set -e
OUT=gpurun_out/r4an
mkdir -p $OUT
ROOT=$(pwd)
(cd /tmp && export TMPDIR=/tmp && timeout -s KILL 200 rocprofv3 --output-format csv \
    --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES \
    -d "$ROOT/$OUT/insts" -o run -- \
    python3 "$ROOT/scripts/bench_configs.py" --config resnet20 --steps 3 --warmup 2 \
    > "$ROOT/$OUT/insts.log" 2>&1)
echo done
