set -e
OUT=gpurun_out/r4j bash scripts/gpu.sh tests:tests/test_resnet_gpu.py,tests/test_lm_gpu.py resnet trace_resnet
ROOT=$(pwd)
for v in 1 2 1 2; do
  MOPT_ATTN_FWD=$v timeout -k 10 300 python scripts/bench_configs.py --config lm-125m --steps 20 --warmup 10 > gpurun_out/r4j/lm_attn$v.json 2> gpurun_out/r4j/lm_attn$v.err
done
OUT=gpurun_out/r4j bash scripts/gpu.sh trace_lm
for pass in "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES" "FETCH_SIZE"; do
  name=pmc_gemm_$(echo $pass | cut -d' ' -f1)
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 120 rocprofv3 --output-format csv --pmc $pass -d "$ROOT/gpurun_out/r4j/$name" -o run -- python3 "$ROOT/scripts/gemm_bench.py" --shapes lm.gu.fwd --no-torch --iters 5 > "$ROOT/gpurun_out/r4j/$name.log" 2>&1)
done
echo done
