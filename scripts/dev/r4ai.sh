set -e
OUT=gpurun_out/r4ai bash scripts/gpu.sh bench bench_long resnet lm hyper trace_lm trace_resnet
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4ai/smoke.log 2>&1
echo done
