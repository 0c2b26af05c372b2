set -e
OUT=gpurun_out/r4ab bash scripts/gpu.sh tests bench bench_long resnet lm hyper trace_bench
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4ab/smoke.log 2>&1
echo done
