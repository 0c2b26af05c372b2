set -e
OUT=gpurun_out/r4al bash scripts/gpu.sh tests bench
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4al/smoke.log 2>&1
echo done
