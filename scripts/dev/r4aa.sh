set -e
OUT=gpurun_out/r4aa bash scripts/gpu.sh pmc_kbench
echo done
