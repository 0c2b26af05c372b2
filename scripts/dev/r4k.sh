set -e
OUT=gpurun_out/r4k bash scripts/gpu.sh tests:tests/test_resnet_gpu.py,tests/test_lm_gpu.py lm resnet trace_lm trace_resnet
echo done
