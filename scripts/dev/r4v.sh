set -e
OUT=gpurun_out/r4v bash scripts/gpu.sh tests:tests/test_resnet_gpu.py resnet trace_resnet
echo done
