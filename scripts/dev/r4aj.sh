set -e
OUT=gpurun_out/r4aj
mkdir -p $OUT
# 8 gloo ranks sharing the one GPU, 128 trials each (1024 slots: staggered start over 2 syncs)
timeout -k 10 500 python bench.py --gpus 8 --steps 8 --warmup 4 --population 128 > $OUT/rehearsal_n8_p128.json 2> $OUT/rehearsal_n8_p128.err
echo done
