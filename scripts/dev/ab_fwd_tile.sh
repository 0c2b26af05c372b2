# A/B of the hidden-layer forward tile width (MOPT_FWD_TN 64 / 32 / 128), one box; TN=128 needs
# widths that pad to multiples of 128, so the fixed-width runs compare all three at width 512
set -e
mkdir -p gpurun_out/ab3
K="timeout -k 10 200 python scripts/kernel_bench.py --momentum-dtype bf16 --iters 30"
for w in 512 1024; do
  for tn in 64 128 32; do
    MOPT_FWD_TN=$tn $K --width $w > gpurun_out/ab3/w${w}_tn$tn.log 2>&1
  done
done
