#!/bin/bash
# One parameterised GPU job runner (run on the box through gpurun, from the repo root):
#
#   OUT=gpurun_out/x bash scripts/gpu.sh STEP [STEP ...]
#
# Every step runs under its own time limit and the job stops at the first failing step (no GPU
# work after a fault, an abort or a timeout).  Steps:
#   tests            pytest -m gpu (whole suite)           tests:FILE[,FILE]  a subset
#   bench            bench.py N=1 (driver shape)           bench_long  60 timed intervals
#   algos            bench.py per algorithm / ASHA variant over 48 intervals (best loss at 12/24/48)
#   random           bench.py --algo random (best-loss@budget at the same budget as ASHA)
#   timeline         bench.py with the GPU-event timeline (MOPT_GPU_TIMELINE=1)
#   streams          bench.py at MOPT_STREAMS=1,2
#   kbench           per-kernel MLP microbench             trace_bench  rocprofv3 kernel trace
#   kbench_ab        the microbench per kernel variant (env $ABVAR set to each of $VARIANTS)
#   kbench_rows      the microbench at 128 / 256 / 512 rows per step (multi-row-block kernels)
#   pmc_kbench       PMC passes of the MLP kernels (fetch/write/MFMA/LDS, one pass each)
#   pmc_attn         PMC passes of the attention microbench (busy / wait / MFMA, LDS / VALU)
#   pmc_resnet       HBM FETCH / WRITE passes of a short ResNet-20 run (scripts/dev/pmc_bytes.py)
#   pmc_gemm         PMC passes of the GEMM microbench ($SHAPES name prefix, $CFGS tile configs)
#   lm resnet hyper  bench_configs.py of one config        trace_lm trace_resnet trace_hyper
#   attn             attention fwd / bwd microbench (LM-125M shape)
#   gemm conv        pgemm / direct-conv microbenches      gemm32  f32-operand (K11) GEMM plans
#   c4copy           one config-5 member: slot <-> pool copies, packed C4 path, copy_member
#   decide           rank-0 decide cost at simulated W=1,8 (host CPU of the box)
#   rehearsal        bench.py --gpus 2 / 4 / 8 over gloo with ranks sharing the GPU
#   northstar_resnet config 3 search quality: TPE vs random, 224 trials, seeds $SEEDS (0 1 2)
#   smoke            __graft_entry__.smoke()
#   ab               interleaved A/B: for rep in 1..$REPS, for v in $AB_VALUES: run the steps of
#                    $AB_STEPS with $AB_VAR=v, outputs under $OUT/ab_<v>_<rep>/ (e.g. AB_VAR=
#                    MOPT_STREAMS AB_VALUES="3 4" AB_STEPS=bench REPS=5).  A value of the form
#                    lib:<dir> runs with MOPT_KERNEL_LIB=<dir>/libmopt_kernels.so instead (a
#                    variant library built on the CPU with ops/build.py build_variant)
#   repeat           the steps of $AB_STEPS $REPS times (run-to-run spread), $OUT/rep_<n>/
set -e
OUT=${OUT:-gpurun_out/job}
mkdir -p "$OUT"
ROOT=$(pwd)
T="timeout -k 10"
PYT="python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu"

prof() {   # prof NAME LIMIT -- cmd...: rocprofv3 kernel trace + stats (own run, no counters)
  local name=$1 lim=$2; shift 3
  (cd /tmp && export TMPDIR=/tmp && $T "$lim" rocprofv3 --kernel-trace --stats \
      --output-format csv -d "$ROOT/$OUT/$name" -o run -- "$@" > "$ROOT/$OUT/$name.log" 2>&1)
}
pmc() {    # pmc NAME COUNTERS...: one counter pass over the MLP kernel microbench
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --output-format csv \
      --pmc "$@" -d "$ROOT/$OUT/$name" -o run -- \
      python3 "$ROOT/scripts/kernel_bench.py" --iters 3 --momentum-dtype bf16 \
      > "$ROOT/$OUT/$name.log" 2>&1)
}

pmcg() {   # pmcg NAME COUNTERS...: one counter pass over the GEMM microbench ($SHAPES, $CFGS)
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --output-format csv \
      --pmc "$@" -d "$ROOT/$OUT/$name" -o run -- \
      python3 "$ROOT/scripts/gemm_bench.py" --iters 5 --no-torch --shapes "${SHAPES:-lm}" \
      --cfgs "${CFGS:-11,12}" > "$ROOT/$OUT/$name.log" 2>&1)
}

pmcr() {   # pmcr NAME COUNTERS...: one counter pass over a short ResNet-20 population run
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 240 rocprofv3 --output-format csv \
      --pmc "$@" -d "$ROOT/$OUT/$name" -o run -- \
      python3 "$ROOT/scripts/bench_configs.py" --config resnet20 --sync-every 4 --steps 4 \
      --warmup 4 > "$ROOT/$OUT/$name.log" 2>&1)
}

pmca() {   # pmca NAME COUNTERS...: one counter pass over the attention microbench
  local name=$1; shift
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 150 rocprofv3 --output-format csv \
      --pmc "$@" -d "$ROOT/$OUT/$name" -o run -- \
      python3 "$ROOT/scripts/attn_bench.py" --iters 3 > "$ROOT/$OUT/$name.log" 2>&1)
}

for step in "$@"; do
  echo "[gpu.sh] $step"
  case "$step" in
    tests)      $T 600 $PYT tests > "$OUT/pytest_gpu.log" 2>&1 ;;
    tests:*)    $T 400 $PYT $(echo "${step#tests:}" | tr ',' ' ') > "$OUT/pytest_sub.log" 2>&1 ;;
    bench)      $T 240 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err" ;;
    bench_long) $T 240 python bench.py --steps 60 --warmup 5 > "$OUT/bench_long.json" 2> "$OUT/bench_long.err" ;;
    algos)      # best-loss@budget per search algorithm / ASHA variant (48 intervals each)
                for v in "random:--algo random" "bounded:--asha-mode bounded" "async:--asha-mode async" \
                         "async_eta2:--asha-mode async --fidelity 2,16,2" "async_g4:--asha-mode async --fidelity 4,16,4"; do
                  $T 240 python bench.py --steps 43 --warmup 5 ${v#*:} > "$OUT/algo_${v%%:*}.json" 2> "$OUT/algo_${v%%:*}.err"; done ;;
    random)     $T 240 python bench.py --steps 20 --warmup 5 --algo random > "$OUT/bench_random.json" 2> "$OUT/bench_random.err" ;;
    timeline)   MOPT_GPU_TIMELINE=1 $T 240 python bench.py --steps 20 --warmup 5 $BENCH_ARGS > "$OUT/bench_timeline$TAG.json" 2> "$OUT/bench_timeline$TAG.err" ;;
    streams)    for s in ${STREAM_SET:-1 2}; do MOPT_STREAMS=$s $T 240 python bench.py --steps 20 --warmup 5 > "$OUT/bench_streams$s.json" 2> "$OUT/bench_streams$s.err"; done ;;
    kbench)     $T 200 python scripts/kernel_bench.py --momentum-dtype bf16 --out "$OUT/kbench.json" > "$OUT/kbench.log" 2>&1 ;;
    kbench_ab)  for v in ${VARIANTS:-0 1}; do env ${ABVAR:-MOPT_AB}=$v $T 200 python scripts/kernel_bench.py --momentum-dtype bf16 --out "$OUT/kbench_v$v.json" > "$OUT/kbench_v$v.log" 2>&1; done ;;
    kbench_rows) for b in 128 256 512; do $T 200 python scripts/kernel_bench.py --momentum-dtype bf16 --batch $b --iters 20 --out "$OUT/kbench_b$b.json" > "$OUT/kbench_b$b.log" 2>&1; done ;;
    trace_bench) prof trace_bench$TAG 300 -- python3 "$ROOT/bench.py" --steps 10 --warmup 3 $BENCH_ARGS ;;
    pmc_kbench)
      pmc pmc_fetch FETCH_SIZE
      pmc pmc_write WRITE_SIZE
      pmc pmc_mfma SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES
      pmc pmc_lds SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES ;;
    pmc_gemm)   # PMC passes of the GEMM microbench (SHAPES prefix, CFGS tiles)
      pmcg pmcg_busy SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
      pmcg pmcg_lds SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES
      pmcg pmcg_fetch FETCH_SIZE ;;
    pmc_resnet) # HBM bytes per ResNet-20 kernel (scripts/dev/pmc_bytes.py reads the two passes)
      pmcr pmc_fetch FETCH_SIZE
      pmcr pmc_write WRITE_SIZE ;;
    pmc_resnet_busy) # issue / wait / LDS counters per ResNet-20 kernel (scripts/pmc_table.py)
      pmcr pmcr_busy SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
      pmcr pmcr_lds SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES ;;
    pmc_attn)   # PMC passes of the attention kernels
      pmca pmca_busy SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
      pmca pmca_lds SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES ;;
    lm)         $T 300 python scripts/bench_configs.py --config lm-125m --steps 600 --warmup 0 > "$OUT/lm.json" 2> "$OUT/lm.err" ;;
    resnet)     $T 300 python scripts/bench_configs.py --config resnet20 --steps 60 --warmup 30 > "$OUT/resnet20.json" 2> "$OUT/resnet20.err" ;;
    hyper)      $T 300 python scripts/bench_configs.py --config hyper --steps 3 --warmup 1 > "$OUT/hyper.json" 2> "$OUT/hyper.err" ;;
    trace_lm)   prof trace_lm 300 -- python3 "$ROOT/scripts/bench_configs.py" --config lm-125m --sync-every 2 --steps 6 --warmup 4 ;;
    trace_resnet) prof trace_resnet 300 -- python3 "$ROOT/scripts/bench_configs.py" --config resnet20 --sync-every 10 --steps 20 --warmup 10 ;;
    trace_hyper) prof trace_hyper 300 -- python3 "$ROOT/scripts/bench_configs.py" --config hyper --steps 1 --warmup 1 ;;
    attn)       $T 200 python scripts/attn_bench.py --out "$OUT/attn.json" > "$OUT/attn.log" 2>&1 ;;
    gemm)       $T 300 python scripts/gemm_bench.py --cfgs "${CFGS:-0,5,6,7}" --splits "${SPLITS:-}" --out "$OUT/gemm.json" > "$OUT/gemm.log" 2>&1 ;;
    gemm32)     $T 300 python scripts/gemm_f32_bench.py --out "$OUT/gemm32.json" > "$OUT/gemm32.log" 2>&1 ;;
    conv)       $T 200 python scripts/conv_bench.py --implicit --out "$OUT/conv_bench.json" > "$OUT/conv_bench.log" 2>&1 ;;
    c4copy)     $T 200 python scripts/c4_copy_bench.py --out "$OUT/c4_copy.json" > "$OUT/c4_copy.log" 2>&1 ;;
    decide)     for w in 1 8; do WORLD=$w $T 300 python scripts/profile_decide.py > "$OUT/decide_world$w.log" 2>&1; done ;;
    rehearsal)  for n in 2 4 8; do $T 400 python bench.py --gpus $n --steps 10 --warmup 3 --population 64 > "$OUT/rehearsal_n$n.json" 2> "$OUT/rehearsal_n$n.err"; done ;;
    northstar_resnet)   # config 3: TPE vs random search, 3120 steps (224 trials) x seeds 0-2
                for sd in ${SEEDS:-0 1 2}; do
                  $T 200 python scripts/bench_configs.py --config resnet20 --steps 3120 --warmup 0 --seed $sd > "$OUT/resnet_tpe_s$sd.json" 2> "$OUT/resnet_tpe_s$sd.err"
                  $T 200 python scripts/bench_configs.py --config resnet20 --steps 3120 --warmup 0 --seed $sd --algo random > "$OUT/resnet_random_s$sd.json" 2> "$OUT/resnet_random_s$sd.err"
                done ;;
    smoke)      $T 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 ;;
    ab)         for rep in $(seq 1 "${REPS:-3}"); do
                  for v in ${AB_VALUES:?AB_VALUES}; do
                    if [ "${v#lib:}" != "$v" ]; then envset="MOPT_KERNEL_LIB=${v#lib:}/libmopt_kernels.so"; tag=$(basename "${v#lib:}")
                    else envset="${AB_VAR:?AB_VAR}=$v"; tag=$v; fi
                    env $envset OUT="$OUT/ab_${tag}_$rep" bash "$0" ${AB_STEPS:?AB_STEPS}
                  done
                done ;;
    repeat)     for rep in $(seq 1 "${REPS:-3}"); do OUT="$OUT/rep_$rep" bash "$0" ${AB_STEPS:?AB_STEPS}; done ;;
    *) echo "unknown step $step" >&2; exit 2 ;;
  esac
done
echo "[gpu.sh] done"
