#!/bin/bash
# Round-6 GPU calls (on the gpurun box): tools/gpu_round6.sh <tag> <phase>
#   a   first look: smoke; the new trig / fused-drift / partition / teacher-forced tests; the fused drift
#       of the variant without the PID error's low part; A/B of C3 against the round-5 library and of the
#       float64 C3 against the two-waves-per-SIMD float64 variant; rocprof of the float64 C3 and of the
#       PyTorch-actor C5 (kernel trace -> tools/trace_breakdown.py); the PyTorch-actor C5 launch shapes
#   pmc64   the PMC passes of the float64 C3 bench shape
#   pmctorch  the PMC passes of the PyTorch-actor C5 step kernel
set -u
export TMPDIR=/tmp
T=${1:-r06a}
P=${2:-a}
O=gpurun_out/$T
mkdir -p $O
F64="--precision 64 --chunk 10000 --steps 30000 --warmup 40000 --no-c5"
TORCH="--mode policy --serve queue --torch-actor --groups 2 --chunk 32 --steps 4096 --warmup 15360"
# the c5_torch_actor line since round 6 (one group, 64-step launches, the actor on its own stream)
TORCH1="--mode policy --serve queue --torch-actor --actor-stream --groups 1 --chunk 64 --steps 8192 --warmup 15360"
case $P in
a)
  tools/gpu_steps.sh \
    $T/smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" --- \
    $T/tests 600 env SIT_TEST_RECORD_DIR=$O python3 -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 \
      --timeout-method thread -s -k "fast_trig or benchmarked_kernel_state or launch_partition or f32_teacher_forced or ieee or transcendentals" --- \
    $T/drift_nopidlo 300 env SIT_LIBRARY=build_diag/libsit_nopidlo.so python3 tools/f32_drift.py --chunk 200 --out $O/drift_nopidlo.json --- \
    $T/ab_c3 600 bash tools/ab_libs.sh 2 sac_maritime_ast_amd/libsit.so build_diag/libsit_r05.so --- \
    $T/ab_f64 400 env BENCH_ARGS="$F64" bash tools/ab_libs.sh 2 sac_maritime_ast_amd/libsit.so build_diag/libsit_f64w2.so --- \
    $T/prof_f64 300 rocprofv3 --kernel-trace --stats -d $O/prof_f64 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra-lines $F64 --- \
    $T/prof_torch 300 rocprofv3 --kernel-trace --stats -d $O/prof_torch -o run --output-format csv -- python3 bench.py --no-cpu-baseline $TORCH
  rc=$?
  f=$(ls $O/prof_torch/*/run_kernel_trace.csv $O/prof_torch/run_kernel_trace.csv 2>/dev/null | head -1)
  [ -n "$f" ] && python3 tools/trace_breakdown.py $f > $O/torch_breakdown.json
  find $O -name "run_kernel_trace.csv" -delete
  exit $rc ;;
b)
  tools/gpu_steps.sh \
    $T/tests 600 env SIT_TEST_RECORD_DIR=$O python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compat.py -m gpu -v \
      --timeout 300 --timeout-method thread -s -k "fast_trig or benchmarked_kernel_state or float32_attribute" --- \
    $T/drift_nopidlo 300 env SIT_LIBRARY=build_diag/libsit_nopidlo.so python3 tools/f32_drift.py --chunk 200 --out $O/drift_nopidlo.json --- \
    $T/f64_16k 200 python3 bench.py --no-cpu-baseline --no-extra-lines $F64 --n-env 16384 --- \
    $T/f64_32k 200 python3 bench.py --no-cpu-baseline --no-extra-lines $F64 --- \
    $T/torch_sweep 900 bash tools/c5_torch_sweep.sh $O/c5t ;;
c)
  tools/gpu_steps.sh \
    $T/tests 900 env SIT_TEST_RECORD_DIR=$O python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compat.py -m gpu -v \
      --timeout 600 --timeout-method thread -s -k "fast_trig or free_running_within or float32_attribute or launch_partition" --- \
    $T/bench 300 python3 -u bench.py --- \
    $T/torch_sweep 600 bash tools/c5_torch_sweep.sh $O/c5t 1:64:3:1 1:64:6:1 1:64:8:1 1:80:4:1 1:64:4:1 ;;
d)
  tools/gpu_steps.sh \
    $T/drift_main 300 python3 tools/f32_drift.py --out $O/drift_main.json --- \
    $T/drift_alphacall 300 env SIT_LIBRARY=build_diag/libsit_alphacall.so python3 tools/f32_drift.py --out $O/drift_alphacall.json --- \
    $T/drift_noalpha 300 env SIT_LIBRARY=build_diag/libsit_noalpha.so python3 tools/f32_drift.py --out $O/drift_noalpha.json --- \
    $T/ab_c3 900 bash tools/ab_libs.sh 2 sac_maritime_ast_amd/libsit.so build_diag/libsit_alphacall.so build_diag/libsit_noalpha.so build_diag/libsit_prev.so --- \
    $T/prof_torch1 300 rocprofv3 --kernel-trace --stats -d $O/prof_torch1 -o run --output-format csv -- python3 bench.py --no-cpu-baseline $TORCH1
  rc=$?
  [ -f $O/prof_torch1/run_kernel_trace.csv ] && python3 tools/trace_breakdown.py $O/prof_torch1/run_kernel_trace.csv > $O/torch1_breakdown.json
  find $O -name "run_kernel_trace.csv" -delete
  exit $rc ;;
e)
  # C5 (in-kernel serving) launch length and the marginal cost of one serving round
  for K in 32 64 128; do
    timeout -k 10 200 python3 bench.py --mode policy --chunk $K --groups 1 --steps 8192 --warmup 30720 --no-cpu-baseline \
      > $O/c5_k$K.json 2> $O/c5_k$K.err || exit 1
  done
  SIT_LIBRARY=build_diag/libsit_serve2.so timeout -k 10 200 python3 bench.py --mode policy --chunk 64 --groups 1 --steps 8192 \
    --warmup 30720 --no-cpu-baseline > $O/c5_k64_serve2.json 2> $O/c5_k64_serve2.err || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5 -o run --output-format csv -- python3 bench.py --mode policy \
    --chunk 64 --groups 1 --steps 8192 --warmup 30720 --no-cpu-baseline > $O/prof_c5.log 2>&1 || exit 1
  SIT_LIBRARY=build_diag/libsit_serve2.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_c5_serve2 -o run \
    --output-format csv -- python3 bench.py --mode policy --chunk 64 --groups 1 --steps 8192 --warmup 30720 --no-cpu-baseline \
    > $O/prof_c5_serve2.log 2>&1 || exit 1
  rm -f $O/prof_*/run_kernel_trace.csv
  tools/gpu_steps.sh \
    $T/tests 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 300 --timeout-method thread \
      -k "launch_partition or equals_classic or f32_teacher_forced or synthetic_rollout or f32_rollout" --- \
    $T/ab_c3 900 bash tools/ab_libs.sh 3 sac_maritime_ast_amd/libsit.so build_diag/libsit_nodist.so || exit $?
  for f in $O/c5_k*.json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', '%.4e' % d['value'], 'frac %.3f' % d['config']['env_step_fraction'], 'launch ms %.4f' % d['roofline']['launch_ms']['median'])"; done ;;
f)
  tools/gpu_steps.sh \
    $T/tests 600 python3 -u -m pytest tests/test_gpu_policy.py tests/test_gpu_debug.py -m gpu -v --timeout 300 --timeout-method thread --- \
    $T/ab 900 bash tools/ab_libs.sh 3 sac_maritime_ast_amd/libsit.so build_diag/libsit_servefix.so ;;
g)
  # A/B of a variant against the main library (3 interleaved rounds), parity subset first
  V=${3:-noahead}
  tools/gpu_steps.sh \
    $T/tests 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sim.py -m gpu -v --timeout 300 --timeout-method thread \
      -k "launch_partition or equals_classic or f32_teacher_forced or synthetic_rollout or f32_rollout or free_running or knife or sim_" --- \
    $T/ab 900 bash tools/ab_libs.sh 3 sac_maritime_ast_amd/libsit.so build_diag/libsit_$V.so ;;
h)
  V=${3:-nocompvel}
  tools/gpu_steps.sh \
    $T/drift 300 python3 tools/f32_drift.py --out $O/drift_main.json --- \
    $T/drift_$V 300 env SIT_LIBRARY=build_diag/libsit_$V.so python3 tools/f32_drift.py --out $O/drift_$V.json --- \
    $T/tests 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sim.py tests/test_gpu_compat.py tests/test_gpu_policy.py \
      -m gpu -v --timeout 300 --timeout-method thread -x -k "not free_running_within" --- \
    $T/ab 900 bash tools/ab_libs.sh 3 sac_maritime_ast_amd/libsit.so build_diag/libsit_$V.so ;;
pmc64)
  tools/gpu_steps.sh $T/pmc_f64 900 bash tools/pmc.sh $O/pmc_f64 $F64
  rc=$?
  python3 tools/pmc_summary.py $O/pmc_f64 "k_env_steps_sync<double" 1 > $O/pmc_summary_f64.json
  python3 tools/make_profile_json.py $O/pmc_summary_f64.json $O/pmc_f64_rollout.json --steps-per-launch 10000 \
    --n-env 32768 --precision 64 --mode rollout --round 6 --kernel "k_env_steps_sync<double, kSynth> (sit_sync.h)" \
    --source "rocprofv3 --kernel-trace --pmc, tools/pmc.sh $F64 (5 passes)"
  find $O -name "*.csv" -size +1M -delete
  exit $rc ;;
pmctorch)
  tools/gpu_steps.sh $T/pmc_torch 900 bash tools/pmc.sh $O/pmc_torch $TORCH
  rc=$?
  python3 tools/pmc_summary.py $O/pmc_torch "k_env_steps_sync<float, 2" 8 > $O/pmc_summary_torch.json
  python3 tools/make_profile_json.py $O/pmc_summary_torch.json $O/pmc_f32_policy_torch.json --steps-per-launch 32 \
    --n-env 16384 --mode policy --round 6 --kernel "k_env_steps_sync<float, kPolicy> (sit_sync.h), request queue" \
    --source "rocprofv3 --kernel-trace --pmc, tools/pmc.sh $TORCH (5 passes; HIP-graph replays, 2 stream groups)"
  find $O -name "*.csv" -size +1M -delete
  exit $rc ;;
esac
