#!/bin/bash
# Round-6 record of the current build (on the GPU box, via gpurun), in two calls:
#   tools/gpu_record6.sh <tag> a   smoke, the GPU suite (records: drift, trig, knife edges), the default bench
#                                  line (every line), rocprofv3 --kernel-trace --stats of each bench line's own launch
#                                  shape (C3, C5, float64 C3, PyTorch-actor C5), timed-launch averages from the traces
#   tools/gpu_record6.sh <tag> b   the PMC passes (tools/pmc.sh) of the four step kernels at the same shapes, as
#                                  profiles-ready JSON, then tools/roofline_sources.py over call a's bench and profiles
set -u
export TMPDIR=/tmp
T=${1:-r06rec}
P=${2:-a}
O=gpurun_out/$T
mkdir -p $O
C3="--no-cpu-baseline --no-extra-lines --no-c5"
C5="--no-cpu-baseline --mode policy --chunk 80 --groups 1 --steps 8192 --warmup 30720"
F64="--no-cpu-baseline --no-extra-lines --no-c5 --precision 64 --chunk 10000 --steps 30000 --warmup 40000"
TORCH="--no-cpu-baseline --mode policy --serve queue --torch-actor --actor-stream --groups 1 --chunk 80 --steps 10240 --warmup 15360"
RP="rocprofv3 --kernel-trace --stats -o run --output-format csv"
case $P in
a)
  tools/gpu_steps.sh \
    $T/smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" --- \
    $T/tests 900 env SIT_TEST_RECORD_DIR=$O python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s --- \
    $T/bench 400 python3 -u bench.py || exit $?
  bash $0 $T p ;;
p)
  # rocprofv3 kernel stats + the step kernel's dispatches (timed-launch averages) of each line's launch shape
  tools/gpu_steps.sh \
    $T/prof_c3 300 $RP -d $O/prof_c3 -- python3 bench.py $C3 --- \
    $T/prof_c5 300 $RP -d $O/prof_c5 -- python3 bench.py $C5 --- \
    $T/prof_f64 300 $RP -d $O/prof_f64 -- python3 bench.py $F64 --- \
    $T/prof_torch 300 $RP -d $O/prof_torch -- python3 bench.py $TORCH
  rc=$?
  for n in c3 c5 f64 torch; do
    f=$O/prof_$n/run_kernel_trace.csv
    [ -f $f ] && python3 -c "
import csv, sys
rows = [r for r in csv.DictReader(open('$f')) if 'k_env_steps_sync' in r['Kernel_Name']]
w = csv.DictWriter(open('$O/prof_$n/step_kernel_trace.csv', 'w'), fieldnames=['Kernel_Name', 'Start_Timestamp', 'End_Timestamp'])
w.writeheader()
for r in rows: w.writerow({k: r[k] for k in ('Kernel_Name', 'Start_Timestamp', 'End_Timestamp')})"
  done
  [ -f $O/prof_torch/run_kernel_trace.csv ] && python3 tools/trace_breakdown.py $O/prof_torch/run_kernel_trace.csv \
    --tail-frac 0.4 > $O/torch_breakdown.json
  find $O -name "run_kernel_trace.csv" -delete
  exit $rc ;;
b)
  tools/gpu_steps.sh \
    $T/pmc_c3 600 bash tools/pmc.sh $O/pmc_c3 --no-c5 --- \
    $T/pmc_c5 600 bash tools/pmc.sh $O/pmc_c5 $C5 --- \
    $T/pmc_f64 600 bash tools/pmc.sh $O/pmc_f64 $F64 --- \
    $T/pmc_torch 600 bash tools/pmc.sh $O/pmc_torch $TORCH
  rc=$?
  python3 tools/pmc_summary.py $O/pmc_c3 "k_env_steps_sync<float, 1" 8 > $O/pmc_summary_c3.json
  python3 tools/make_profile_json.py $O/pmc_summary_c3.json $O/pmc_f32_rollout.json --steps-per-launch 40000 \
    --n-env 32768 --mode rollout --round 6 --kernel "k_env_steps_sync<float, kSynth> (sit_sync.h)" \
    --source "rocprofv3 --kernel-trace --pmc, tools/pmc.sh --no-c5 (5 passes)"
  python3 tools/pmc_summary.py $O/pmc_c5 "k_env_steps_sync<float, 2" 8 > $O/pmc_summary_c5.json
  python3 tools/make_profile_json.py $O/pmc_summary_c5.json $O/pmc_f32_policy.json --steps-per-launch 80 \
    --n-env 32768 --mode policy --serve kernel --round 6 --kernel "k_env_steps_sync<float, kPolicy> (sit_sync.h), in-kernel serving" \
    --source "rocprofv3 --kernel-trace --pmc, tools/pmc.sh $C5 (5 passes; HIP-graph replays, 1 stream group)"
  python3 tools/pmc_summary.py $O/pmc_f64 "k_env_steps_sync<double" 1 > $O/pmc_summary_f64.json
  python3 tools/make_profile_json.py $O/pmc_summary_f64.json $O/pmc_f64_rollout.json --steps-per-launch 10000 \
    --n-env 32768 --precision 64 --mode rollout --round 6 --kernel "k_env_steps_sync<double, kSynth> (sit_sync.h)" \
    --source "rocprofv3 --kernel-trace --pmc, tools/pmc.sh $F64 (5 passes)"
  python3 tools/pmc_summary.py $O/pmc_torch "k_env_steps_sync<float, 2" 8 > $O/pmc_summary_torch.json
  python3 tools/make_profile_json.py $O/pmc_summary_torch.json $O/pmc_f32_policy_queue.json --steps-per-launch 80 \
    --n-env 32768 --mode policy --serve queue --round 6 --kernel "k_env_steps_sync<float, kPolicy> (sit_sync.h), request queue" \
    --source "rocprofv3 --kernel-trace --pmc, tools/pmc.sh $TORCH (5 passes; HIP-graph replays, actor on its own stream)"
  find $O -name "*.csv" -size +1M -delete
  exit $rc ;;
esac
