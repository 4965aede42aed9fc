#!/bin/bash
# Record run of the current build (the supported profiling recipe):
#   smoke, the default bench line (C3 + C5 + CPU baseline), rocprofv3 kernel stats of the default
#   bench and of the single-step path, the PMC passes (tools/pmc.sh) of the C3 kernel and of the C5
#   policy kernel, summarised into profiles-ready JSON under gpurun_out/<tag>/.
#   usage (on the GPU box, via gpurun): tools/gpu_record.sh <tag>
set -u
export TMPDIR=/tmp
T=${1:-rec}
O=gpurun_out/$T
C5="--mode policy --chunk 64 --groups 1 --steps 8192 --warmup 16384"
tools/gpu_steps.sh \
 $T/smoke 200 python3 -u -c "import __graft_entry__ as g; g.smoke()" --- \
 $T/bench 400 python3 -u bench.py --- \
 $T/prof_c3 400 rocprofv3 --kernel-trace --stats -d $O/prof_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-extra-lines --- \
 $T/prof_step 300 rocprofv3 --kernel-trace --stats -d $O/prof_step -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mode step --no-c5 --steps 2000 --warmup 200 --- \
 $T/pmc_c3 900 bash tools/pmc.sh $O/pmc_c3 --no-c5 --- \
 $T/pmc_c5 900 bash tools/pmc.sh $O/pmc_c5 $C5
rc=$?
python3 tools/pmc_summary.py $O/pmc_c3 k_env_steps_sync 8 > $O/pmc_summary_c3.json
python3 tools/make_profile_json.py $O/pmc_summary_c3.json $O/pmc_f32_rollout.json --steps-per-launch 40000 \
  --n-env 32768 --mode rollout --round 5 --source "rocprofv3 --kernel-trace --pmc, tools/pmc.sh --no-c5 (5 passes)"
python3 tools/pmc_summary.py $O/pmc_c5 "k_env_steps_sync<float, 2" 8 > $O/pmc_summary_c5.json
python3 tools/make_profile_json.py $O/pmc_summary_c5.json $O/pmc_f32_policy.json --steps-per-launch 64 \
  --n-env 32768 --mode policy --round 5 --kernel "k_env_steps_sync<float, kPolicy> (sit_sync.h), in-kernel serving" \
  --source "rocprofv3 --kernel-trace --pmc, tools/pmc.sh $C5 (5 passes; HIP-graph replays, 1 stream group)"
python3 tools/pmc_summary.py $O/pmc_c5 k_policy_actor 8 > $O/pmc_summary_actor.json
python3 tools/pmc_summary.py $O/pmc_c5 k_policy_admit 8 > $O/pmc_summary_admit.json
find $O -name "*.csv" -size +1M -delete
rm -f $O/prof_*/run_kernel_trace.csv
exit $rc
