#!/bin/bash
# C5 (policy mode, fused actor) profile: kernel-trace stats, then the PMC passes of the env-step
# kernel in that configuration (per group launch: 16384 envs x 32 steps), summarised on the box.
export TMPDIR=/tmp
R=${1:-r02}
tools/gpu_steps.sh \
 prof_c5 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mode policy --- \
 pmc 900 bash tools/pmc.sh --mode policy
rc=$?
mv gpurun_out/pmc gpurun_out/pmc_c5
python3 tools/pmc_summary.py gpurun_out/pmc_c5 k_env_steps > gpurun_out/pmc_summary_c5.json
python3 tools/make_profile_json.py gpurun_out/pmc_summary_c5.json gpurun_out/${R}_pmc_f32_policy.json \
  --steps-per-launch 32 --n-env 16384 --mode policy --round ${R#r} \
  --source "rocprofv3 --kernel-trace --pmc, tools/pmc.sh --mode policy (5 passes; HIP-graph replays, 2 stream groups)"
python3 tools/pmc_summary.py gpurun_out/pmc_c5 k_policy_actor > gpurun_out/pmc_summary_actor.json
rm -f gpurun_out/prof_*/run_kernel_trace.csv
find gpurun_out/pmc_c5 -name "*.csv" -size +1M -delete
du -sh gpurun_out
exit $rc
