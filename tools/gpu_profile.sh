#!/bin/bash
# Round profile: rocprofv3 kernel-trace stats of the default bench (C3) and of the policy bench
# (C5), then the PMC passes of the step kernel (tools/pmc.sh; steady state), summarised on the
# box (raw traces are deleted: gpurun copies back at most 64 MiB).
export TMPDIR=/tmp
R=${1:-r01}
tools/gpu_steps.sh \
 prof_c3 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --- \
 prof_c5 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mode policy --- \
 prof_step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_step -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mode step --- \
 pmc 900 bash tools/pmc.sh
rc=$?
python3 tools/pmc_summary.py gpurun_out/pmc k_env_steps 8 > gpurun_out/pmc_summary.json
python3 tools/make_profile_json.py gpurun_out/pmc_summary.json gpurun_out/${R}_pmc_f32_rollout.json \
  --steps-per-launch 40000 --round ${R#r} --source "rocprofv3 --kernel-trace --pmc, tools/pmc.sh (5 passes) on the default bench.py (chunk 40000; the 3 timed launches averaged per pass, the 8 warm-up launches skipped)"
rm -f gpurun_out/prof_*/run_kernel_trace.csv
find gpurun_out/pmc -name "*.csv" -size +1M -delete
du -sh gpurun_out
exit $rc
