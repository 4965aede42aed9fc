#!/bin/bash
# Round 3 record run of the current build: smoke, the default bench line (C3 + C5, CPU baseline),
# rocprofv3 kernel stats of it and of the single-step path, the PMC passes of the C3 kernel.
export TMPDIR=/tmp
mkdir -p gpurun_out/r03f2
tools/gpu_steps.sh \
 r03f2/smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" --- \
 r03f2/bench 400 python -u bench.py --- \
 r03f2/prof_c3 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03f2/prof_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --- \
 r03f2/prof_step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03f2/prof_step -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mode step --no-c5 --steps 2000 --warmup 200 --- \
 r03f2/pmc 900 bash tools/pmc.sh --no-c5
rc=$?
python3 tools/pmc_summary.py gpurun_out/pmc k_env_steps_sync 8 > gpurun_out/r03f2/pmc_summary.json
find gpurun_out/pmc -name "*.csv" -size +1M -delete
rm -f gpurun_out/r03f2/prof_*/run_kernel_trace.csv
exit $rc
