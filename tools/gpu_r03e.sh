#!/bin/bash
# Round 3 record run of the max-ILP-scheduled float32 TU: GPU parity suite, smoke, the default bench
# line (C3 + C5, CPU baseline), rocprofv3 kernel stats of it and of the single-step path.
# PMC passes: tools/pmc.sh --no-c5 in a call of their own.
export TMPDIR=/tmp
mkdir -p gpurun_out/r03e
tools/gpu_steps.sh \
 r03e/tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread --- \
 r03e/smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" --- \
 r03e/bench 400 python -u bench.py --- \
 r03e/prof_c3 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03e/prof_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --- \
 r03e/prof_step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03e/prof_step -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mode step --no-c5 --steps 2000 --warmup 200
rc=$?
rm -f gpurun_out/r03e/prof_*/run_kernel_trace.csv
exit $rc
