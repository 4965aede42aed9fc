#!/bin/bash
# Round 3 record run of the current build: the full GPU suite, smoke, the default bench line (with
# the CPU baseline), rocprofv3 kernel stats of the default bench and of the step path, the drop-in
# latency and the float32 free-running drift report.  Each step has its own time limit
# (tools/gpu_steps.sh stops at the first fault / abort / timeout).
export TMPDIR=/tmp
mkdir -p gpurun_out/r03f
tools/gpu_steps.sh \
 r03f/tests 420 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --- \
 r03f/smoke 200 python -u -c "import __graft_entry__ as g; g.smoke()" --- \
 r03f/bench 400 python -u bench.py --- \
 r03f/prof_c3 400 rocprofv3 --kernel-trace --stats -d gpurun_out/r03f/prof_c3 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --- \
 r03f/prof_step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03f/prof_step -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mode step --no-c5 --steps 2000 --warmup 200 --- \
 r03f/compat 300 python -u tools/compat_latency.py --- \
 r03f/drift 400 python -u tools/f32_drift.py --out gpurun_out/r03f/f32_drift.json --- \
 r03f/diag_sync 200 env SIT_LIBRARY=build_diag/libsit_diagsync.so python -u tools/diag_sync.py
rc=$?
rm -f gpurun_out/r03f/prof_*/run_kernel_trace.csv
exit $rc
