#!/bin/bash
# Round 3: explicit inputs loaded a step ahead; the P after-B stores back inline -- the GPU suite subset,
# the single-step path, then a C3 A/B against the committed build.
export TMPDIR=/tmp
mkdir -p gpurun_out/r03p
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compat.py tests/test_gpu_sim.py \
  -k "partition or compat or reference or sync_kernel or teacher_forced or state_roundtrip or explicit or step" -m gpu -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03p/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r03p/tests.log; [ $rc -eq 0 ] || exit $rc
tools/gpu_steps.sh \
 r03p/prof_step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03p/prof_step -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mode step --no-c5 --steps 2000 --warmup 200 || exit $?
rm -f gpurun_out/r03p/prof_step/run_kernel_trace.csv
head -2 gpurun_out/r03p/prof_step/run_kernel_stats.csv | cut -c1-200
grep -o '"launch_ms": {[^}]*}' gpurun_out/r03p/prof_step.log
BENCH_ARGS="--no-c5" timeout -k 10 500 bash tools/ab_libs.sh 2 build_diag/libsit_base.so build_diag/libsit_noships.so \
  build_diag/libsit_noships_iwc.so build_diag/libsit_cur.so
