#!/bin/bash
# Round 3: explicit actions (sit_step / the drop-in) on the two-wave kernel -- the full GPU suite, the
# single-step path and drop-in latency, then a C3 A/B (IW cache off, P constants from LDS).
export TMPDIR=/tmp
mkdir -p gpurun_out/r03o
tools/gpu_steps.sh \
 r03o/tests 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider --- \
 r03o/step 200 python -u bench.py --mode step --no-c5 --steps 2000 --warmup 200 --no-cpu-baseline --- \
 r03o/prof_step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03o/prof_step -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mode step --no-c5 --steps 2000 --warmup 200 --- \
 r03o/compat 300 python -u tools/compat_latency.py || exit $?
rm -f gpurun_out/r03o/prof_step/run_kernel_trace.csv
grep -E "passed|failed" gpurun_out/r03o/tests.log | tail -2
head -3 gpurun_out/r03o/prof_step/run_kernel_stats.csv | cut -c1-200
BENCH_ARGS="--no-c5" timeout -k 10 500 bash tools/ab_libs.sh 2 build_diag/libsit_base.so build_diag/libsit_cur.so \
  build_diag/libsit_iwc0.so build_diag/libsit_pcref.so
