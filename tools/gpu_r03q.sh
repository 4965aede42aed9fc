#!/bin/bash
# Round 3: the build with explicit actions on the two-wave kernel (no IW-cache field) -- the full GPU
# suite, the single-step path under rocprof, and a C3/C5 A/B against the committed build.
export TMPDIR=/tmp
mkdir -p gpurun_out/r03q
tools/gpu_steps.sh \
 r03q/tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider --- \
 r03q/prof_step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03q/prof_step -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mode step --no-c5 --steps 2000 --warmup 200 || exit $?
rm -f gpurun_out/r03q/prof_step/run_kernel_trace.csv
tail -2 gpurun_out/r03q/tests.log
head -2 gpurun_out/r03q/prof_step/run_kernel_stats.csv | cut -c1-200
BENCH_ARGS="--c5-steps 16384" timeout -k 10 500 bash tools/ab_libs.sh 2 build_diag/libsit_base.so build_diag/libsit_cur.so
for f in gpurun_out/ab/libsit_*_[12].json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', 'C5 %.4e' % d['c5']['value'])"; done
