#!/bin/bash
# Round 3: the single-step path with the IW-test cache keyed by the IW point -- GPU suite, sit_step
# under rocprof, its per-role cycles, the drop-in latency, and a C3/C5 A/B against the committed build.
export TMPDIR=/tmp
mkdir -p gpurun_out/r03t
tools/gpu_steps.sh \
 r03t/tests 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider --- \
 r03t/prof_step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03t/prof_step -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mode step --no-c5 --steps 2000 --warmup 200 --- \
 r03t/diag_step 200 env SIT_LIBRARY=build_diag/libsit_diagsync.so python -u tools/diag_sync.py --step --- \
 r03t/compat 300 python -u tools/compat_latency.py || exit $?
rm -f gpurun_out/r03t/prof_step/run_kernel_trace.csv
tail -2 gpurun_out/r03t/tests.log
head -2 gpurun_out/r03t/prof_step/run_kernel_stats.csv | cut -c1-200
grep -o '"launch_ms": {[^}]*}' gpurun_out/r03t/prof_step.log
BENCH_ARGS="--c5-steps 16384" timeout -k 10 500 bash tools/ab_libs.sh 2 build_diag/libsit_base.so build_diag/libsit_cur.so
for f in gpurun_out/ab/libsit_*_[12].json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', 'C5 %.4e' % d['c5']['value'])"; done
