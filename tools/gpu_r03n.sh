#!/bin/bash
# Round 3: the IW-test cache carried across launches -- parity (launch-partition invariance, drop-in,
# debug variant, sync vs classic), then the single-step path, the drop-in latency and a C3 A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out/r03n
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_compat.py tests/test_gpu_debug.py \
  -k "partition or compat or reference or debug or sync_kernel or teacher_forced or state_roundtrip" -m gpu -v -s \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03n/tests.log 2>&1
rc=$?; grep -E "FAILED|ERROR|passed|failed|launch partition" gpurun_out/r03n/tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
tools/gpu_steps.sh \
 r03n/step 200 python -u bench.py --mode step --no-c5 --steps 2000 --warmup 200 --no-cpu-baseline --- \
 r03n/prof_step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03n/prof_step -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mode step --no-c5 --steps 2000 --warmup 200 --- \
 r03n/compat 300 python -u tools/compat_latency.py || exit $?
rm -f gpurun_out/r03n/prof_step/run_kernel_trace.csv
head -3 gpurun_out/r03n/prof_step/run_kernel_stats.csv | cut -c1-200
BENCH_ARGS="--no-c5" timeout -k 10 400 bash tools/ab_libs.sh 2 build_diag/libsit_base.so build_diag/libsit_iwc.so
