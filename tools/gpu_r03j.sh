#!/bin/bash
# Round 3: C3 A/B of the next-heading trig carried (spec) and the split dynamics (split) against the
# previous build, then the sync-kernel parity tests on the split build.
export TMPDIR=/tmp
mkdir -p gpurun_out/r03j
BENCH_ARGS="--no-c5" timeout -k 10 400 bash tools/ab_libs.sh 3 build_diag/libsit_base.so build_diag/libsit_spec.so \
  build_diag/libsit_split.so > gpurun_out/r03j/ab.log 2>&1
rc=$?; cat gpurun_out/r03j/ab.log; [ $rc -eq 0 ] || exit $rc
SIT_LIBRARY=build_diag/libsit_split.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_policy.py \
  -k "sync_kernel or synthetic or f32_policy or two_shards or free_running" -m gpu -v -s --timeout 300 \
  --timeout-method thread -p no:cacheprovider > gpurun_out/r03j/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|f32 vs f64|sync vs" gpurun_out/r03j/tests.log | tail -40; exit $rc
