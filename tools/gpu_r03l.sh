#!/bin/bash
# Round 3: C3 A/B of P-wave reorderings (P0 lookups before outputs; rows deferred a step) against the
# committed build, then per-role sub-segment cycles of the committed build (C3 and policy mode).
export TMPDIR=/tmp
mkdir -p gpurun_out/r03l
BENCH_ARGS="--no-c5" timeout -k 10 400 bash tools/ab_libs.sh 3 build_diag/libsit_base.so build_diag/libsit_p0early.so \
  build_diag/libsit_pdefer.so > gpurun_out/r03l/ab.log 2>&1
rc=$?; cat gpurun_out/r03l/ab.log; [ $rc -eq 0 ] || exit $rc
tools/gpu_steps.sh \
 r03l/diag_c3 200 env SIT_LIBRARY=build_diag/libsit_diagsync.so python -u tools/diag_sync.py --- \
 r03l/diag_c5 200 env SIT_LIBRARY=build_diag/libsit_diagsync.so python -u tools/diag_sync.py --policy
