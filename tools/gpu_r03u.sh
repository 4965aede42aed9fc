#!/bin/bash
# Round 3: the matrix-core actor (k_policy_actor_mfma) -- policy/actor parity tests, standalone actor
# timing of both kernels, and a C5 A/B (MFMA actor vs the VALU actor).
export TMPDIR=/tmp
mkdir -p gpurun_out/r03u
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py -m gpu -v --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r03u/tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|passed|failed|Error" gpurun_out/r03u/tests.log | tail -20; [ $rc -eq 0 ] || exit $rc
for lib in build_diag/libsit_valuactor.so build_diag/libsit_cur.so; do
  SIT_LIBRARY=$lib timeout -k 10 120 python -u tools/actor_bench.py > gpurun_out/r03u/actor_$(basename $lib .so).log 2>&1 || exit $?
  echo "== $lib"; cat gpurun_out/r03u/actor_$(basename $lib .so).log | grep rows
done
BENCH_ARGS="--mode policy --steps 16384 --warmup 30720 --chunk 64 --groups 1" timeout -k 10 500 bash tools/ab_libs.sh 2 build_diag/libsit_valuactor.so build_diag/libsit_cur.so
