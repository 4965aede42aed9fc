#!/bin/bash
# Round 3: (1) the matrix-core actor: policy/actor tests (in-tree lib), standalone actor timing, C5 A/B;
# (2) barrier A as one-sided LDS step counters (build_diag/libsit_flags.so): parity subset, C3/C5 A/B.
export TMPDIR=/tmp
mkdir -p gpurun_out/r03v
timeout -k 10 600 python -u -m pytest tests/test_gpu_policy.py -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r03v/tests_actor.log 2>&1
rc=$?; tail -3 gpurun_out/r03v/tests_actor.log; [ $rc -eq 0 ] || exit $rc
for lib in build_diag/libsit_valuactor.so build_diag/libsit_cur.so; do
  SIT_LIBRARY=$lib timeout -k 10 120 python -u tools/actor_bench.py > gpurun_out/r03v/actor_$(basename $lib .so).log 2>&1 || exit $?
  echo "== $lib"; grep rows gpurun_out/r03v/actor_$(basename $lib .so).log
done
SIT_LIBRARY=build_diag/libsit_flags.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_policy.py \
  -k "sync_kernel or partition or synthetic or f32_policy or two_shards or free_running or teacher_forced or c5" -m gpu -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03v/tests_flags.log 2>&1
rc=$?; tail -3 gpurun_out/r03v/tests_flags.log; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--c5-steps 16384" timeout -k 10 600 bash tools/ab_libs.sh 2 build_diag/libsit_base.so build_diag/libsit_flags.so \
  build_diag/libsit_valuactor.so build_diag/libsit_cur.so
for f in gpurun_out/ab/libsit_*_[12].json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', 'C5 %.4e' % d['c5']['value'])"; done
