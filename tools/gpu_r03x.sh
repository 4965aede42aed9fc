#!/bin/bash
# Round 3: wave placement -- roles mirrored by blockIdx / 256 (place8) and roles by SIMD with a per-CU
# ticket (placert); C3/C5 A/B against the current build; parity subset on the runtime placement.
export TMPDIR=/tmp
mkdir -p gpurun_out/r03x
for v in place8 placert; do
  SIT_LIBRARY=build_diag/libsit_$v.so timeout -k 10 200 python -u tools/diag_place.py > gpurun_out/r03x/$v.json 2>&1 || exit $?
  echo "== $v"; grep -A4 roles_per_simd gpurun_out/r03x/$v.json
done
BENCH_ARGS="--c5-steps 16384" timeout -k 10 700 bash tools/ab_libs.sh 2 build_diag/libsit_cur.so build_diag/libsit_mirror8.so build_diag/libsit_rt.so
for f in gpurun_out/ab/libsit_*_[12].json; do python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', 'C5 %.4e' % d['c5']['value'])"; done
SIT_LIBRARY=build_diag/libsit_rt.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_policy.py \
  -k "sync_kernel or partition or synthetic or two_shards or c4_last" -m gpu -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r03x/tests_rt.log 2>&1
rc=$?; tail -3 gpurun_out/r03x/tests_rt.log; exit $rc
