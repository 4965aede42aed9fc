#!/bin/bash
# Round 3: C3 A/B of the D waves' register copy of the hot constants (hotc) against the committed build,
# with C5 in the same lines.
export TMPDIR=/tmp
mkdir -p gpurun_out/r03m
BENCH_ARGS="--c5-steps 16384" timeout -k 10 500 bash tools/ab_libs.sh 3 build_diag/libsit_base.so build_diag/libsit_hotc.so \
  > gpurun_out/r03m/ab.log 2>&1
rc=$?; cat gpurun_out/r03m/ab.log
for f in gpurun_out/ab/libsit_*_[123].json; do python3 -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', 'C5 %.4e' % d['c5']['value'])"; done
exit $rc
