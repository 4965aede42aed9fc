#!/bin/bash
# Round 3: the sync kernel with the position predicates on the P waves -- parity first, then an
# interleaved A/B against the previous build (build_diag/libsit_base.so) on the default bench (C3)
# and C5 (one group, 64 steps per launch).
set -u
mkdir -p gpurun_out/r03
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_policy.py tests/test_gpu_compat.py \
  -k "${K:-sync_kernel or synthetic or policy or compat or reference or two_shards or transitions or done_count}" \
  -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/tests_c.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "FAILED|ERROR|passed|failed|Error" gpurun_out/r03/tests_c.log | tail -20
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for lib in build_diag/libsit_base.so sac_maritime_ast_amd/libsit.so; do
    n=$(basename $(dirname $lib))_$(basename $lib .so)
    SIT_LIBRARY=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --c5-steps 16384 \
      > gpurun_out/r03/ab_${n}_$r.json 2> gpurun_out/r03/ab_${n}_$r.err || { echo "$n failed"; tail -3 gpurun_out/r03/ab_${n}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/r03/ab_${n}_$r.json'))
print('%-34s r$r C3 %.4e  launch %.3f ms   C5 %.4e' % ('$n', d['value'], d['roofline']['launch_ms']['median'], d['c5']['value']))"
  done
done
