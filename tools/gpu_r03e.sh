#!/bin/bash
# Round 3: P1 assembles the outputs after barrier B -- parity, debug variant, C4 last shard, then an
# interleaved A/B against build_diag/libsit_base.so and the per-role segment cycles.
set -u
mkdir -p gpurun_out/r03
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_policy.py tests/test_gpu_compat.py tests/test_gpu_debug.py \
  -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/tests_e.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "FAILED|ERROR|passed|failed|Error|debug variant" gpurun_out/r03/tests_e.log | tail -20
if [ $rc -ne 0 ]; then exit $rc; fi
for r in 1 2; do
  for lib in build_diag/libsit_base.so sac_maritime_ast_amd/libsit.so; do
    n=$(basename $(dirname $lib))_$(basename $lib .so)
    SIT_LIBRARY=$lib timeout -k 10 200 python bench.py --no-cpu-baseline --c5-steps 16384 \
      > gpurun_out/r03/abe_${n}_$r.json 2> gpurun_out/r03/abe_${n}_$r.err || { echo "$n failed"; tail -3 gpurun_out/r03/abe_${n}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('gpurun_out/r03/abe_${n}_$r.json'))
print('%-34s r$r C3 %.4e  launch %.3f ms   C5 %.4e (%s)' % ('$n', d['value'], d['roofline']['launch_ms']['median'], d['c5']['value'], d['c5']['config']['env_step_fraction']))"
  done
done
SIT_LIBRARY=build_diag/libsit_diagsync.so timeout -k 10 200 python -u tools/diag_sync.py > gpurun_out/r03/diag_sync_e.json 2> gpurun_out/r03/diag_sync_e.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/r03/diag_sync_e.json'))
for r,v in d['roles'].items(): print('%-28s' % r, v)"
