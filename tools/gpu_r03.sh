#!/bin/bash
# Round-3 GPU check: selected tests (one process, per-test limits), the default bench line (C3 + the
# C5 key), then the drop-in sit_step path with the map read through the caches (default at K = 1)
# and staged in LDS (SIT_LDS_MAP=1), for the A/B.
#   usage: [K=<pytest -k expr>] tools/gpu_r03.sh "<test paths>" [bench args]
set -u
mkdir -p gpurun_out/r03
T=${1:-tests}
shift
timeout -k 10 900 python -u -m pytest $T ${K:+-k "$K"} -m gpu -v -s --timeout 300 --timeout-method thread \
  -p no:cacheprovider > gpurun_out/r03/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|worst|sync vs" gpurun_out/r03/tests.log | tail -60
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/r03/bench.json 2> gpurun_out/r03/bench.err
brc=$?
echo "bench rc=$brc"
[ $brc -eq 0 ] || exit $brc
python3 -c "
import json;d=json.load(open('gpurun_out/r03/bench.json'))
print('C3', d['value'], d['roofline']['kernel'], d['roofline']['kernel_ms_per_launch'], d['roofline']['frac'])
c=d.get('c5')
if c: print('C5', c['value'], c['roofline']['kernel'], c['config']['env_step_fraction'], c['roofline']['launch_ms'])
"
for lm in auto 1; do
  if [ $lm = auto ]; then unset SIT_LDS_MAP; else export SIT_LDS_MAP=$lm; fi
  timeout -k 10 200 python -u bench.py --mode step --steps 2000 --warmup 200 --no-cpu-baseline \
    > gpurun_out/r03/step_$lm.json 2> gpurun_out/r03/step_$lm.err || exit $?
  python3 -c "
import json;d=json.load(open('gpurun_out/r03/step_$lm.json'))
print('step lds=$lm', d['value'], d['roofline']['kernel'], d['roofline']['launch_ms'])
"
done
unset SIT_LDS_MAP
