#!/bin/bash
# Round 3, second GPU check: drop-in tests, sync-vs-classic configs, compat latency, the sit_step path,
# and C5 launch-shape variants (stream groups, steps per launch).
set -u
mkdir -p gpurun_out/r03
timeout -k 10 900 python -u -m pytest tests/test_gpu_compat.py tests/test_gpu_parity.py -k "${K:-compat or reference or sync_kernel}" \
  -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r03/tests_b.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|sync vs" gpurun_out/r03/tests_b.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then exit $rc; fi
timeout -k 10 300 python -u tools/compat_latency.py > gpurun_out/r03/compat_latency.json 2> gpurun_out/r03/compat_latency.err || exit $?
cat gpurun_out/r03/compat_latency.json
timeout -k 10 200 python -u bench.py --mode step --steps 2000 --warmup 200 --no-cpu-baseline \
  > gpurun_out/r03/step_b.json 2> gpurun_out/r03/step_b.err || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/r03/step_b.json'))
print('step', d['value'], d['roofline']['kernel'], d['roofline']['launch_ms'])"
for cfg in "1 32" "2 32" "4 32" "1 64" "2 64"; do
  set -- $cfg
  timeout -k 10 200 python -u bench.py --mode policy --groups $1 --chunk $2 --steps 16384 --warmup 30000 --no-cpu-baseline \
    > gpurun_out/r03/c5_g$1_k$2.json 2> gpurun_out/r03/c5_g$1_k$2.err || exit $?
  python3 -c "
import json;d=json.load(open('gpurun_out/r03/c5_g$1_k$2.json'))
print('C5 groups $1 chunk $2', '%.4e' % d['value'], d['config']['env_step_fraction'], d['roofline']['launch_ms'])"
done
