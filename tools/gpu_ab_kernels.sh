#!/bin/bash
# Selected GPU tests (one process), then the default bench with each step kernel (sync = the default
# two-wave kernel, classic = k_env_steps, pipelined = the speculative split):   [K=<pytest -k expr>] tools/gpu_ab_kernels.sh "<test paths>" [bench args]
set -u
mkdir -p gpurun_out
T=${1:-tests}
shift
timeout -k 10 600 python -u -m pytest $T ${K:+-k "$K"} -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/ab_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|pipelined vs|assert" gpurun_out/ab_tests.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then exit $rc; fi
for kern in sync classic pipelined; do
  export SIT_STEP_KERNEL=$kern
  timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/ab_$kern.json 2> gpurun_out/ab_$kern.err
  brc=$?
  echo "bench $kern rc=$brc"
  if [ $brc -ne 0 ]; then tail -5 gpurun_out/ab_$kern.err; exit $brc; fi
  python3 -c "import json;d=json.load(open('gpurun_out/ab_$kern.json'));print('$kern', d['value'], d['roofline']['kernel_ms_per_launch'], d['roofline']['launch_ms'])"
done
