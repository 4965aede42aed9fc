#!/bin/bash
# Quick GPU check: selected test files (one process, per-test limits), then one default bench run.
#   usage: [K=<pytest -k expr>] tools/gpu_quick.sh "<test paths>" [bench args]
set -u
mkdir -p gpurun_out
T=${1:-tests}
shift
timeout -k 10 600 python -u -m pytest $T ${K:+-k "$K"} -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/quick_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/quick_tests.log | tail -40
if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then exit $rc; fi
timeout -k 10 300 python -u bench.py --no-cpu-baseline "$@" > gpurun_out/quick_bench.json 2> gpurun_out/quick_bench.err
brc=$?
echo "bench rc=$brc"
python3 -c "import json;d=json.load(open('gpurun_out/quick_bench.json'));print(d['value'], d['roofline']['kernel_ms_per_launch'], d['roofline']['launch_ms'])"
exit $brc
