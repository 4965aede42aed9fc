#!/bin/bash
# Round-2 GPU check: the -m gpu suite (one process, per-test time limits), then one default bench run.
set -u
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc"
grep -E "PASSED|FAILED|ERROR|passed|failed|worst|diverged|probes" gpurun_out/gpu_tests.log | tail -60
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py ${BENCH_ARGS:-} > gpurun_out/bench.json 2> gpurun_out/bench.err
brc=$?
echo "bench rc=$brc"
tail -c 3000 gpurun_out/bench.json
exit $brc
