#!/bin/bash
# C5 quick check: fused-actor tests, then kernel-trace stats of the policy-mode bench.
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_policy.py -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/c5_tests.log 2>&1
rc=$?
tail -3 gpurun_out/c5_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5q -o run --output-format csv -- python3 bench.py --no-cpu-baseline --mode policy "$@" > gpurun_out/c5q.log 2>&1
rc=$?
grep '^{' gpurun_out/c5q.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['kernel_ms_per_launch'], d['config']['env_step_fraction'])"
cut -d, -f1-5 gpurun_out/prof_c5q/run_kernel_stats.csv | cut -c1-160 | head -6
rm -f gpurun_out/prof_c5q/run_kernel_trace.csv
exit $rc
