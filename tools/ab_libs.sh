#!/bin/bash
# Interleaved A/B of library builds on the default bench (C3): tools/ab_libs.sh <rounds> <lib1> <lib2> ...
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
rounds=$1; shift
for r in $(seq 1 $rounds); do
  for lib in "$@"; do
    n=$(basename $lib .so)
    SIT_LIBRARY=$lib timeout -k 10 150 python bench.py --no-cpu-baseline --no-extra-lines ${BENCH_ARGS:-} \
      > gpurun_out/ab/${n}_$r.json 2> gpurun_out/ab/${n}_$r.err || { echo "$n failed"; tail -3 gpurun_out/ab/${n}_$r.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/ab/${n}_$r.json').read().strip().splitlines()[-1])
c5 = d.get('c5', {}).get('value')
print('%-22s r%d %.4e env-steps/s  median launch %.3f ms  c5 %s' % ('$n', $r, d['value'], d['roofline']['launch_ms']['median'], '%.4e' % c5 if c5 else '-'))"
  done
done
