#!/bin/bash
# Occupancy experiment: libraries x n_env (C3 = 32768; 65536 = two waves per SIMD when the map is
# shared by the block's groups).   usage: tools/occ.sh "<n_env list>" <lib1> <lib2> ...
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/occ
ns=$1; shift
for n in $ns; do
  for lib in "$@"; do
    b=$(basename $lib .so)
    SIT_LIBRARY=$lib timeout -k 10 150 python bench.py --no-cpu-baseline --n-env $n --chunk 10000 --warmup 40000 \
      --steps 30000 > gpurun_out/occ/${b}_$n.json 2> gpurun_out/occ/${b}_$n.err || { echo "$b $n failed"; tail -3 gpurun_out/occ/${b}_$n.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/occ/${b}_$n.json').read().strip().splitlines()[-1])
print('%-14s n_env %6d  %.4e env-steps/s  median launch %.3f ms' % ('$b', $n, d['value'], d['roofline']['launch_ms']['median']))"
  done
done
