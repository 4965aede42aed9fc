#!/bin/bash
# C5 chunk sweep (graph launches, every output written, transitions gathered)
set -u
mkdir -p gpurun_out/c5k
for K in 32 64 128 256; do
  timeout -k 10 150 python bench.py --mode policy --chunk $K --groups 1 --steps 8192 --warmup 30720 --no-cpu-baseline > gpurun_out/c5k/k$K.json 2> gpurun_out/c5k/k$K.err || { echo "K=$K failed"; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/c5k/k$K.json').read().strip().splitlines()[-1])
print('K=$K', '%.4e' % d['value'], 'frac %.3f' % d['config']['env_step_fraction'], 'launch ms %.1f' % d['roofline']['launch_ms']['median'])"
done
