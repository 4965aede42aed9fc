#!/bin/bash
# C5 stream groups with in-kernel serving (graph launches, every output written, transitions gathered):
# one group of 32 768 envs against two of 16 384 on their own streams, at a few launch lengths
set -u
O=${1:-gpurun_out/c5g}
mkdir -p $O
for GK in 1:64 2:64 2:32 2:128 1:64; do
  G=${GK%%:*}; K=${GK##*:}
  timeout -k 10 150 python bench.py --mode policy --chunk $K --groups $G --steps 8192 --warmup 30720 --no-cpu-baseline \
    > $O/g${G}k$K.json 2> $O/g${G}k$K.err || { echo "G=$G K=$K failed"; exit 1; }
  python -c "
import json; d=json.loads(open('$O/g${G}k$K.json').read().strip().splitlines()[-1])
print('G=$G K=$K', '%.4e' % d['value'], 'frac %.3f' % d['config']['env_step_fraction'], 'launch ms %.3f' % d['roofline']['launch_ms']['median'])"
done
