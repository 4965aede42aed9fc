#!/bin/bash
# C5 launch-shape sweep: groups x chunk (one box)
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/c5sweep
for g in 1 2; do for c in 32 64 96 128; do
  timeout -k 10 120 python bench.py --mode policy --no-cpu-baseline --groups $g --chunk $c --steps 16384 --warmup 30720 > gpurun_out/c5sweep/g${g}_c${c}.json 2>/dev/null || { echo "g$g c$c failed"; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/c5sweep/g${g}_c${c}.json').read().strip().splitlines()[-1])
print('groups $g chunk $c: %.4e env-steps/s  fraction %.3f' % (d['value'], d['config']['env_step_fraction']))"
done; done
