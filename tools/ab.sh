#!/bin/bash
# A/B steady-state timing of library builds: tools/ab.sh <lib1> <lib2> ...  (default libsit.so first)
export TMPDIR=/tmp
args=()
for lib in "$@"; do
  n=$(basename $lib .so)
  args+=("$n" 120 env SIT_LIBRARY=$lib python bench.py --no-cpu-baseline --warmup 40000 --steps 20000 --chunk 200 "---")
  args+=("${n}_c5000" 120 env SIT_LIBRARY=$lib python bench.py --no-cpu-baseline --warmup 40000 --steps 20000 --chunk 5000 "---")
done
tools/gpu_steps.sh "${args[@]}"
for lib in "$@"; do
  n=$(basename $lib .so)
  for f in $n ${n}_c5000; do
    python -c "
import json
for l in open('gpurun_out/$f.log'):
    if l.startswith('{'):
        d=json.loads(l); print('%-24s %.4e env-steps/s  %.3f us/step' % ('$f', d['value'], d['ms_per_step']*1e3))
"
  done
done
