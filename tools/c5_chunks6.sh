#!/bin/bash
# C5 (in-kernel serving) by steps per launch: tools/c5_chunks6.sh <out dir> K...
set -u
O=$1; shift
mkdir -p $O
for K in "$@"; do
  timeout -k 10 200 python3 bench.py --mode policy --chunk $K --groups 1 --steps 8192 --warmup 30720 --no-cpu-baseline \
    > $O/k$K.json 2> $O/k$K.err || exit 1
  python3 -c "
import json; d=json.loads(open('$O/k$K.json').read().strip().splitlines()[-1])
print('K=$K', '%.4e' % d['value'], 'frac %.3f' % d['config']['env_step_fraction'], 'kernel ms %.4f' % d['roofline']['kernel_ms_per_launch'])"
done
