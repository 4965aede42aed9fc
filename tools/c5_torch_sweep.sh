#!/bin/bash
# C5 with the actor forward in PyTorch-ROCm on the request queue (bench.py's c5_torch_actor line):
# stream groups G, steps per launch K, request capacity n/D, the actor on its own stream (S = 1)
#   usage: tools/c5_torch_sweep.sh <out dir> [G:K:D:S ...]
set -u
O=${1:-gpurun_out/c5t}
shift
mkdir -p $O
CFGS=${*:-2:32:4:0 1:64:4:0 1:64:4:1 1:32:4:0 1:64:2:0 2:64:4:0 1:96:4:0}
for C in $CFGS; do
  IFS=: read G K D S <<< "$C"
  X=""; [ "$S" = 1 ] && X="--actor-stream"
  n=g${G}k${K}d${D}s${S}
  timeout -k 10 150 python bench.py --mode policy --serve queue --torch-actor --chunk $K --groups $G --request-div $D $X \
    --steps 8192 --warmup 15360 --no-cpu-baseline > $O/$n.json 2> $O/$n.err || { echo "$n failed"; tail -3 $O/$n.err; exit 1; }
  python -c "
import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1])
print('$n', '%.4e' % d['value'], 'frac %.3f' % d['config']['env_step_fraction'], 'launch ms %.3f' % d['roofline']['launch_ms']['median'])"
done
