#!/bin/bash
# Throughput of the C3 kernel against the env population on one GPU (8 k ... 128 k envs): where the
# per-step latency floor sits.  usage (on the GPU box): tools/nenv_curve.sh <out dir>
set -u
export TMPDIR=/tmp
out=$1
mkdir -p $out
for n in 8192 16384 24576 32768 49152 65536 98304 131072; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-c5 --no-extra-lines --n-env $n --chunk 20000 \
    --steps 40000 --warmup 40000 > $out/n$n.json 2> $out/n$n.err || { echo "n=$n failed"; tail -3 $out/n$n.err; exit 1; }
  python3 - $out/n$n.json $n <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
n = int(sys.argv[2])
print(f"n_env {n:6d}  blocks {n // 64:5d}  {d['value']:.4e} env-steps/s  {d['roofline']['kernel_ms_per_launch'] / 20000 * 1e3:.3f} us/step")
PY
done
