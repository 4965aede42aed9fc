#!/bin/bash
# Round-5 record of the current build (on the GPU box, via gpurun), in two calls (a call is limited to
# 20 minutes):
#   tools/gpu_round5.sh <tag> a   the GPU suite (knife-edge counts recorded), role placement probe,
#                                 float32 drift attribution, drop-in latency
#   tools/gpu_round5.sh <tag> b   the record recipe (tools/gpu_record.sh: smoke, bench with every line,
#                                 rocprof stats, PMC of both step kernels)
#   tools/gpu_round5.sh <tag> c   the env-population curve (tools/nenv_curve.sh)
set -u
export TMPDIR=/tmp
T=${1:-r05rec}
P=${2:-a}
O=gpurun_out/$T
mkdir -p $O
case $P in
a) tools/gpu_steps.sh \
     $T/tests 600 env SIT_TEST_RECORD_DIR=$O python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s --- \
     $T/roles 120 python3 tools/role_probe.py --- \
     $T/drift 300 python3 tools/f32_drift.py --attribute --out $O/f32_flip_attribution.json --- \
     $T/compat 200 python3 tools/compat_latency.py ;;
b) bash tools/gpu_record.sh $T/rec ;;
c) bash tools/nenv_curve.sh $O/nenv ;;
esac
