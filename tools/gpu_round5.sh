#!/bin/bash
# Round-5 record of the current build (on the GPU box, via gpurun): the GPU suite, the record recipe
# (tools/gpu_record.sh: smoke, bench with every line, rocprof stats, PMC of both step kernels), then the
# round-5 measurements: env-population curve, role placement probe, float32 drift attribution, drop-in
# latency.  usage: tools/gpu_round5.sh <tag>
set -u
export TMPDIR=/tmp
T=${1:-r05rec}
O=gpurun_out/$T
mkdir -p $O
tools/gpu_steps.sh \
 $T/tests 600 env SIT_TEST_RECORD_DIR=$O python3 -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -s --- \
 $T/roles 120 python3 tools/role_probe.py --- \
 $T/drift 300 python3 tools/f32_drift.py --attribute --out $O/f32_flip_attribution.json --- \
 $T/compat 200 python3 tools/compat_latency.py || exit $?
bash tools/gpu_record.sh $T/rec || exit $?
bash tools/nenv_curve.sh $O/nenv
