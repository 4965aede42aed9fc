#!/bin/bash
# float32 drift (envs diverged, max) of library variants: tools/comp_drift.sh [lib ...]
# (default: the round-5 compensation variants)
set -u
mkdir -p gpurun_out/compdrift
LIBS=("$@")
[ ${#LIBS[@]} -eq 0 ] && LIBS=(sac_maritime_ast_amd/libsit.so build_diag/libsit_nopsi.so build_diag/libsit_nopi.so build_diag/libsit_nopsipi.so)
for L in "${LIBS[@]}"; do
  n=$(basename $L .so)
  SIT_LIBRARY=$L timeout -k 10 200 python tools/f32_drift.py --out gpurun_out/compdrift/$n.json > gpurun_out/compdrift/$n.log 2>&1 || { echo "$n failed"; exit 1; }
  python -c "
import json; d=json.load(open('gpurun_out/compdrift/$n.json'))
print('$n', 'f32 diverged', d['f32']['envs_diverged'], 'max %.3g' % d['f32']['next_state_max'], 'earliest', d['f32']['earliest_divergence_step'])"
done
