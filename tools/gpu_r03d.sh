#!/bin/bash
# Round 3: per-role segment cycles of the sync kernel (diagnostic build), C5 chunk sweep.
set -u
mkdir -p gpurun_out/r03
SIT_LIBRARY=build_diag/libsit_diagsync.so timeout -k 10 200 python -u tools/diag_sync.py > gpurun_out/r03/diag_sync.json 2> gpurun_out/r03/diag_sync.err || exit $?
cat gpurun_out/r03/diag_sync.json
SIT_LIBRARY=build_diag/libsit_diagsync.so timeout -k 10 200 python -u tools/diag_sync.py --policy > gpurun_out/r03/diag_sync_policy.json 2> gpurun_out/r03/diag_sync_policy.err || exit $?
cat gpurun_out/r03/diag_sync_policy.json
for k in 48 96 128; do
  timeout -k 10 200 python -u bench.py --mode policy --groups 1 --chunk $k --steps 32768 --warmup 30000 --no-cpu-baseline \
    > gpurun_out/r03/c5d_k$k.json 2> gpurun_out/r03/c5d_k$k.err || exit $?
  python3 -c "
import json;d=json.load(open('gpurun_out/r03/c5d_k$k.json'))
print('C5 g1 chunk $k', '%.4e' % d['value'], d['config']['env_step_fraction'], d['roofline']['launch_ms'])"
done
timeout -k 10 400 python -u tools/f32_drift.py --out gpurun_out/r03/f32_drift.json > gpurun_out/r03/f32_drift.log 2>&1 || exit $?
python3 -c "
import json;d=json.load(open('gpurun_out/r03/f32_drift.json'))
for k in ('f32','s32'): r=d[k]; print(k, r['envs_diverged'], r['earliest_divergence_step'], '%.2e %.2e' % (r['next_state_max'], r['next_state_p99']), r['next_state_per_field_max'])
"
