#!/bin/bash
# Round 3: per-role sub-segment cycles of the current sync kernel (C3 and policy mode).
export TMPDIR=/tmp
mkdir -p gpurun_out/r03k
tools/gpu_steps.sh \
 r03k/diag_c3 200 env SIT_LIBRARY=build_diag/libsit_diagsync.so python -u tools/diag_sync.py --- \
 r03k/diag_c5 200 env SIT_LIBRARY=build_diag/libsit_diagsync.so python -u tools/diag_sync.py --policy
