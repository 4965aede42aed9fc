#!/bin/bash
# Round 3: per-role cycles of the two-wave kernel for single-step launches (sit_step) and for C3.
export TMPDIR=/tmp
mkdir -p gpurun_out/r03s
tools/gpu_steps.sh \
 r03s/diag_step 200 env SIT_LIBRARY=build_diag/libsit_diagsync.so python -u tools/diag_sync.py --step --- \
 r03s/diag_c3 200 env SIT_LIBRARY=build_diag/libsit_diagsync.so python -u tools/diag_sync.py
