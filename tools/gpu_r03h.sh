#!/bin/bash
# Round 3: the full GPU suite on the current build, then the per-role sub-segment cycles (diagnostic build).
export TMPDIR=/tmp
mkdir -p gpurun_out/r03h
tools/gpu_steps.sh \
 r03h/tests 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider --- \
 r03h/diag_sync 200 env SIT_LIBRARY=build_diag/libsit_diagsync.so python -u tools/diag_sync.py
