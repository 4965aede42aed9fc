#!/bin/bash
# Diagnostic GPU call: PMC passes, phase/path diagnostics, ablation benches.
export TMPDIR=/tmp
tools/gpu_steps.sh \
 pmc 900 bash tools/pmc.sh --- \
 phases 120 env SIT_LIBRARY=build_diag/libsit_phases.so python tools/diag_paths.py --- \
 paths 120 env SIT_LIBRARY=build_diag/libsit_paths.so python tools/diag_paths.py --- \
 nopred 120 env SIT_LIBRARY=build_diag/libsit_nopred.so python bench.py --no-cpu-baseline --- \
 nohull 120 env SIT_LIBRARY=build_diag/libsit_nohull.so python bench.py --no-cpu-baseline --- \
 chunk1000 120 python bench.py --no-cpu-baseline --chunk 1000 --steps 10000 --- \
 n65k 120 python bench.py --no-cpu-baseline --n-env 65536
