#!/bin/bash
# Round 3: debug-variant bisect over revisions, then the PMC passes of the current default bench (C3 only).
export TMPDIR=/tmp
mkdir -p gpurun_out/r03g
tools/gpu_steps.sh \
 r03g/debug 300 python -u tools/debug_libs.py build_diag/libsit_dbg_acaeb96.so build_diag/libsit_dbg_c69dd22.so sac_maritime_ast_amd/libsit_debug.so --- \
 r03g/pmc 900 bash tools/pmc.sh --no-c5
rc=$?
python3 tools/pmc_summary.py gpurun_out/pmc k_env_steps_sync 8 > gpurun_out/r03g/pmc_summary.json
find gpurun_out/pmc -name "*.csv" -size +1M -delete
exit $rc
