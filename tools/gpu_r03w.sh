#!/bin/bash
# A/B: scheduler occupancy target (SIT_SYNC_WPE=2) and the max-ILP machine scheduler against the current build, C3 and C5.
set -eu
cd "$(dirname "$0")/.."
bash tools/ab_libs.sh 3 build_diag/libsit_base.so build_diag/libsit_wpe2.so build_diag/libsit_ilpf.so build_diag/libsit_ilpfw.so
