#!/bin/bash
# Round 3: timing ablations of the sync kernel (C3, interleaved) and the K = 1 launch's phases.
export TMPDIR=/tmp
mkdir -p gpurun_out/r03i
BENCH_ARGS="--no-c5" timeout -k 10 400 bash tools/ab_libs.sh 2 build_diag/libsit_base.so build_diag/libsit_abl_dg.so \
  build_diag/libsit_abl_dk.so build_diag/libsit_abl_po.so build_diag/libsit_abl_pp.so > gpurun_out/r03i/ab.log 2>&1
rc=$?; cat gpurun_out/r03i/ab.log; [ $rc -eq 0 ] || exit $rc
SIT_LIBRARY=build_diag/libsit_phases.so timeout -k 10 200 python -u tools/diag_step.py > gpurun_out/r03i/diag_step.json 2> gpurun_out/r03i/diag_step.err
rc=$?; cat gpurun_out/r03i/diag_step.json; tail -3 gpurun_out/r03i/diag_step.err; exit $rc
