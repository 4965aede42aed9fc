#!/bin/bash
# SQ PMC passes on the default bench (C3, K=5000) + the phase-split diagnostic build.
set -u
export TMPDIR=/tmp
out=gpurun_out/pmc2
mkdir -p $out
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
           "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_IFETCH"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $grp -d $out/p$i -o run --output-format csv -- python3 bench.py --no-cpu-baseline > $out/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/p$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py $out > $out/summary.json && head -c 1500 $out/summary.json
SIT_LIBRARY=build_diag/libsit_phases.so timeout -k 10 120 python tools/diag_paths.py > gpurun_out/phases.txt 2>&1; echo "phases rc=$?"; tail -30 gpurun_out/phases.txt
