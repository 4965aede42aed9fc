#!/bin/bash
# Extra PMC passes for the step kernel: instruction fetch / mix (diagnostic).
set -u
out=gpurun_out/pmcx
mkdir -p $out
BENCH="python3 bench.py --no-cpu-baseline --warmup 40000 --steps 2000"
i=0
for grp in "SQ_WAVES SQ_IFETCH SQ_INSTS_BRANCH SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_WAIT_INST_LDS" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_TC_INST_REQ" \
           "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_CVT SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $grp -d $out/p$i -o run --output-format csv -- $BENCH > $out/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $out/p$i.log; exit $rc; fi
done
python3 tools/pmc_summary.py $out k_env_steps > gpurun_out/pmcx_summary.json
find $out -name "*.csv" -size +1M -delete
exit 0
