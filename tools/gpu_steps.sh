#!/bin/bash
# Run GPU steps in order on the gpurun box.  Each step has its own time limit.  A failing
# test (exit 1) does not stop the sequence; a fault, abort, segfault, timeout or any other
# non-zero exit does (nothing more touches the GPU in that call).
#   usage: tools/gpu_steps.sh <name> <timeout_s> <cmd...> [--- <name> <timeout_s> <cmd...>]...
set -u
mkdir -p gpurun_out
while [ $# -gt 0 ]; do
  name=$1; to=$2; shift 2
  cmd=()
  while [ $# -gt 0 ] && [ "$1" != "---" ]; do cmd+=("$1"); shift; done
  [ $# -gt 0 ] && shift
  mkdir -p "gpurun_out/$(dirname "$name")"
  start=$(date +%s)
  timeout -k 10 "$to" "${cmd[@]}" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc t=$(( $(date +%s) - start ))s" | tee -a gpurun_out/steps.log
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "stopping after $name (rc=$rc)"
    exit $rc
  fi
done
exit 0
