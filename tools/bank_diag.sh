#!/bin/bash
# LDS bank-conflict diagnostic of the C3 step kernel (one PMC pass each): the default launch, the map
# read through the caches (SIT_LDS_MAP=0), and without the replay-transition stream (no LDS ring).
#   usage (on the GPU box): tools/bank_diag.sh <out dir>
set -u
export TMPDIR=/tmp
out=$1
mkdir -p $out
CNT="SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS"
run() {
  tag=$1; shift
  timeout -s KILL 150 "$@" > $out/$tag.log 2>&1
  rc=$?
  echo "$tag rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $out/$tag.log; exit $rc; }
  python3 tools/pmc_summary.py $out/$tag k_env_steps_sync 1 > $out/$tag.json
}
B="python3 bench.py --no-cpu-baseline --no-extra-lines --no-c5 --steps 20000 --warmup 40000"
run lds rocprofv3 --kernel-trace --pmc $CNT -d $out/lds/p1 -o run --output-format csv -- $B
SIT_LDS_MAP=0 run global rocprofv3 --kernel-trace --pmc $CNT -d $out/global/p1 -o run --output-format csv -- $B
run nogather rocprofv3 --kernel-trace --pmc $CNT -d $out/nogather/p1 -o run --output-format csv -- $B --no-gather
find $out -name "*.csv" -size +1M -delete
python3 - $out <<'PY'
import json, sys
o = sys.argv[1]
for t in ("lds", "global", "nogather"):
    d = json.load(open(f"{o}/{t}.json"))
    ws = d["SQ_WAVES"] * 40000 if "SQ_WAVES" in d else None
    print(t, {k: round(d[k] / ws, 2) for k in ("SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS", "SQ_WAVE_CYCLES", "SQ_ACTIVE_INST_LDS") if k in d})
PY
