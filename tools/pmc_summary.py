#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (tools/pmc.sh output) for one kernel: per-dispatch means.

    python3 tools/pmc_summary.py <dir> [kernel substring] [leading dispatches to skip]
"""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
kern = sys.argv[2] if len(sys.argv) > 2 else "k_env_steps"
skip = int(sys.argv[3]) if len(sys.argv) > 3 else 0     # leading dispatches to ignore (warm-up)
vals = defaultdict(list)
meta = {}
for f in sorted(glob.glob(f"{root}/p*/run_counter_collection.csv")):
    per_disp = defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if kern not in r["Kernel_Name"]:
            continue
        d = r["Dispatch_Id"]
        per_disp[d][r["Counter_Name"]] = per_disp[d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        per_disp[d]["_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        meta.update(grid=int(r["Grid_Size"]), wg=int(r["Workgroup_Size"]), lds=int(r["LDS_Block_Size"]),
                    vgpr=int(r["VGPR_Count"]), sgpr=int(r["SGPR_Count"]), scratch=int(r["Scratch_Size"]))
    for d in sorted(per_disp, key=int)[skip:]:
        for k, v in per_disp[d].items():
            vals[k].append(v)
out = {k: sum(v) / len(v) for k, v in vals.items()}
out.update(meta)
print(json.dumps(out, indent=1))
