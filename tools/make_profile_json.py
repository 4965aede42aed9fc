#!/usr/bin/env python3
"""profiles/<round>_pmc_f32_rollout.json from tools/pmc_summary.py output (bench.py reads its
hbm_bytes_per_launch as the roofline `traffic` of the matching launch configuration).

    python3 tools/make_profile_json.py gpurun_out/pmc_summary.json profiles/r01_pmc_f32_rollout.json \
        --steps-per-launch 1000 --n-env 32768 --source "..."
"""
import argparse
import json

ap = argparse.ArgumentParser()
ap.add_argument("summary")
ap.add_argument("out")
ap.add_argument("--steps-per-launch", type=int, required=True)
ap.add_argument("--n-env", type=int, default=32768)
ap.add_argument("--precision", type=int, default=32)
ap.add_argument("--mode", default="rollout")
ap.add_argument("--serve", default="kernel", help="policy mode: kernel (in-kernel serving) or queue")
ap.add_argument("--round", type=int, default=1)
ap.add_argument("--source", default="")
ap.add_argument("--kernel", default="k_env_steps_sync<float, 0> (D and P waves per ship, sit_sync.h)")
a = ap.parse_args()
d = json.load(open(a.summary))
ws = d["SQ_WAVES"] * a.steps_per_launch
keys = ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_WR", "SQ_INSTS_VMEM_RD",
        "SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAVE_CYCLES", "SQ_LDS_BANK_CONFLICT",
        "SQ_INSTS_VALU_TRANS_F32")
out = {"kernel": a.kernel, "precision": a.precision, "mode": a.mode, "serve": a.serve if a.mode == "policy" else None,
       "n_env": a.n_env, "steps_per_launch": a.steps_per_launch, "round": a.round, "source": a.source,
       "kernel_ns_per_launch": d["_ns"], "fetch_size_kb": d["FETCH_SIZE"], "write_size_kb": d["WRITE_SIZE"],
       "hbm_bytes_per_launch": (2 * d["FETCH_SIZE"] + d["WRITE_SIZE"]) * 1024,
       "hbm_bytes_note": "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B requests at 64 B); "
                         "WRITE_SIZE as reported; both in KiB",
       "per_wave_step": {k: d[k] / ws for k in keys if k in d},
       "per_wave_step_unit": "instructions; *_CYCLES / ACTIVE / WAIT in quad-cycles (x4 = shader cycles)",
       "vgpr": d.get("vgpr"), "sgpr": d.get("sgpr"), "waves": d["SQ_WAVES"], "raw": d}
json.dump(out, open(a.out, "w"), indent=1)
print(f"{a.out}: {out['hbm_bytes_per_launch'] / 1e6:.1f} MB per launch, {d['_ns'] / 1e6:.3f} ms per launch")
