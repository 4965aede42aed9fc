#!/usr/bin/env python3
"""Per-call latency of the scalar drop-in (compat.MultiShipRLEnv.step: one sit_step_host call -- the
inputs staged in pinned coherent memory the kernel reads and writes directly, one launch, the state blob
copied when recording, one synchronisation -- plus the host bookkeeping) on the reference's nominal
episode, built from the reference-form constructor (stand-ins of its ShipAssets, tests/ref_assets.py).
Writes one JSON line.
The reference's own env step measured 0.86 ms (full two-ship MultiShipRLEnv.step with
reward, one core)."""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from helpers import golden  # noqa: E402
from ref_assets import args, fixture_assets, polygon_obstacle  # noqa: E402

from sac_maritime_ast_amd.compat import MultiShipRLEnv  # noqa: E402


def run(precision, record, n=600):
    d = golden("env_nominal")
    env = MultiShipRLEnv(fixture_assets(d), polygon_obstacle(), False, 30, args(), device="cuda:0",
                         precision=precision, wpt_capacity=d["routes"].shape[1], record=record)
    env.reset()
    env.init_step()
    # the recorded actions as plain Python values (an NpzFile re-reads and decompresses an array on
    # every d[key] access: inside the timed call that was most of round 3's 173 us)
    acts = [(float(a), float(b)) for a, b in zip(d["action_n"][:n], d["action_e"][:n])]
    sacs, inits = [bool(x) for x in d["sac_update"][:n]], [bool(x) for x in d["init"][:n]]
    lat = []
    for i in range(n):
        a, sac, ini = acts[i], sacs[i], inits[i]
        t0 = time.perf_counter()
        env.step(a, sac, ini)
        lat.append(time.perf_counter() - t0)
    v = np.asarray(lat[50:]) * 1e6
    kernel = env.vec.lib.sit_step_kernel(env.vec.handle).decode()
    return {"precision": precision, "record": record, "kernel": kernel, "steps": len(v), "median_us": float(np.median(v)),
            "p10_us": float(np.percentile(v, 10)), "p90_us": float(np.percentile(v, 90)),
            "mean_us": float(v.mean())}


if __name__ == "__main__":
    torch.cuda.init()
    res = [run(p, r) for p in (64, 32) for r in (True, False)]
    print(json.dumps({"what": "compat.MultiShipRLEnv.step wall time per call (host perf_counter), after 50 "
                              "warm-up calls, env_nominal actions", "reference_ms_per_env_step": 0.86,
                      "reference_source": "SURVEY.md §3.1 (one core, full two-ship step with reward)",
                      "results": res, "host": os.uname().nodename}))
