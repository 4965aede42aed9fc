#!/usr/bin/env python3
"""float32 free-running deviation from the float64 kernel, attributed per field (full
trajectories are reported, not gated).

Three handles run the same synthetic-sampler episodes with auto-reset from identical starts, one
step per launch (the benchmarked kernel, k_env_steps_sync, takes K = 1 like any other K):
  f64   the reference's arithmetic (the baseline)
  f32   the benchmarked float32 handle
  s32   the float64 kernel whose state is rounded to float32 after every step: what float32 STATE
        STORAGE alone costs (SURVEY §8(d) bounds it at <= 2.5e-5 over 7 200 steps)
Per env the runs agree until the first step whose discrete outcome differs (done, status, sampling
event, or a state integer: waypoint index, route length, stop flags, episode step, sampler counter).
Before that step, per field: max and p99 over envs of the largest relative deviation (contract floors:
next_state OBS_SCALE, state SCALE).  Writes one JSON document (profiles/r03_f32_free_running.json)."""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from helpers import OBS_SCALE, SCALE  # noqa: E402

from sac_maritime_ast_amd import VecMultiShipRLEnv, make_scenario  # noqa: E402

NS_NAMES = ["test north", "test east", "test yaw", "test rpm", "test |e_ct|", "test P_me",
            "obs north", "obs east", "obs yaw", "obs |e_ct|"]
REAL = ("north", "east", "yaw", "surge", "sway", "yaw_rate", "shaft_speed", "ship_speed_i", "shaft_speed_i",
        "heading_i", "heading_prev", "e_ct_int")
INTS = ("next_wpt", "n_wpt", "stop", "ep_step", "event")


def state(env):
    return {k: v.cpu().numpy() for k, v in env.get_state().items()}


def rel(a, b, floor):
    return np.abs(a.astype(np.float64) - b.astype(np.float64)) / np.maximum(np.abs(b.astype(np.float64)), floor)


def measure(n_env=4096, steps=2000, seed=77, log=True):
    """The report (a dict) of n_env envs x steps steps; tests/test_gpu_parity.py gates on it."""
    args = argparse.Namespace(n_env=n_env, steps=steps, seed=seed)
    n = args.n_env
    sc = make_scenario(n, cap=48)
    envs = {k: VecMultiShipRLEnv(scenario=sc, precision=p, device="cuda:0") for k, p in (("f64", 64), ("f32", 32),
                                                                                        ("s32", 64))}
    for e in envs.values():
        e.reset()
        e.init_step()
    first = {k: np.full(n, args.steps) for k in ("f32", "s32")}
    ns_dev = {k: np.zeros((n, 10)) for k in first}
    st_dev = {k: {f: np.zeros((2, n)) for f in REAL} for k in first}
    outs = {k: {} for k in envs}
    for step in range(args.steps):
        res = {}
        for k, e in envs.items():
            o = e.rollout(1, seed=args.seed, out=outs[k])
            res[k] = ({q: o[q][0].cpu().numpy() for q in ("next_state", "reward", "done", "status")} |
                      {"sac": o["action"][0, :, 3].cpu().numpy()}, state(e))
        # s32: float32 state storage (every real field of the state rounded after the step)
        s = res["s32"][1]
        envs["s32"].set_state({f: v.astype(np.float32).astype(np.float64) for f, v in s.items()
                               if v.dtype == np.float64})
        ref_o, ref_s = res["f64"]
        for k in first:
            o, st = res[k]
            diff = (o["done"] != ref_o["done"]) | (o["status"] != ref_o["status"]) | (o["sac"] != ref_o["sac"])
            for f in INTS:
                d = st[f] != ref_s[f]
                diff |= d.any(0) if d.ndim == 2 else d
            first[k] = np.where(diff & (first[k] == args.steps), step, first[k])
            ok = step < first[k]
            e = rel(o["next_state"], ref_o["next_state"], OBS_SCALE)
            ns_dev[k] = np.where(ok[:, None], np.maximum(ns_dev[k], e), ns_dev[k])
            for f in REAL:
                e = rel(st[f], ref_s[f], SCALE[f])
                st_dev[k][f] = np.where(ok[None, :], np.maximum(st_dev[k][f], e), st_dev[k][f])
        if log and step % 200 == 0:
            print(f"step {step}: diverged f32 {int((first['f32'] < args.steps).sum())}, "
                  f"s32 {int((first['s32'] < args.steps).sum())}", file=sys.stderr, flush=True)
    report = {"what": __doc__.split("\n\n")[0], "n_env": n, "steps": args.steps,
              "kernel": envs["f32"].lib.sit_step_kernel(envs["f32"].handle).decode()}
    for k, label in (("f32", "float32 kernel vs float64 kernel"), ("s32", "float32 state storage only")):
        div = first[k] < args.steps
        r = {"label": label, "envs_diverged": int(div.sum()),
             "earliest_divergence_step": int(first[k].min()) if div.any() else None,
             "median_divergence_step": float(np.median(first[k][div])) if div.any() else None,
             "next_state_max": float(ns_dev[k].max()), "next_state_p99": float(np.percentile(ns_dev[k].max(1), 99)),
             "next_state_median": float(np.median(ns_dev[k].max(1))),
             "next_state_per_field_max": {nm: float(ns_dev[k][:, j].max()) for j, nm in enumerate(NS_NAMES)},
             "next_state_per_field_p99": {nm: float(np.percentile(ns_dev[k][:, j], 99)) for j, nm in enumerate(NS_NAMES)},
             "state_per_field_max": {f"{f}[{s}]": float(st_dev[k][f][s].max()) for f in REAL for s in (0, 1)},
             "argmax_env": int(ns_dev[k].max(1).argmax())}
        report[k] = r
    return report


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-env", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=77)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    report = measure(args.n_env, args.steps, args.seed)
    txt = json.dumps(report, indent=1)
    print(txt)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
