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
    """The state with the float32 handle's double-float fields as their float64 values hi + lo."""
    return {k: v.cpu().numpy() for k, v in env.get_state(combined=True).items()}


def rel(a, b, floor):
    return np.abs(a.astype(np.float64) - b.astype(np.float64)) / np.maximum(np.abs(b.astype(np.float64)), floor)


def _discrete(o, st):
    """The discrete outcome of a step per env: done, status, sampling event, state integers."""
    d = {"done": o["done"], "status": o["status"], "sac": o["sac"]}
    for f in INTS:
        d[f] = st[f]
    return d


def _differs(a, b):
    """Per env: which discrete quantities differ (list of names per env)."""
    n = a["done"].shape[-1]
    out = [[] for _ in range(n)]
    for k in a:
        d = a[k] != b[k]
        d = d.any(0) if d.ndim == 2 else d
        for e in np.nonzero(d)[0]:
            out[e].append(k)
    return out


def measure(n_env=4096, steps=2000, seed=77, log=True, attribute=False, fused_chunk=0, storage_fields=None):
    """The report (a dict) of n_env envs x steps steps; tests/test_gpu_parity.py gates on it.
    attribute: for every env at its first float32 divergence, re-run that step in float64 from the
    float32 run's own pre-step state (a float64 handle of the same envs and global ids, teacher-forced
    for one step) and record which of the two decisions the exact arithmetic takes there.
    fused_chunk > 0: a fourth handle, float32, runs the same episodes as bench.py times them — fused
    launches of `fused_chunk` steps (k_env_steps_sync with the LDS-staged map, replay transitions
    written) — and every one of its steps' outputs and its state at every launch end are compared
    bit for bit with the one-step-per-launch float32 run: where they are identical, the deviations
    measured per step on the one-step run are those of the benchmarked instantiation.
    storage_fields: round only these state fields to float32 in the storage-only run (an attribution of
    the float32 run's deviations to the storage of individual fields; None = every real field)."""
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
    flips = []
    tf = VecMultiShipRLEnv(scenario=sc, precision=64, device="cuda:0") if attribute else None
    fz = None
    if fused_chunk:
        fz = VecMultiShipRLEnv(scenario=sc, precision=32, device="cuda:0")
        fz.reset()
        fz.init_step()
        fz_out, fz_rows, fz_bad = {}, [], np.zeros(n, dtype=bool)
        fz_tcap = max(n, n * fused_chunk // 96)
        fz_kernel = None
    for step in range(args.steps):
        if fz is not None and step % fused_chunk == 0:
            k = min(fused_chunk, args.steps - step)
            o = fz.rollout(k, seed=args.seed, out=fz_out, transition_capacity=fz_tcap)
            fz_kernel = fz.lib.sit_step_kernel(fz.handle).decode()
            fz_rows = [{q: o[q][i].cpu().numpy() for q in ("next_state", "reward", "done", "status", "action")}
                       for i in range(k)]
            fz_state = {q: v.cpu().numpy() for q, v in fz.get_state().items()}
        res = {}
        pre = {k: state(envs[k]) for k in ("f32", "f64")} if attribute else None
        for k, e in envs.items():
            o = e.rollout(1, seed=args.seed, out=outs[k])
            if k == "f32" and fz is not None:
                e._last_rows = {q: o[q][0].cpu().numpy() for q in ("next_state", "reward", "done", "status", "action")}
            res[k] = ({q: o[q][0].cpu().numpy() for q in ("next_state", "reward", "done", "status")} |
                      {"sac": o["action"][0, :, 3].cpu().numpy()}, state(e))
        if attribute:
            d32, d64 = _discrete(*res["f32"]), _discrete(*res["f64"])
            w32 = _differs(d32, d64)
            new_div = [e for e, w in enumerate(w32) if w and first["f32"][e] == args.steps]
            if new_div:
                # the float64 kernel, one step from the float32 run's pre-step state (every env; the
                # sampler draws are keyed by (seed, global env id, event), so they are the same draws)
                tf.set_state({f: v.astype(np.float64) if v.dtype == np.float32 else v for f, v in pre["f32"].items()})
                o = tf.rollout(1, seed=args.seed)
                dtf = _discrete({q: o[q][0].cpu().numpy() for q in ("done", "status")} |
                                {"sac": o["action"][0, :, 3].cpu().numpy()}, state(tf))
                wtf32, wtf64 = _differs(dtf, d32), _differs(dtf, d64)
                # post-step positions before any auto reset: the next_state rows (test n, e at 0, 1;
                # obstacle n, e at 6, 7)
                ns32, ns64 = res["f32"][0]["next_state"], res["f64"][0]["next_state"]
                for e in new_div:
                    # status flips are terrain / hull predicates of the post-step position: the exact
                    # (float64, GEOS-restated) hull and corner distances at the float32 run's and at the
                    # float64 run's post-step positions (sit_probe_map on the float64 handle)
                    hull = {}
                    if d32["status"][e] != d64["status"][e]:
                        half = 0.5 * float(envs["f64"].params.length_of_ship)
                        for t in (0, 1):
                            pts = []
                            for src in (ns32, ns64):
                                n0, e0 = float(src[e, 6 * t]), float(src[e, 6 * t + 1])
                                pts += [[n0, e0]] + [[n0 + a * half, e0 + b * half] for a in (-1, 1) for b in (-1, 1)]
                            dist, _, hl = tf.probe_map(np.asarray(pts))
                            dist, hl = dist.cpu().numpy(), hl.cpu().numpy()
                            hull[f"ship{t}"] = {
                                "hull_in_terrain_exact_at_f32_position": bool(hl[0]),
                                "hull_in_terrain_exact_at_f64_position": bool(hl[5]),
                                "min_corner_boundary_distance_m_f32": float(dist[1:5].min()),
                                "min_corner_boundary_distance_m_f64": float(dist[6:10].min()),
                                "position_difference_m": float(np.hypot(ns32[e, 6 * t] - ns64[e, 6 * t],
                                                                        ns32[e, 6 * t + 1] - ns64[e, 6 * t + 1]))}
                    flips.append({
                        "env": int(e), "step": int(step), "flipped": w32[e],
                        "exact_from_f32_state_takes": ("f32 decision" if not wtf32[e] else
                                                       "f64 decision" if not wtf64[e] else "neither"),
                        "status_bits_f32": int(d32["status"][e]), "status_bits_f64": int(d64["status"][e]),
                        "next_wpt_f32": [int(x) for x in d32["next_wpt"][:, e]],
                        "next_wpt_f64": [int(x) for x in d64["next_wpt"][:, e]],
                        # how far the float32 run's state had drifted from the float64 run's before the step
                        "pre_state_rel_dev_max": float(max(rel(pre["f32"][f][:, e], pre["f64"][f][:, e],
                                                               SCALE[f]).max() for f in REAL)),
                        "hull": hull,
                    })
        if fz is not None:
            # the fused launch's row of this step against the one-step launch's, bit for bit
            o1 = envs["f32"]._last_rows
            row = fz_rows[step % fused_chunk]
            for q in row:
                a, b = row[q], o1[q]
                eq = (a == b) | (np.isnan(a) & np.isnan(b)) if a.dtype.kind == "f" else a == b
                fz_bad |= ~eq.reshape(n, -1).all(1)
            if (step + 1) % fused_chunk == 0 or step + 1 == args.steps:
                s1 = {q: v.cpu().numpy() for q, v in envs["f32"].get_state().items()}
                for q, v in fz_state.items():
                    if q.startswith("iw_key"):        # the single-step launches' IW-test cache, not model state
                        continue
                    d = v != s1[q]
                    fz_bad |= d.reshape(-1, n).any(0) if d.ndim > 1 else d
        # s32: float32 state storage (every real field of the state rounded after the step)
        s = res["s32"][1]
        envs["s32"].set_state({f: v.astype(np.float32).astype(np.float64) for f, v in s.items()
                               if v.dtype == np.float64 and (storage_fields is None or f in storage_fields)})
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
    if fz is not None:
        report["fused"] = {"kernel": fz_kernel, "steps_per_launch": fused_chunk,
                           "envs_differing_from_one_step_run": int(fz_bad.sum()),
                           "how": "every step's outputs (next_state, reward, done, status, action) and the state at "
                                  "every launch end of the fused float32 run, bit for bit against the one-step "
                                  "float32 run"}
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
    if attribute:
        for f in flips:
            f["storage_only_run_diverges_at"] = int(first["s32"][f["env"]]) if first["s32"][f["env"]] < args.steps else None
        takes = [f["exact_from_f32_state_takes"] for f in flips]
        report["f32_flip_attribution"] = {
            "how": "for every env at its first float32 divergence (step t): the float64 kernel re-runs step t "
                   "from the float32 run's own pre-step state (same envs, global ids and sampler draws). "
                   "'f32 decision': exact arithmetic from the drifted state decides as the float32 step did, so "
                   "the flip comes from the state's accumulated float32 rounding (storage), not from the float32 "
                   "arithmetic of that step; 'f64 decision': the float32 arithmetic of the step flipped it.",
            "envs": len(flips), "exact_takes_f32_decision": takes.count("f32 decision"),
            "exact_takes_f64_decision": takes.count("f64 decision"), "neither": takes.count("neither"),
            "also_diverge_in_storage_only_run": sum(1 for f in flips if f["storage_only_run_diverges_at"] is not None),
            "flips": flips}
    return report


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-env", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--seed", type=int, default=77)
    ap.add_argument("--out", default=None)
    ap.add_argument("--attribute", action="store_true", help="attribute every float32 divergence (see measure)")
    ap.add_argument("--fused-chunk", type=int, default=0, help="> 0: also run the benchmarked instantiation "
                    "(fused launches of this many steps) and compare it bit for bit with the one-step run")
    ap.add_argument("--storage-fields", default=None, help="comma-separated: the storage-only run rounds only these")
    args = ap.parse_args()
    report = measure(args.n_env, args.steps, args.seed, attribute=args.attribute, fused_chunk=args.fused_chunk,
                     storage_fields=args.storage_fields.split(",") if args.storage_fields else None)
    txt = json.dumps(report, indent=1)
    print(txt)
    if args.out:
        with open(args.out, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
