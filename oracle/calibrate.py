#!/usr/bin/env python3
"""CPU calibration of the NumPy restatement against the reference (BASELINE.md CPU plan, item 1).

MEASUREMENT INFRASTRUCTURE ONLY — runs in the build container, where /root/reference exists (it
is imported read-only, through tests/golden/make_golden.py's constructors; nothing of it is copied).
Never imported by the product path, bench.py or the GPU tests.

On one pinned core, best of N:
  * C1 (BASELINE config 1): 1 ship, route [[0, 0], [10000, 10000]], 1000 zero-action simulator steps
    as MSRL_Env.obs_step's non-stop path runs them (store_simulation_data included) — the reference
    simulator (ship-steps/s) and oracle/sit_oracle.py with one env (``sim_step``);
  * the full two-ship ``MultiShipRLEnv.step`` with reward and done under the synthetic IW sampler —
    the reference env (RLEnv/MSRL_env_ex.py under make_golden.py's shims) and the oracle with one env
    (``OracleEnvs.rollout``), env-steps/s.
The ratio reference / restatement converts the bench's scalar restatement timing on the GPU box's
host (bench.py ``cpu_baseline``, where the reference cannot run) into an estimate of the reference's
own speed there.

    python oracle/calibrate.py --out profiles/r02_cpu_calibration.json
"""
from __future__ import annotations

import argparse
import json
import math
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def best_rate(fn, units, reps):
    best = math.inf
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        best = min(best, time.perf_counter() - t0)
    return units / best, best


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_cpu_calibration.json"))
    ap.add_argument("--core", type=int, default=0)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--env-steps", type=int, default=300)
    a = ap.parse_args()
    os.sched_setaffinity(0, {a.core})

    import make_golden as mg                       # reference constructors (imports /root/reference)
    from helpers import POLYS, init_rows           # noqa: E402
    from oracle import sit_oracle as so            # noqa: E402
    from sac_maritime_ast_amd.scenario import make_scenario  # noqa: E402

    ref = mg._import_reference()
    c1_route, c1_pose = [[0.0, 0.0], [10000.0, 10000.0]], (0, 0, np.pi / 4, 0, 0, 0)

    # ---- C1: reference simulator vs oracle (1 env) ----
    def ref_c1():
        ship, thr, ap_ = mg.build_ship(ref, c1_route, c1_pose)
        for _ in range(1000):
            mg.sim_step(ship, thr, ap_)
    ref_c1_rate, _ = best_rate(ref_c1, 1000, a.reps)

    routes = np.zeros((1, 2, 8, 2))
    routes[0, :, :2] = c1_route
    init = init_rows(np.asarray([[c1_pose, c1_pose]], float))

    def orc_c1():
        o = so.OracleEnvs(dict(so.DEFAULT_PARAMS), routes, np.array([[2, 2]]), init, POLYS)
        for _ in range(1000):
            o.sim_step(1)
    orc_c1_rate, _ = best_rate(orc_c1, 1000, a.reps)

    # ---- two-ship env step: reference env (shims) vs oracle (1 env), synthetic IW sampler ----
    ref2, obstacle, env_mod = mg.install_env_shims()
    rng = np.random.default_rng(25450)
    pose_t = (mg.R_TEST[0][0], mg.R_TEST[0][1], math.atan2(4000, 300), 0, 0, 0)
    pose_o = (mg.R_OBS[0][0], mg.R_OBS[0][1], math.atan2(-100, 6400), 0, 0, 0)
    n_env_steps = a.env_steps

    def ref_env():
        env = mg.make_env(ref2, obstacle, env_mod, pose_t, pose_o)
        env.reset()
        env.init_step()
        iw, t = (0.0, 0.0), 1
        for _ in range(n_env_steps):
            init = t == 1
            sample = init or (env.sampling_distance_travelled >= env.AB_segment_length and not env.obs.stop_flag)
            if sample:
                ang = rng.uniform(-np.pi / 6, np.pi / 6)
                iw = (env.obs.ship_model.north + env.AB_segment_length * np.cos(env.AB_alpha + ang),
                      env.obs.ship_model.east + env.AB_segment_length * np.sin(env.AB_alpha + ang))
            _, _, done, _ = env.step(iw, bool(sample), init)
            t += 1
            if done:
                env.reset()
                env.init_step()
                t = 1
    ref_env_rate, _ = best_rate(ref_env, n_env_steps, max(2, a.reps // 2))

    sc = make_scenario(1, cap=32, jitter=False)

    def orc_env():
        o = so.OracleEnvs(dict(so.DEFAULT_PARAMS), sc.routes, sc.n_wpt, sc.init, sc.polys)
        o.reset()
        o.init_step()
        o.rollout(n_env_steps, 25450)
    orc_env_rate, _ = best_rate(orc_env, n_env_steps, max(2, a.reps // 2))

    out = {
        "what": "reference vs oracle/sit_oracle.py on one pinned core of the build container (BASELINE.md CPU plan 1)",
        "cpu_model": cpu_model(), "core": a.core, "python": platform.python_version(), "numpy": np.__version__,
        "c1_ship_steps_per_s": {"reference": ref_c1_rate, "restatement_1env": orc_c1_rate,
                                "ratio_reference_over_restatement": ref_c1_rate / orc_c1_rate,
                                "workload": "1 ship, 1000 zero-action simulator steps incl. store_simulation_data, best of "
                                            f"{a.reps}"},
        "env_steps_per_s": {"reference": ref_env_rate, "restatement_1env": orc_env_rate,
                            "ratio_reference_over_restatement": ref_env_rate / orc_env_rate,
                            "workload": f"two-ship MultiShipRLEnv.step with reward/done, synthetic IW sampler, "
                                        f"{n_env_steps} steps with auto-reset; reference env under make_golden.py's "
                                        "shims (shapely replaced by a NumPy/matplotlib stand-in)"},
    }
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(out, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
