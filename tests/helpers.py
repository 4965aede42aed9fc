"""Shared test helpers: load golden fixtures into oracle / product state dictionaries."""
from __future__ import annotations

import glob
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from oracle import sit_oracle as so  # noqa: E402  (test infrastructure)

# the island map of test_beds/test_policy.py:189-194, as (east, north) vertices
MAP = [
    [(0, 10000), (5500, 10000), (5300, 9000), (4800, 8500), (4200, 7300), (4000, 5700), (4300, 4900),
     (4900, 4400), (4400, 4000), (3200, 4100), (2000, 4500), (1000, 4000), (900, 3500), (500, 2600),
     (0, 2350)],
    [(10000, 0), (4000, 0), (4250, 250), (5000, 400), (6000, 900), (8000, 1100), (8500, 1500),
     (9000, 2250), (9500, 3500), (10000, 4000)],
    [(5500, 5500), (5700, 7000), (6200, 8100), (7500, 8000), (7800, 7000), (7600, 5500), (6900, 4700),
     (6000, 5000)],
    [(2000, 2000), (2500, 2300), (4000, 2500), (5000, 3000), (4200, 2100), (3400, 1900)],
]
POLYS = [np.asarray(p, dtype=np.float64) for p in MAP]
OMEGA0 = 400 * np.pi / 30

SIM_FIELDS = ("north", "east", "yaw", "surge", "sway", "yaw_rate", "shaft_speed", "ship_speed_i",
              "shaft_speed_i", "heading_i", "heading_prev", "e_ct_int", "next_wpt")

# per-field scale floors of the parity contract
SCALE = dict(north=1e4, east=1e4, yaw=np.pi, surge=10.0, sway=10.0, yaw_rate=0.1, shaft_speed=100.0,
             ship_speed_i=1e3, shaft_speed_i=1e5, heading_i=10.0, heading_prev=np.pi, e_ct_int=1e2,
             last_rpm=1e3, last_e_ct=1e3, last_power_me=1e3, sampling_dist=1e4, eps_dist=1e4,
             prev_pre_north=1e4, prev_pre_east=1e4, iw_north=1e4, iw_east=1e4,
             rudder=np.pi, throttle=1.0, heading_ref=np.pi, e_ct=1e3, rpm=1e3, power_me=1e3,
             d_north=10.0, d_east=10.0, d_yaw=0.1, d_surge=0.1, d_sway=0.1, d_yaw_rate=1e-3,
             d_shaft_speed=1.0, thrust=1e5, reward=1.0, wpt_north=1e4, wpt_east=1e4)
# SimplifiedMachineryModel fixtures: the shaft-speed slot holds the thrust force [N] and its rate
# d_thrust = (power - k F) / tau [N/s] (a difference of ~1e6 N terms near equilibrium)
SCALE_SIMPL = dict(SCALE, shaft_speed=1e5, d_shaft_speed=1e4)
OBS_SCALE = np.array([1e4, 1e4, np.pi, 1e3, 1e3, 1e3, 1e4, 1e4, np.pi, 1e3])


def golden(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)


def golden_names(prefix):
    return sorted(os.path.basename(f)[:-4] for f in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


def params_for(mode_row=None, **over):
    p = dict(so.DEFAULT_PARAMS)
    if mode_row is not None:
        p["shaft_generator_state"] = int(mode_row[0])
        p["main_engine_capacity"] = float(mode_row[1])
        p["electrical_capacity"] = float(mode_row[2])
    p.update(over)
    return p


def init_rows(poses, omega0=OMEGA0, v_des=8.5, pi2=114.0):
    """init[n_env, 2, NF] from per-ship poses [n_env, 2, 6]."""
    poses = np.asarray(poses, dtype=np.float64)
    n_env = poses.shape[0]
    init = np.zeros((n_env, 2, len(so.INIT_FIELDS)))
    init[:, :, :6] = poses
    init[:, :, 6] = omega0
    init[:, :, 7] = v_des
    init[:, :, 9] = pi2
    return init


def sim_scale(d):
    return SCALE_SIMPL if "simplified" in d.files else SCALE


def sim_params(d, **over):
    """Oracle parameters of a sim_* fixture: its machinery mode, and for the SimplifiedMachineryModel
    fixtures (key "simplified" = time constant, throttle kp, ki) that model."""
    p = params_for(d["mode"] if "mode" in d.files else None, **over)
    if "simplified" in d.files:
        tau, kp, ki = (float(x) for x in d["simplified"])
        p.update(machinery_model=so.MACH_SIMPLIFIED, thrust_force_dynamic_time_constant=tau, kp_ship_speed=kp,
                 ki_ship_speed=ki)
    return p


def sim_init(d, poses):
    """init rows for a sim_* fixture (desired speed, initial shaft speed / thrust, shaft PI integral)."""
    if "simplified" in d.files:
        return init_rows(poses, omega0=float(d["pre_shaft_speed"][0]), v_des=float(d["v_des"]), pi2=0.0)
    return init_rows(poses)


def sim_oracle(d):
    """Oracle with one env whose two ships both carry the fixture's ship."""
    route = d["route"]
    nr = int(d["n_route"])
    routes = np.stack([route, route])[None]
    n_wpt = np.array([[nr, nr]])
    pose = d["pose"] if "pose" in d.files else np.zeros(6)
    init = sim_init(d, np.stack([pose, pose])[None])
    return so.OracleEnvs(sim_params(d), routes, n_wpt, init, POLYS)


def sim_state_from(d, prefix, i, oracle):
    """Put fixture ship state (prefix 'pre_' or 'post_', row i) into both ship slots."""
    st = oracle.get_state()
    for k in SIM_FIELDS:
        st[k][:] = d[prefix + k][i]
    return st


def env_oracle(d, n_env=1):
    routes = np.repeat(d["routes"][None], n_env, axis=0)
    n_wpt = np.repeat(d["n_wpt"][None], n_env, axis=0)
    init = init_rows(np.repeat(d["pose"][None], n_env, axis=0))
    return so.OracleEnvs(params_for(d["mode"]), routes, n_wpt, init, POLYS)


ENV_STATE_SHIP = so.SHIP_REAL + so.SHIP_INT
ENV_STATE_ENV = ("sampling_dist", "eps_dist", "prev_pre_north", "prev_pre_east", "iw_north", "iw_east")


def env_state_from(d, prefix, i, oracle):
    """Oracle state dict from an env fixture row (pre_/post_ snapshot of the reference)."""
    st = oracle.get_state()
    for k in ENV_STATE_SHIP:
        st[k][:, 0] = d[prefix + k][i]
    for k in ENV_STATE_ENV:
        st[k][0] = d[prefix + k][i]
    cap = oracle.cap
    st["wpt_north"][:, :, 0] = d[prefix + "wpt_north"][i][:, :cap]
    st["wpt_east"][:, :, 0] = d[prefix + "wpt_east"][i][:, :cap]
    return st


def env_state_all_rows(d, prefix, oracle):
    """Oracle state with env j = fixture row j (for batched teacher forcing)."""
    st = oracle.get_state()
    for k in ENV_STATE_SHIP:
        st[k][:] = d[prefix + k].T
    for k in ENV_STATE_ENV:
        st[k][:] = d[prefix + k]
    cap = oracle.cap
    st["wpt_north"][:] = np.transpose(d[prefix + "wpt_north"][:, :, :cap], (1, 2, 0))
    st["wpt_east"][:] = np.transpose(d[prefix + "wpt_east"][:, :, :cap], (1, 2, 0))
    return st


def sim_state_all_rows(d, prefix, oracle):
    st = oracle.get_state()
    for k in SIM_FIELDS:
        st[k][:] = d[prefix + k][None, :]
    return st


def sim_oracle_batch(d, n_env):
    route = d["route"]
    nr = int(d["n_route"])
    routes = np.repeat(np.stack([route, route])[None], n_env, axis=0)
    n_wpt = np.full((n_env, 2), nr)
    pose = d["pose"] if "pose" in d.files else np.zeros(6)
    init = sim_init(d, np.repeat(np.stack([pose, pose])[None], n_env, axis=0))
    return so.OracleEnvs(sim_params(d), routes, n_wpt, init, POLYS)


def rel_err(a, b, scale):
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    return np.abs(a - b) / np.maximum(np.abs(b), scale)
