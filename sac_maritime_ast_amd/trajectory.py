"""Trajectory and logging formats of the reference, from the device-side rollout outputs.

The reference logs every step of every ship into ``ShipModelAST.simulation_results`` (a dict of
27 lists, ship_model.py:645-700; plotted by test_beds/*), the env's per-episode running reward
components into ``MultiShipRLEnv.reward_results`` (MSRL_env_ex.py:926-964), and the driver keeps
per-episode action records (test_beds/main_ast.py:369-375: [time, scoping angle in degrees,
IW north, IW east] on sampling events).  The HIP rollout writes the same quantities for all envs
as strided device buffers (``VecMultiShipRLEnv.rollout(..., log=True)``: log[K, 62, n_env]);
this module turns one env's rows back into the reference's containers and saves whole
trajectories as .npz.
"""
from __future__ import annotations

import numpy as np

from . import _lib

LOG_KEYS = ("time [s]", "north position [m]", "east position [m]", "yaw angle [deg]", "rudder angle [deg]",
            "forward speed [m/s]", "sideways speed [m/s]", "yaw rate [deg/sec]", "propeller shaft speed [rpm]",
            "commanded load fraction me [-]", "commanded load fraction hsg [-]", "power me [kw]",
            "available power me [kw]", "power electrical [kw]", "available power electrical [kw]", "power [kw]",
            "propulsion power [kw]", "fuel rate me [kg/s]", "fuel rate hsg [kg/s]", "fuel rate [kg/s]",
            "fuel consumption me [kg]", "fuel consumption hsg [kg]", "fuel consumption [kg]", "motor torque [Nm]",
            "thrust force [kN]", "cross track error [m]", "heading error [deg]")
REWARD_SERIES = (("test_ship", "reward_e_ct"), ("test_ship", "reward_near_col"), ("test_ship", "total_non_terminal"),
                 ("obs_ship", "reward_base"), ("obs_ship", "reward_e_ct"), ("obs_ship", "reward_near_col"),
                 ("obs_ship", "total_non_terminal"), ("shared", "total_non_terminal"))
assert len(LOG_KEYS) == _lib.SIT_LOG_KEYS and 2 * len(LOG_KEYS) + len(REWARD_SERIES) == _lib.SIT_LOG_ROWS


def _np(x):
    return x.detach().cpu().numpy() if hasattr(x, "detach") else np.asarray(x)


def simulation_results(log, env: int, ship: int = 0) -> dict:
    """ShipModelAST.simulation_results of one env's ship (0 = under test, 1 = obstacle) over the
    logged steps: {key: np.ndarray[K]} with the reference's key names."""
    lg = _np(log)
    base = ship * len(LOG_KEYS)
    return {k: lg[:, base + i, env].copy() for i, k in enumerate(LOG_KEYS)}


def reward_results(log, env: int, episode_start=None) -> dict:
    """MultiShipRLEnv.reward_results of one env: running sums of the per-step reward components,
    restarted at every episode start (reset() re-creates the lists, MSRL_env_ex.py:133-141).
    episode_start: bool[K] marking the first step of an episode (e.g. the step after a done)."""
    lg = _np(log)
    terms = lg[:, 2 * len(LOG_KEYS):, env]
    K = terms.shape[0]
    starts = np.zeros(K, bool) if episode_start is None else np.asarray(episode_start, bool)
    out = {"test_ship": {}, "obs_ship": {}, "shared": {}}
    acc = np.zeros(terms.shape[1])
    cum = np.zeros_like(terms)
    for k in range(K):
        if starts[k]:
            acc = np.zeros(terms.shape[1])
        acc = acc + terms[k]
        cum[k] = acc
    for j, (who, name) in enumerate(REWARD_SERIES):
        out[who][name] = cum[:, j]
    return out


def episode_starts(done) -> np.ndarray:
    """First step of each episode of an auto-reset rollout: the step after a done (done [K, n])."""
    d = _np(done).astype(bool)
    s = np.zeros_like(d)
    s[1:] = d[:-1]
    return s


def action_records(out: dict, env: int, log=None) -> np.ndarray:
    """test_beds/main_ast.py:369-375 records of one env: [time, scoping angle (deg), IW north,
    IW east] for every sampling event (rows of action[..., 3] == 1).  The time is the obstacle
    ship's simulator time of the step (from the log when given, else the step index * dt)."""
    act = _np(out["action"])[:, env]
    sel = act[:, 3] > 0.5
    if log is not None:
        t = _np(log)[:, len(LOG_KEYS), env]
    else:
        t = np.arange(act.shape[0]) * 0.5
    return np.stack([t[sel], np.degrees(act[sel, 2]), act[sel, 0], act[sel, 1]], axis=1)


def save_npz(path: str, out: dict, **extra) -> None:
    """A rollout's device outputs (next_state, reward, done, status, action, log, transitions)
    as a compressed .npz with the log's key names."""
    arrays = {k: _np(v) for k, v in out.items() if v is not None}
    arrays["log_keys"] = np.asarray(LOG_KEYS)
    arrays["reward_series"] = np.asarray(["/".join(s) for s in REWARD_SERIES])
    arrays.update({k: np.asarray(v) for k, v in extra.items()})
    np.savez_compressed(path, **arrays)
