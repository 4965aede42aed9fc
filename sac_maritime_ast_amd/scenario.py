"""Synthetic benchmark scenario.

The reference's route files are referenced by absolute Windows paths and are not in the
repository (test_beds/main_ast.py:221, test_beds/test_policy.py:210), so the benchmark uses
synthetic routes validated against the island map of test_beds/test_policy.py:189-194:
  test ship  R_test = [[1200,500],[1500,4500],[3500,7000],[7000,9000],[9500,9000]] (north, east)
  obstacle   R_obs  = [[2200,5300],[8600,5200]] (start -> end pair, MSRL_env_ex.py:464)
Initial state u = v = r = 0, shaft speed 400*pi/30, shaft-speed PI integral 114,
desired speed 8.5 m/s; for N > 1 envs each ship's start is jittered by +-100 m and +-0.05 rad.
The jitter of env g is a pure function of (seed, g) (splitmix64), so a shard of envs
[offset, offset + n) on one GPU equals the same envs of a single large run.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from ._lib import INIT_FIELDS

R_TEST = [[1200.0, 500.0], [1500.0, 4500.0], [3500.0, 7000.0], [7000.0, 9000.0], [9500.0, 9000.0]]
R_OBS = [[2200.0, 5300.0], [8600.0, 5200.0]]
# PolygonObstacle vertex lists, (east, north) tuples (test_beds/test_policy.py:189-194)
ISLANDS = [
    [(0, 10000), (5500, 10000), (5300, 9000), (4800, 8500), (4200, 7300), (4000, 5700), (4300, 4900),
     (4900, 4400), (4400, 4000), (3200, 4100), (2000, 4500), (1000, 4000), (900, 3500), (500, 2600),
     (0, 2350)],
    [(10000, 0), (4000, 0), (4250, 250), (5000, 400), (6000, 900), (8000, 1100), (8500, 1500),
     (9000, 2250), (9500, 3500), (10000, 4000)],
    [(5500, 5500), (5700, 7000), (6200, 8100), (7500, 8000), (7800, 7000), (7600, 5500), (6900, 4700),
     (6000, 5000)],
    [(2000, 2000), (2500, 2300), (4000, 2500), (5000, 3000), (4200, 2100), (3400, 1900)],
]
OMEGA0 = 400 * math.pi / 30
V_DES = 8.5
SHAFT_PI_I0 = 114.0


@dataclass
class Scenario:
    routes: np.ndarray   # float64[n_env, 2, cap, 2] (north, east)
    n_wpt: np.ndarray    # int32[n_env, 2]
    init: np.ndarray     # float64[n_env, 2, SIT_INIT_NF]
    polys: list          # list of float64[m, 2] (east, north)

    @property
    def n_env(self):
        return self.routes.shape[0]


def polygons(islands=ISLANDS):
    return [np.asarray(p, dtype=np.float64) for p in islands]


def heading(a, b):
    return math.atan2(b[1] - a[1], b[0] - a[0])


_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & _M64
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & _M64
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & _M64
    return z ^ (z >> np.uint64(31))


def env_uniform(seed: int, env_ids: np.ndarray, k: int) -> np.ndarray:
    """k-th uniform [0,1) draw of each env id, independent of how envs are sharded."""
    with np.errstate(over="ignore"):
        base = _splitmix64(np.uint64(seed & 0xFFFFFFFFFFFFFFFF) ^ np.uint64(0x5CE7A710))
        x = _splitmix64(base ^ (env_ids.astype(np.uint64) * np.uint64(0x100000001B3) + np.uint64(k)))
    return (x >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


def make_scenario(n_env: int, cap: int = 32, seed: int = 25450, jitter: bool = True,
                  r_test=R_TEST, r_obs=R_OBS, v_des: float = V_DES, env_offset: int = 0) -> Scenario:
    routes = np.zeros((n_env, 2, cap, 2))
    routes[:, 0, :len(r_test)] = r_test
    routes[:, 1, :len(r_obs)] = r_obs
    n_wpt = np.zeros((n_env, 2), dtype=np.int32)
    n_wpt[:, 0], n_wpt[:, 1] = len(r_test), len(r_obs)
    init = np.zeros((n_env, 2, len(INIT_FIELDS)))
    for t, r in enumerate((r_test, r_obs)):
        init[:, t, 0], init[:, t, 1] = r[0]
        init[:, t, 2] = heading(r[0], r[1])
    init[:, :, 6] = OMEGA0
    init[:, :, 7] = v_des
    init[:, :, 9] = SHAFT_PI_I0
    if jitter and (n_env > 1 or env_offset > 0):
        ids = np.arange(env_offset, env_offset + n_env, dtype=np.uint64)
        for t in range(2):
            init[:, t, 0] += 200.0 * env_uniform(seed, ids, 3 * t) - 100.0
            init[:, t, 1] += 200.0 * env_uniform(seed, ids, 3 * t + 1) - 100.0
            init[:, t, 2] += 0.1 * env_uniform(seed, ids, 3 * t + 2) - 0.05
    return Scenario(routes, n_wpt, init, polygons())
