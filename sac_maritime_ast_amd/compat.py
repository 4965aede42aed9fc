"""Scalar drop-in with the reference's exact ``MultiShipRLEnv`` surface.

``MultiShipRLEnv.reset() -> np.float32[10]``, ``init_step() -> None`` and
``step(converted_action, SAC_update, init) -> (list[10] of float, float, bool, str)`` behave
like RLEnv/MSRL_Env.py:147-442 + RLEnv/MSRL_env_ex.py:906-980, backed by a one-env
``VecMultiShipRLEnv`` on the GPU.  Attributes read by the reference's callers are provided:
``AB_segment_length``, ``AB_alpha`` (MSRL_Env.py:127-128), ``sampling_distance_travelled``,
``observation_space``/``action_space`` bounds (:69-85).
"""
from __future__ import annotations

import math
from types import SimpleNamespace

import numpy as np
import torch

from .env import VecMultiShipRLEnv
from .scenario import Scenario, make_scenario
from .status import status_string


class _Box(SimpleNamespace):
    pass


class MultiShipRLEnv:
    def __init__(self, scenario: Scenario | None = None, params=None, precision: int = 64,
                 wpt_capacity: int = 32, device=None, args=None):
        if scenario is None:
            scenario = make_scenario(1, cap=wpt_capacity, jitter=False)
        if args is not None and params is not None:
            params.sampling_frequency = int(args.sampling_frequency)
            params.theta = float(args.theta)
        self.vec = VecMultiShipRLEnv(scenario=scenario, params=params, precision=precision, device=device)
        p = self.vec.params
        r = scenario.routes[0, 1]
        nw = int(scenario.n_wpt[0, 1])
        dn, de = r[nw - 1, 0] - r[0, 0], r[nw - 1, 1] - r[0, 1]
        self.AB_distance = math.sqrt(dn ** 2 + de ** 2)
        self.AB_segment_length = self.AB_distance / p.sampling_frequency
        self.AB_alpha = math.atan2(de, dn)
        self.AB_beta = math.pi / 2 - self.AB_alpha
        self.theta = p.theta
        self.e_tolerance = p.e_tolerance
        self.observation_space = _Box(
            low=np.array([0, 0, -np.pi, -3000, 0, 0, 0, 0, -np.pi, 0], dtype=np.float32),
            high=np.array([10000, 20000, np.pi, 3000, 1000, 2000, 10000, 20000, np.pi, 1000], dtype=np.float32))
        self.action_space = _Box(low=np.array([-np.pi / 6], dtype=np.float32),
                                 high=np.array([np.pi / 6], dtype=np.float32))
        self.np_random = np.random.default_rng()

    def seed(self, seed=None):
        self.np_random = np.random.default_rng(seed)

    def reset(self):
        return self.vec.reset()[0].cpu().numpy().astype(np.float32)

    def init_step(self):
        self.vec.init_step()

    def step(self, converted_action, SAC_update, init):
        a = torch.tensor([[float(converted_action[0]), float(converted_action[1])]], dtype=torch.float64)
        ns, rew, done, st = self.vec.step(a, [bool(SAC_update)], [bool(init)])
        return ([float(x) for x in ns[0].cpu().tolist()], float(rew[0].item()), bool(done[0].item()),
                status_string(int(st[0].item())))

    @property
    def sampling_distance_travelled(self):
        return float(self.vec.get_state()["sampling_dist"][0].item())

    @property
    def eps_distance_travelled(self):
        return float(self.vec.get_state()["eps_dist"][0].item())
