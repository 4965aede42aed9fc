"""Scalar drop-in with the reference's exact ``MultiShipRLEnv`` surface.

``MultiShipRLEnv.reset() -> np.float32[10]``, ``init_step() -> None`` and
``step(converted_action, SAC_update, init) -> (list[10] of float, float, bool, str)`` behave
like RLEnv/MSRL_Env.py:147-442 + RLEnv/MSRL_env_ex.py:906-980, backed by a one-env
``VecMultiShipRLEnv`` on the GPU.  Attributes read by the reference's callers are provided:
``AB_distance``, ``AB_segment_length``, ``AB_alpha``, ``AB_beta`` (MSRL_Env.py:119-128),
``e_tolerance``, ``theta``, ``sampling_distance_travelled``, ``eps_distance_travelled``,
``state``, ``initial_state`` (:88-92) and ``observation_space``/``action_space`` bounds (:69-85).

``make_gpu_env`` builds it from the reference's own configuration objects (the NamedTuples of
test_beds/test_policy.py:94-226), routes and island vertex lists; INTEGRATION.md shows the binding.
"""
from __future__ import annotations

import math
from types import SimpleNamespace

import numpy as np
import torch

from . import _lib
from .config import params_from_reference
from .env import VecMultiShipRLEnv
from .scenario import Scenario, make_scenario, polygons
from .status import status_string


class _Box(SimpleNamespace):
    pass


class MultiShipRLEnv:
    """One two-ship env with the reference's scalar API (float64 by default: the reference's
    arithmetic).  A step is one host->device copy of the 18-byte action record, one kernel launch
    and one device->host copy of the outputs."""

    def __init__(self, scenario: Scenario | None = None, params=None, precision: int = 64,
                 wpt_capacity: int = 32, device=None, args=None):
        if scenario is None:
            scenario = make_scenario(1, cap=wpt_capacity, jitter=False)
        if scenario.n_env != 1:
            raise ValueError("MultiShipRLEnv is one env; use VecMultiShipRLEnv for batches")
        if args is not None and params is not None:
            params.sampling_frequency = int(args.sampling_frequency)
            params.theta = float(args.theta)
        self.vec = VecMultiShipRLEnv(scenario=scenario, params=params, precision=precision, device=device)
        p = self.vec.params
        r = scenario.routes[0, 1]
        nw = int(scenario.n_wpt[0, 1])
        # reward_function_params (MSRL_Env.py:119-128)
        self.AB_distance_n = float(r[nw - 1, 0] - r[0, 0])
        self.AB_distance_e = float(r[nw - 1, 1] - r[0, 1])
        self.AB_distance = math.sqrt(self.AB_distance_n ** 2 + self.AB_distance_e ** 2)
        self.AB_segment_length = self.AB_distance / p.sampling_frequency
        self.AB_alpha = math.atan2(self.AB_distance_e, self.AB_distance_n)
        self.AB_beta = math.pi / 2 - self.AB_alpha
        self.theta = p.theta
        self.e_tolerance = p.e_tolerance
        self.observation_space = _Box(
            low=np.array([0, 0, -np.pi, -3000, 0, 0, 0, 0, -np.pi, 0], dtype=np.float32),
            high=np.array([10000, 20000, np.pi, 3000, 1000, 2000, 10000, 20000, np.pi, 1000], dtype=np.float32))
        self.action_space = _Box(low=np.array([-np.pi / 6], dtype=np.float32),
                                 high=np.array([np.pi / 6], dtype=np.float32))
        self.np_random = np.random.default_rng()
        # the construction-time observation (MSRL_Env.py:88-92): float32
        i = scenario.init[0]
        self.initial_state = np.array([i[0, 0], i[0, 1], i[0, 2], 0, 0, 0, i[1, 0], i[1, 1], i[1, 2], 0],
                                      dtype=np.float32)
        self.state = self.initial_state
        # per-step staging: inputs [action (2 reals) | sac u8 | init u8], outputs
        # [next_state (10 reals) | reward | status i32 | done u8 | done-count i32]
        rs = 8 if precision == 64 else 4
        self._rs, self._np_real = rs, (np.float64 if precision == 64 else np.float32)
        dev = self.vec.device
        self._in_host = torch.zeros(2 * rs + 2, dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        self._in_dev = torch.zeros(2 * rs + 2, dtype=torch.uint8, device=dev)
        self._o_ns, self._o_rw = 0, 10 * rs
        self._o_st = 11 * rs
        self._o_dn = 11 * rs + 4
        self._out_dev = torch.zeros(11 * rs + 8, dtype=torch.uint8, device=dev)

    def seed(self, seed=None):
        """Seeds ``np_random`` as the reference's ``seed`` does (MSRL_Env.py:444-446, gymnasium's
        ``seeding.np_random``).  As in the reference, nothing on the step path draws from it: the
        caller chooses the actions; the batched envs' on-device sampler is keyed by its rollout
        seed (``VecMultiShipRLEnv.rollout(seed=...)``)."""
        self.np_random = np.random.default_rng(seed)
        return [seed]

    def reset(self):
        """MultiShipRLEnv.reset (MSRL_Env.py:147-188): the construction-time observation."""
        self.vec.reset()
        self.state = self.initial_state
        return self.initial_state.copy()

    def init_step(self):
        """MultiShipRLEnv.init_step (MSRL_Env.py:190-217)."""
        self.vec.init_step()

    def step(self, converted_action, SAC_update, init):
        """MultiShipRLEnv.step (MSRL_Env.py:404-442): returns (next_state list of 10 float,
        reward float, done bool, status str)."""
        rs = self._rs
        inp = self._in_host.numpy()
        inp[:2 * rs].view(self._np_real)[:] = (float(converted_action[0]), float(converted_action[1]))
        inp[2 * rs] = 1 if SAC_update else 0
        inp[2 * rs + 1] = 1 if init else 0
        self._in_dev.copy_(self._in_host, non_blocking=True)
        base_in, base_out = self._in_dev.data_ptr(), self._out_dev.data_ptr()
        with torch.cuda.device(self.vec.device):
            self.vec._call("sit_step", base_in, base_in + 2 * rs, base_in + 2 * rs + 1, base_out + self._o_ns,
                           base_out + self._o_rw, base_out + self._o_dn, base_out + self._o_st, None,
                           self.vec._stream())
        out = self._out_dev.cpu().numpy()
        ns = out[:10 * rs].view(self._np_real)
        reward = float(out[self._o_rw:self._o_rw + rs].view(self._np_real)[0])
        status = int(out[self._o_st:self._o_st + 4].view(np.uint32)[0])
        next_state = [float(x) for x in ns]
        self.state = next_state
        return next_state, reward, bool(out[self._o_dn]), status_string(status)

    @property
    def sampling_distance_travelled(self):
        return float(self.vec.get_state()["sampling_dist"][0].item())

    @property
    def eps_distance_travelled(self):
        return float(self.vec.get_state()["eps_dist"][0].item())


def make_gpu_env(ship_config, env_config, sim_config_test, sim_config_obs, machinery_config, throttle_gains,
                 heading_gains, los_params, route_test, route_obs, obstacle_vertices, args,
                 desired_speed=(8.5, 8.5), omega0=400 * np.pi / 30, shaft_speed_i0=114.0, wpt_capacity=32,
                 precision=64, device=None) -> MultiShipRLEnv:
    """The drop-in env from the reference's configuration objects (test_beds/test_policy.py:94-226):
    ShipConfiguration, EnvironmentConfiguration, the two SimulationConfiguration (initial poses),
    MachinerySystemConfiguration, ThrottleControllerGains, HeadingControllerGains, LosParameters,
    the two routes as [[north, east], ...], the PolygonObstacle vertex lists ((east, north) tuples)
    and the env ``args`` (sampling_frequency, theta).  ``desired_speed`` is ShipAssets.
    desired_forward_speed per ship, ``omega0`` the initial shaft speed (ship_model.py:567) and
    ``shaft_speed_i0`` the shaft-speed PI's initial integral (controllers.py:119, 129)."""
    p = params_from_reference(ship_config, env_config, sim_config_test, machinery_config, throttle_gains,
                              heading_gains, los_params, args)
    routes = np.zeros((1, 2, wpt_capacity, 2))
    routes[0, 0, :len(route_test)] = route_test
    routes[0, 1, :len(route_obs)] = route_obs
    n_wpt = np.array([[len(route_test), len(route_obs)]], dtype=np.int32)
    init = np.zeros((1, 2, len(_lib.INIT_FIELDS)))
    for t, sc in enumerate((sim_config_test, sim_config_obs)):
        init[0, t, :6] = (sc.initial_north_position_m, sc.initial_east_position_m, sc.initial_yaw_angle_rad,
                          sc.initial_forward_speed_m_per_s, sc.initial_sideways_speed_m_per_s,
                          sc.initial_yaw_rate_rad_per_s)
        init[0, t, 6:10] = (omega0, desired_speed[t], 0.0, shaft_speed_i0)
    scen = Scenario(routes, n_wpt, init, polygons(obstacle_vertices))
    return MultiShipRLEnv(scenario=scen, params=p, precision=precision, device=device)
