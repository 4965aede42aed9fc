"""Scalar drop-in with the reference's exact ``MultiShipRLEnv`` surface.

Constructed like the reference (RLEnv/MSRL_Env.py:42-116)::

    env = MultiShipRLEnv([test, obs], map, ship_draw, time_since_last_ship_drawing, args)

from the reference's own objects: two ``ShipAssets`` (MSRL_Env.py:25-35) holding a ``ShipModelAST``
(ship_model.py:545-574) with its ``ShipMachineryModel`` (ship_engine.py:298-353), an
``EngineThrottleFromSpeedSetPoint`` (controllers.py:108-151) and a ``HeadingBySampledRouteController``
(controllers.py:253-350), a ``PolygonObstacle`` (obstacle.py:92-124) and the env ``args``
(sampling_frequency, theta).  The objects are read duck-typed, attribute by attribute (the paths are
listed in ``ASSET_PATHS``; any object with the same attributes works), never called.

``reset() -> np.float32[10]``, ``init_step() -> None`` and ``step(converted_action, SAC_update, init)
-> (list[10] of float, float, bool, str)`` behave like MSRL_Env.py:147-442 + MSRL_env_ex.py:906-980,
backed by a one-env ``VecMultiShipRLEnv`` on the GPU (one host->device copy, one kernel launch, one
device->host copy per step).  Attributes the reference's callers read are provided: ``AB_distance``,
``AB_segment_length``, ``AB_alpha``, ``AB_beta`` (MSRL_Env.py:119-128), ``e_tolerance``, ``theta``,
``sampling_distance_travelled``, ``eps_distance_travelled``, ``state``, ``initial_state`` (:88-92),
``observation_space`` / ``action_space`` (:69-85), ``map``, ``args``, ``ship_draw``,
``time_since_last_ship_drawing``, ``prev_route_coordinate``, ``reward_results`` (MSRL_env_ex.py:
133-141, 926-964), and ``test`` / ``obs`` / ``assets``: live views of the device state with the
reference's attribute names (``test.ship_model.north``, ``obs.ship_model.int.time``,
``obs.auto_pilot.navigate.north``, ``obs.throttle_controller.shaft_speed_controller.error_i``,
``test.ship_model.simulation_results``, ...; the table is ``ShipAssetsView``).  Assigning one of the
state attributes writes it to the device, as assigning the reference object's attribute changes
the next step.

``make_gpu_env`` builds the same env from the reference's configuration NamedTuples
(test_beds/test_policy.py:94-226) instead of constructed objects; INTEGRATION.md shows the binding.
"""
from __future__ import annotations

import math
from ctypes import c_void_p
from functools import lru_cache
from types import SimpleNamespace

import numpy as np
import torch

from . import _lib
from .config import params as default_params
from .config import params_from_reference
from .env import LO_FIELDS, VecMultiShipRLEnv
from .scenario import Scenario, polygons
from .status import status_string
from .trajectory import LOG_KEYS, REWARD_SERIES

_status_string = lru_cache(maxsize=8192)(status_string)   # the per-step status decode, memoised

_REQUIRED = object()

# Every attribute the adapter reads from a ShipAssets, relative to the asset (MSRL_Env.py:25-35),
# with the reference line that defines it.  (tests/golden/make_golden.py records these paths on the
# reference's own objects: tests/golden/asset_paths.json.)
SHIP_CONFIG_FIELDS = (       # ShipConfiguration (ship_model.py:20-35), kept as ship_model.ship_config (:66)
    "dead_weight_tonnage", "coefficient_of_deadweight_to_displacement", "bunkers", "ballast", "length_of_ship",
    "width_of_ship", "added_mass_coefficient_in_surge", "added_mass_coefficient_in_sway",
    "added_mass_coefficient_in_yaw", "mass_over_linear_friction_coefficient_in_surge",
    "mass_over_linear_friction_coefficient_in_sway", "mass_over_linear_friction_coefficient_in_yaw",
    "nonlinear_friction_coefficient__in_surge", "nonlinear_friction_coefficient__in_sway",
    "nonlinear_friction_coefficient__in_yaw")
ENV_CONFIG_FIELDS = ("current_velocity_component_from_north", "current_velocity_component_from_east",
                     "wind_speed", "wind_direction")        # EnvironmentConfiguration (ship_model.py:38-42)
POSE_FIELDS = ("north", "east", "yaw_angle", "forward_speed", "sideways_speed", "yaw_rate")   # ship_model.py:159-164
ASSET_PATHS = (
    *[f"ship_model.ship_config.{f}" for f in SHIP_CONFIG_FIELDS],
    *[f"ship_model.environment_config.{f}" for f in ENV_CONFIG_FIELDS],
    "ship_model.simulation_config.integration_step",                     # ship_model.py:176
    # wind model constants of BaseShipModel (ship_model.py:184-191)
    "ship_model.rho_a", "ship_model.h_f", "ship_model.h_s", "ship_model.cx", "ship_model.cy", "ship_model.cn",
    # the construction pose reset() restores (ship_model.py:103-108, 368-373) and the live pose
    *[f"ship_model.init_{f}" for f in POSE_FIELDS], *[f"ship_model.{f}" for f in POSE_FIELDS],
    "ship_model.int.time",                                               # utils.py:23, 42-48
    # ShipMachineryModel (ship_engine.py:177-230, 298-325)
    "ship_model.ship_machinery_model.hotel_load",
    "ship_model.ship_machinery_model.mode.main_engine_capacity",
    "ship_model.ship_machinery_model.mode.electrical_capacity",
    "ship_model.ship_machinery_model.mode.shaft_generator_state",
    "ship_model.ship_machinery_model.w_rated_me", "ship_model.ship_machinery_model.d_me",
    "ship_model.ship_machinery_model.d_hsg", "ship_model.ship_machinery_model.r_me",
    "ship_model.ship_machinery_model.r_hsg", "ship_model.ship_machinery_model.jp",
    "ship_model.ship_machinery_model.kp", "ship_model.ship_machinery_model.dp",
    "ship_model.ship_machinery_model.kt", "ship_model.ship_machinery_model.c_rudder_v",
    "ship_model.ship_machinery_model.c_rudder_r", "ship_model.ship_machinery_model.omega",
    "ship_model.ship_machinery_model.fuel_coeffs_for_main_engine.a",
    "ship_model.ship_machinery_model.fuel_coeffs_for_main_engine.b",
    "ship_model.ship_machinery_model.fuel_coeffs_for_main_engine.c",
    "ship_model.ship_machinery_model.fuel_coeffs_for_diesel_gen.a",
    "ship_model.ship_machinery_model.fuel_coeffs_for_diesel_gen.b",
    "ship_model.ship_machinery_model.fuel_coeffs_for_diesel_gen.c",
    # EngineThrottleFromSpeedSetPoint's two PiControllers (controllers.py:45-62, 114-136)
    "throttle_controller.ship_speed_controller.kp", "throttle_controller.ship_speed_controller.ki",
    "throttle_controller.ship_speed_controller.error_i",
    "throttle_controller.shaft_speed_controller.kp", "throttle_controller.shaft_speed_controller.ki",
    "throttle_controller.shaft_speed_controller.error_i",
    # HeadingBySampledRouteController (controllers.py:253-296): PID, LOS, waypoint index, route
    "auto_pilot.heading_controller.max_rudder_angle",
    "auto_pilot.heading_controller.ship_heading_controller.kp",
    "auto_pilot.heading_controller.ship_heading_controller.kd",
    "auto_pilot.heading_controller.ship_heading_controller.ki",
    "auto_pilot.heading_controller.ship_heading_controller.error_i",
    "auto_pilot.heading_controller.ship_heading_controller.prev_error",
    "auto_pilot.next_wpt",
    "auto_pilot.navigate.ra", "auto_pilot.navigate.r", "auto_pilot.navigate.ki",
    "auto_pilot.navigate.integrator_limit", "auto_pilot.navigate.e_ct_int",     # LOS_guidance.py:46-61
    "auto_pilot.navigate.init_route", "auto_pilot.navigate.north", "auto_pilot.navigate.east",
    # ShipAssets fields (MSRL_Env.py:30-34)
    "desired_forward_speed", "stop_flag",
)
# optional: ShipMachineryModel.hotel_load exists only for a truthy hotel load (ship_engine.py:190-191);
# a SimplifiedMachineryModel (ship_engine.py:398-428) has thrust / thrust_time_constant instead of a shaft
_OPTIONAL = {"ship_model.ship_machinery_model.hotel_load": 0.0}
_SIMPLIFIED_PATHS = ("ship_model.ship_machinery_model.thrust", "ship_model.ship_machinery_model.thrust_time_constant")
_SHAFT_ONLY = {p for p in ASSET_PATHS if p.split(".")[-1] in (
    "w_rated_me", "d_me", "d_hsg", "r_me", "r_hsg", "jp", "kp", "dp", "kt", "omega")
    and p.startswith("ship_model.ship_machinery_model.")} | {
    "throttle_controller.shaft_speed_controller.kp", "throttle_controller.shaft_speed_controller.ki",
    "throttle_controller.shaft_speed_controller.error_i"}


def _get(obj, path: str, default=_REQUIRED, who: str = "asset"):
    cur = obj
    for part in path.split("."):
        if isinstance(cur, dict) and part in cur:
            cur = cur[part]
            continue
        if not hasattr(cur, part):
            if default is not _REQUIRED:
                return default
            raise AttributeError(f"{who}.{path}: the reference object has no attribute {part!r} "
                                 f"(MultiShipRLEnv reads the attributes listed in compat.ASSET_PATHS)")
        cur = getattr(cur, part)
    return cur


def read_asset(asset, who: str = "asset") -> dict:
    """The values of every ASSET_PATHS attribute of one ShipAssets (duck-typed)."""
    simpl = hasattr(_get(asset, "ship_model.ship_machinery_model", who=who), "thrust_time_constant")
    vals = {}
    for p in ASSET_PATHS:
        if simpl and p in _SHAFT_ONLY:
            continue
        vals[p] = _get(asset, p, _OPTIONAL.get(p, _REQUIRED), who)
    if simpl:
        for p in _SIMPLIFIED_PATHS:
            vals[p] = _get(asset, p, who=who)
    return vals


def _unscaled(y: float, div: float) -> float:
    """The x whose x * pi / div (how the reference converts degrees to radians, test_policy.py:223,
    and rpm to rad/s, ship_engine.py:316) is exactly y: the round-trip value, snapped to a short
    decimal when that reproduces y."""
    x0 = y * div / math.pi
    for x in [round(x0, 9), x0] + [float(np.nextafter(x0, x0 + s * 1e9)) for s in (1, -1)]:
        if x * math.pi / div == y:
            return x
    return x0


def _degrees_of(rad: float) -> float:
    return _unscaled(rad, 180.0)


def _route_of(data) -> np.ndarray:
    """NavigationSystem.load_waypoints (LOS_guidance.py:65-86): a route file path or an array of
    (north, east) rows."""
    if isinstance(data, str):
        data = np.loadtxt(data)
    a = np.asarray(data, dtype=np.float64)
    return a.reshape(-1, 2)


def _polygons_of(m) -> list:
    """The vertex lists ((east, north) tuples) of a PolygonObstacle (obstacle.py:98-109: shapely
    Polygons in .polygons, their rings in .exterior.coords, closed by a repeated first vertex), or of
    a plain list of vertex lists."""
    if hasattr(m, "polygons"):
        out = []
        for poly in m.polygons:
            c = np.asarray(list(poly.exterior.coords), dtype=np.float64)
            if len(c) > 1 and np.array_equal(c[0], c[-1]):
                c = c[:-1]
            out.append(c)
        return out
    return [np.asarray(p, dtype=np.float64) for p in m]


def params_from_assets(test_vals: dict, obs_vals: dict, args=None):
    """sit_params of a two-ship env from the values read_asset() took from its ShipAssets.  Both
    ships must share every configuration value (one sit_params per handle); the poses, routes,
    desired speeds and controller states are per ship."""
    config_paths = [p for p in test_vals if not p.endswith((".error_i", ".prev_error", ".e_ct_int", ".omega",
                                                            ".thrust", ".time", "next_wpt", "init_route",
                                                            "navigate.north", "navigate.east",
                                                            "desired_forward_speed", "stop_flag"))
                    and not p.startswith(("ship_model.init_",)) and p.split(".")[-1] not in POSE_FIELDS]
    for p in config_paths:
        a, b = test_vals[p], obs_vals.get(p)
        if not (a == b or (isinstance(a, float) and isinstance(b, float) and np.isnan(a) and np.isnan(b))):
            raise ValueError(f"the two ships differ in {p} ({a!r} vs {b!r}): one handle holds one configuration")
    v = test_vals
    mm = "ship_model.ship_machinery_model."
    simpl = (mm + "thrust_time_constant") in v
    ship = SimpleNamespace(**{f: v["ship_model.ship_config." + f] for f in SHIP_CONFIG_FIELDS})
    envc = SimpleNamespace(**{f: v["ship_model.environment_config." + f] for f in ENV_CONFIG_FIELDS})
    sim = SimpleNamespace(integration_step=v["ship_model.simulation_config.integration_step"])
    mode = SimpleNamespace(main_engine_capacity=v[mm + "mode.main_engine_capacity"],
                           electrical_capacity=v[mm + "mode.electrical_capacity"],
                           shaft_generator_state=v[mm + "mode.shaft_generator_state"])
    mc = dict(hotel_load=v[mm + "hotel_load"], machinery_modes=SimpleNamespace(list_of_modes=[mode]),
              machinery_operating_mode=0,
              rudder_angle_to_sway_force_coefficient=v[mm + "c_rudder_v"],
              rudder_angle_to_yaw_force_coefficient=v[mm + "c_rudder_r"],
              max_rudder_angle_degrees=_degrees_of(float(v["auto_pilot.heading_controller.max_rudder_angle"])),
              specific_fuel_consumption_coefficients_me=SimpleNamespace(
                  **{k: v[mm + "fuel_coeffs_for_main_engine." + k] for k in "abc"}),
              specific_fuel_consumption_coefficients_dg=SimpleNamespace(
                  **{k: v[mm + "fuel_coeffs_for_diesel_gen." + k] for k in "abc"}))
    if simpl:
        mc["thrust_force_dynamic_time_constant"] = v[mm + "thrust_time_constant"]
        thr = SimpleNamespace(kp=v["throttle_controller.ship_speed_controller.kp"],
                              ki=v["throttle_controller.ship_speed_controller.ki"])
    else:
        mc.update(rated_speed_main_engine_rpm=_unscaled(float(v[mm + "w_rated_me"]), 30.0),
                  linear_friction_main_engine=v[mm + "d_me"], linear_friction_hybrid_shaft_generator=v[mm + "d_hsg"],
                  gear_ratio_between_main_engine_and_propeller=v[mm + "r_me"],
                  gear_ratio_between_hybrid_shaft_generator_and_propeller=v[mm + "r_hsg"],
                  propeller_inertia=v[mm + "jp"], propeller_speed_to_torque_coefficient=v[mm + "kp"],
                  propeller_diameter=v[mm + "dp"], propeller_speed_to_thrust_force_coefficient=v[mm + "kt"])
        thr = SimpleNamespace(**{f"{k}_{s}_speed": v[f"throttle_controller.{s}_speed_controller.{k}"]
                                 for k in ("kp", "ki") for s in ("ship", "shaft")})
    hc = "auto_pilot.heading_controller.ship_heading_controller."
    hdg = SimpleNamespace(kp=v[hc + "kp"], kd=v[hc + "kd"], ki=v[hc + "ki"])
    nav = "auto_pilot.navigate."
    los = SimpleNamespace(radius_of_acceptance=v[nav + "ra"], lookahead_distance=v[nav + "r"],
                          integral_gain=v[nav + "ki"], integrator_windup_limit=v[nav + "integrator_limit"])
    p = params_from_reference(ship, envc, sim, SimpleNamespace(**mc), thr, hdg, los, args)
    for f, path in (("rho_air", "rho_a"), ("front_height", "h_f"), ("side_height", "h_s"), ("cx", "cx"),
                    ("cy", "cy"), ("cn", "cn")):
        setattr(p, f, float(v["ship_model." + path]))
    return p


class _Box:
    """gymnasium.spaces.Box as the reference constructs it (MSRL_Env.py:69-85): low / high / shape /
    dtype, seed(), sample(), contains()."""

    def __init__(self, low, high):
        self.low, self.high = low, high
        self.shape, self.dtype = low.shape, low.dtype
        self.np_random = np.random.default_rng()

    def seed(self, seed=None):
        self.np_random = np.random.default_rng(seed)
        return [seed]

    def sample(self):
        return self.np_random.uniform(self.low, self.high).astype(self.dtype)

    def contains(self, x):
        x = np.asarray(x)
        return x.shape == self.shape and bool(np.all(x >= self.low) and np.all(x <= self.high))


# ---------------------------------------------------------------------------------------------
# live views with the reference's attribute names
# ---------------------------------------------------------------------------------------------
class _View:
    """Attributes backed by the env's device state (read: the cached state of the env; write: the
    field is written to the device) or by host values."""
    _fields: dict = {}

    def __init__(self, env, t):
        object.__setattr__(self, "_env", env)
        object.__setattr__(self, "_t", t)

    def __getattr__(self, name):
        f = type(self)._fields.get(name)
        if f is None:
            raise AttributeError(f"{type(self).__name__} has no attribute {name!r}")
        return f[0](self._env, self._t)

    def __setattr__(self, name, value):
        f = type(self)._fields.get(name)
        if f is None or len(f) < 2 or f[1] is None:
            raise AttributeError(f"{type(self).__name__}.{name} is read-only")
        f[1](self._env, self._t, value)

    def __dir__(self):
        return sorted(type(self)._fields)


def _real(field, scale=1.0):
    """A ship-state real [2, n_env] as a float attribute (scaled on read, divided on write)."""
    return (lambda env, t: env._read(field, t) * scale,
            lambda env, t, v: env._write(field, t, float(v) / scale))


class _IntView(_View):
    """ShipModelAST.int, the EulerInt (utils.py:7-53): time = the ship's ticks x dt."""
    _fields = {
        "time": (lambda env, t: int(env._state()["ticks"][t, 0]) * env._dt,
                 lambda env, t, v: env._write("ticks", t, int(round(float(v) / env._dt)))),
        "dt": (lambda env, t: env._dt,),
    }


class _MachineryView(_View):
    """ShipModelAST.ship_machinery_model: omega (shaft speed, ship_engine.py:327), or thrust for the
    SimplifiedMachineryModel (ship_engine.py:416)."""
    _fields = {"omega": _real("shaft_speed"), "thrust": _real("shaft_speed")}


class _ShipModelView(_View):
    """ShipModelAST: pose and velocities (ship_model.py:159-164), int, ship_machinery_model, the
    construction pose init_* (:103-108) and simulation_results (:645-684; recorded host-side from the
    kernel's trajectory log when the env records, else empty)."""
    _fields = {
        "north": _real("north"), "east": _real("east"), "yaw_angle": _real("yaw"),
        "forward_speed": _real("surge"), "sideways_speed": _real("sway"), "yaw_rate": _real("yaw_rate"),
        "int": (lambda env, t: _IntView(env, t),),
        "ship_machinery_model": (lambda env, t: _MachineryView(env, t),),
        "simulation_results": (lambda env, t: (env._flush(), env._sim_results[t])[1],),
        **{f"init_{f}": (lambda env, t, j=j: float(env.vec.scenario.init[0, t, j]),)
           for j, f in enumerate(POSE_FIELDS)},
    }


def _pi_view(field, kp, ki):
    cls = type("PiControllerView", (_View,), {"_fields": {
        "error_i": _real(field),
        "kp": (lambda env, t: getattr(env.vec.params, kp),),
        "ki": (lambda env, t: getattr(env.vec.params, ki),),
        "time_step": (lambda env, t: env._dt,)}})
    return cls


_ShipPi = _pi_view("ship_speed_i", "kp_ship_speed", "ki_ship_speed")
_ShaftPi = _pi_view("shaft_speed_i", "kp_shaft_speed", "ki_shaft_speed")


class _ThrottleView(_View):
    """EngineThrottleFromSpeedSetPoint (controllers.py:108-151)."""
    _fields = {"ship_speed_controller": (lambda env, t: _ShipPi(env, t),),
               "shaft_speed_controller": (lambda env, t: _ShaftPi(env, t),)}


class _PidView(_View):
    """PidController of the heading (controllers.py:72-93)."""
    _fields = {"error_i": _real("heading_i"), "prev_error": _real("heading_prev"),
               "kp": (lambda env, t: env.vec.params.heading_kp,), "kd": (lambda env, t: env.vec.params.heading_kd,),
               "ki": (lambda env, t: env.vec.params.heading_ki,), "time_step": (lambda env, t: env._dt,)}


class _HeadingView(_View):
    """HeadingByReferenceController (controllers.py:175-189)."""
    _fields = {"ship_heading_controller": (lambda env, t: _PidView(env, t),),
               "max_rudder_angle": (lambda env, t: env.vec.params.max_rudder_angle_degrees * math.pi / 180,)}


def _route_lists(env, t):
    st = env._state()
    nw = int(st["n_wpt"][t, 0])
    n = [float(x) for x in st["wpt_north"][t, :nw - 1, 0]] + [float(env.vec.scenario.routes[0, t, int(
        env.vec.scenario.n_wpt[0, t]) - 1, 0])]
    e = [float(x) for x in st["wpt_east"][t, :nw - 1, 0]] + [float(env.vec.scenario.routes[0, t, int(
        env.vec.scenario.n_wpt[0, t]) - 1, 1])]
    return n, e


class _NavView(_View):
    """NavigationSystem (LOS_guidance.py:26-136): the route lists (copies; update_route inserts at
    index -1), |e_ct| of the last guidance call, the LOS integral and parameters."""
    _fields = {
        "north": (lambda env, t: _route_lists(env, t)[0],),
        "east": (lambda env, t: _route_lists(env, t)[1],),
        "e_ct": _real("last_e_ct"), "e_ct_int": _real("e_ct_int"),
        "ra": (lambda env, t: env.vec.params.radius_of_acceptance,),
        "r": (lambda env, t: env.vec.params.lookahead_distance,),
        "ki": (lambda env, t: env.vec.params.los_integral_gain,),
        "integrator_limit": (lambda env, t: env.vec.params.integrator_windup_limit,),
        "init_route": (lambda env, t: env.vec.scenario.routes[0, t, :int(env.vec.scenario.n_wpt[0, t])].copy(),),
    }


class _AutoPilotView(_View):
    """HeadingBySampledRouteController (controllers.py:253-350)."""
    _fields = {
        "next_wpt": (lambda env, t: int(env._state()["next_wpt"][t, 0]),
                     lambda env, t, v: env._write("next_wpt", t, int(v))),
        "navigate": (lambda env, t: _NavView(env, t),),
        "heading_controller": (lambda env, t: _HeadingView(env, t),),
    }

    def get_cross_track_error(self):
        return self.navigate.e_ct


class ShipAssetsView(_View):
    """One ship of the env with ShipAssets' attributes (MSRL_Env.py:25-35):

    ========================================================  ===============================
    attribute                                                  device state field
    ========================================================  ===============================
    ship_model.north / east / yaw_angle                        north / east / yaw
    ship_model.forward_speed / sideways_speed / yaw_rate       surge / sway / yaw_rate
    ship_model.int.time                                        ticks x dt
    ship_model.ship_machinery_model.omega (.thrust)            shaft_speed
    throttle_controller.ship_speed_controller.error_i          ship_speed_i
    throttle_controller.shaft_speed_controller.error_i         shaft_speed_i
    auto_pilot.heading_controller.ship_heading_controller      heading_i / heading_prev
      .error_i / .prev_error
    auto_pilot.next_wpt                                        next_wpt
    auto_pilot.navigate.north / east (lists)                   wpt_north / wpt_east + route end
    auto_pilot.navigate.e_ct / e_ct_int                        last_e_ct / e_ct_int
    stop_flag                                                  stop
    desired_forward_speed                                      construction value (scenario)
    ========================================================  ===============================
    State attributes are writable (the value goes to the device before the next step)."""
    _fields = {
        "ship_model": (lambda env, t: _ShipModelView(env, t),),
        "throttle_controller": (lambda env, t: _ThrottleView(env, t),),
        "auto_pilot": (lambda env, t: _AutoPilotView(env, t),),
        "desired_forward_speed": (lambda env, t: float(env.vec.scenario.init[0, t, 7]),),
        "stop_flag": (lambda env, t: bool(env._state()["stop"][t, 0]),
                      lambda env, t, v: env._write("stop", t, int(bool(v)))),
        "type_tag": (lambda env, t: ("test_ship", "obs_ship")[t],),
        "integrator_term": (lambda env, t: (env._flush(), env._integrator_term[t])[1],),
        "time_list": (lambda env, t: (env._flush(), env._time_list[t])[1],),
    }


class MultiShipRLEnv:
    """One two-ship env with the reference's scalar API (float64 by default: the reference's
    arithmetic).

    MultiShipRLEnv(assets, map, ship_draw, time_since_last_ship_drawing, args) — the reference's
    constructor (MSRL_Env.py:42-116) on its ShipAssets / PolygonObstacle objects; or
    MultiShipRLEnv(scenario=..., params=...) from this package's Scenario (see make_gpu_env).
    record: keep ship_model.simulation_results, reward_results, integrator_term and time_list like the
    reference (from the kernel's trajectory log; one extra 62-value row per step)."""

    def __init__(self, assets=None, map=None, ship_draw: bool = False, time_since_last_ship_drawing: float = 0.0,
                 args=None, *, scenario: Scenario | None = None, params=None, precision: int = 64,
                 wpt_capacity: int = 32, device=None, record: bool = True):
        live = None
        if assets is not None:
            if scenario is not None or params is not None:
                raise ValueError("give the reference's assets or a scenario, not both")
            if map is None:
                raise ValueError("MultiShipRLEnv(assets, map, ...): the PolygonObstacle map is required")
            test, obs = assets
            vals = [read_asset(test, "assets[0]"), read_asset(obs, "assets[1]")]
            params = params_from_assets(vals[0], vals[1], args)
            scenario, live = _scenario_from_assets(vals, map, wpt_capacity)
        elif scenario is None:
            from .scenario import make_scenario
            scenario = make_scenario(1, cap=wpt_capacity, jitter=False)
        if scenario.n_env != 1:
            raise ValueError("MultiShipRLEnv is one env; use VecMultiShipRLEnv for batches")
        if args is not None and params is not None and live is None:
            params.sampling_frequency = int(args.sampling_frequency)
            params.theta = float(args.theta)
        self.vec = VecMultiShipRLEnv(scenario=scenario, params=params if params is not None else default_params(),
                                     precision=precision, device=device)
        self._cache = None
        if live is not None:
            self.vec.set_state(live)
        p = self.vec.params
        self._dt = float(p.integration_step)
        self.map = map if map is not None else scenario.polys
        self.args = args if args is not None else SimpleNamespace(sampling_frequency=p.sampling_frequency,
                                                                  theta=p.theta)
        self.ship_draw = bool(ship_draw)
        self.time_since_last_ship_drawing = time_since_last_ship_drawing
        self.record = bool(record)
        # per-step host arrays of sit_step_host (one ctypes call per step: the library stages the inputs
        # in pinned coherent memory the kernel reads and writes directly, launches, copies the state
        # blob when recording, synchronises once)
        rs = 8 if precision == 64 else 4
        self._rs, self._np_real = rs, (np.float64 if precision == 64 else np.float32)
        self._act = np.zeros(2, self._np_real)
        self._sac, self._init = np.zeros(1, np.uint8), np.zeros(1, np.uint8)
        self._ns, self._rw = np.zeros(10, self._np_real), np.zeros(1, self._np_real)
        self._dn, self._st = np.zeros(1, np.uint8), np.zeros(1, np.uint32)
        self._log = np.zeros(_lib.SIT_LOG_ROWS, self._np_real)
        # the state blob after a step (recording envs: every step; else fetched when a view reads it) and
        # numpy views of it made once (building views per step cost ~0.15 ms of torch view calls)
        self._blob_t = torch.zeros(self.vec._state_bytes, dtype=torch.uint8, pin_memory=torch.cuda.is_available())
        self._host_state = {k: v.numpy() for k, v in self.vec._views(self._blob_t).items()}
        ptr = lambda a: c_void_p(a.ctypes.data)  # noqa: E731
        # (the array pointers are cached; the stream is the caller's current one, taken per call under
        # the handle's device, so a step is ordered after a reset or state write on the same stream)
        self._step_args = (self.vec.handle, ptr(self._act), ptr(self._sac), ptr(self._init), ptr(self._ns),
                           ptr(self._rw), ptr(self._dn), ptr(self._st), ptr(self._log) if self.record else None,
                           c_void_p(self._blob_t.data_ptr()) if self.record else None)
        self._step_fn = self.vec.lib.sit_step_host
        r = scenario.routes[0, 1]
        nw = int(scenario.n_wpt[0, 1])
        self.observation_space = _Box(
            np.array([0, 0, -np.pi, -3000, 0, 0, 0, 0, -np.pi, 0], dtype=np.float32),
            np.array([10000, 20000, np.pi, 3000, 1000, 2000, 10000, 20000, np.pi, 1000], dtype=np.float32))
        self.action_space = _Box(np.array([-np.pi / 6], dtype=np.float32), np.array([np.pi / 6], dtype=np.float32))
        self.np_random = np.random.default_rng()
        # the construction-time observation (MSRL_Env.py:88-92): float32, from the live pose
        st = self._state()
        self.initial_state = np.array([st["north"][0, 0], st["east"][0, 0], st["yaw"][0, 0], 0, 0, 0,
                                       st["north"][1, 0], st["east"][1, 0], st["yaw"][1, 0], 0], dtype=np.float32)
        self.state = self.initial_state
        self.initial_next_states = np.zeros(10, dtype=np.float32)      # (:98-99)
        self.next_states = self.initial_next_states
        self.eps_simu_time = 0
        self.simu_time = 0
        self.prev_route_coordinate = None
        self._AB = (r[0], r[nw - 1])
        self.reward_function_params()
        self._obs_stop_pre = bool(st["stop"][1, 0])       # the obstacle ship's stop flag before a step
        self.test, self.obs = ShipAssetsView(self, 0), ShipAssetsView(self, 1)
        self.assets = [self.test, self.obs]
        self._sim_results = [{}, {}]
        self._integrator_term, self._time_list = [[], []], [[], []]
        self._rows, self._n_flushed = [], 0

    # ---------------- reference methods ----------------
    def reward_function_params(self):
        """MSRL_Env.py:119-143: reward constants, the AB segment of the obstacle ship's route, and the
        reward_results containers."""
        p = self.vec.params
        self.e_tolerance = p.e_tolerance
        a, b = self._AB
        self.AB_distance_n = float(b[0] - a[0])
        self.AB_distance_e = float(b[1] - a[1])
        self.AB_distance = math.sqrt(self.AB_distance_n ** 2 + self.AB_distance_e ** 2)
        self.AB_segment_length = self.AB_distance / p.sampling_frequency
        self.AB_alpha = math.atan2(self.AB_distance_e, self.AB_distance_n)
        self.AB_beta = math.pi / 2 - self.AB_alpha
        self.theta = p.theta
        self.reward_results = {who: {name: [] for w, name in REWARD_SERIES if w == who}
                               for who in ("test_ship", "obs_ship", "shared")}

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
        self._cache = None
        self.simu_time = 0
        self.prev_route_coordinate = None
        self.state = self.initial_state
        self._sim_results = [{}, {}]
        self._integrator_term, self._time_list = [[], []], [[], []]
        self._rows, self._n_flushed = [], 0
        self._obs_stop_pre = False
        self.reward_function_params()
        return self.initial_state.copy()

    def init_step(self):
        """MultiShipRLEnv.init_step (MSRL_Env.py:190-217)."""
        self.vec.init_step()
        self._cache = None

    def step(self, converted_action, SAC_update, init):
        """MultiShipRLEnv.step (MSRL_Env.py:404-442): returns (next_state list of 10 float,
        reward float, done bool, status str)."""
        a = self._act
        a[0] = converted_action[0]
        a[1] = converted_action[1]
        self._sac[0] = 1 if SAC_update else 0
        self._init[0] = 1 if init else 0
        dev = self.vec.device
        # (the device context costs ~4 us per call: skipped when the handle's device is current)
        if dev.index is None or torch.cuda.current_device() == dev.index:
            rc = self._step_fn(*self._step_args, self.vec._stream())
        else:
            with torch.cuda.device(dev):
                rc = self._step_fn(*self._step_args, self.vec._stream())
        if rc:
            _lib.check(rc, self.vec.handle)
        # recording envs have the post-step state on the host; otherwise a view fetches it on demand
        self._cache = self._host_state if self.record else None
        reward = float(self._rw[0])
        status = int(self._st[0])
        next_state = self._ns.tolist()
        if SAC_update:                                  # obs_step (MSRL_Env.py:326-340)
            self.prev_route_coordinate = (converted_action[0], converted_action[1])
        if self.ship_draw:                              # ship drawing timer (MSRL_Env.py:418-423; no drawing)
            if self.time_since_last_ship_drawing > 30:
                self.time_since_last_ship_drawing = 0
            self.time_since_last_ship_drawing += self._dt
        if self.record:
            st = self._host_state
            self._rows.append((self._log.copy(), self._read("e_ct_int", 0), self._read("e_ct_int", 1),
                               self._obs_stop_pre))
            self._obs_stop_pre = bool(st["stop"][1, 0])
        self.state = next_state
        return next_state, reward, bool(self._dn[0]), _status_string(status)

    def _flush(self):
        """The recorded steps not yet in the reference's containers: simulation_results of both ships
        (store_simulation_data / store_last_simulation_data, ship_model.py:645-700), reward_results running
        sums (MSRL_env_ex.py:926-964), and the assets' integrator_term / time_list (MSRL_Env.py:264-265,
        305-306, 374-375).  Built when read, not on the step path."""
        nk = len(LOG_KEYS)
        for row, ect0, ect1, stop_pre in self._rows[self._n_flushed:]:
            for t, ect in ((0, ect0), (1, ect1)):
                res = self._sim_results[t]
                for i, k in enumerate(LOG_KEYS):
                    res.setdefault(k, []).append(float(row[t * nk + i]))
                self._integrator_term[t].append(ect)
                # the simulator time after the integration, before int.next_time(); a stopped obstacle ship
                # appends it after the first of its two next_time() calls (MSRL_Env.py:293-309)
                stop_path = t == 1 and stop_pre
                self._time_list[t].append(float(row[t * nk]) + (self._dt if stop_path else 0.0))
            for j, (who, name) in enumerate(REWARD_SERIES):
                lst = self._reward_results[who][name]
                lst.append((lst[-1] if lst else 0) + float(row[2 * nk + j]))
        self._n_flushed = len(self._rows)

    @property
    def reward_results(self):
        self._flush()
        return self._reward_results

    @reward_results.setter
    def reward_results(self, v):
        self._reward_results = v

    # ---------------- state access ----------------
    def _state(self):
        """The env's device state as numpy arrays (the state blob, copied to the host once per step
        when the env records, else when a view first reads it after a step; then cached)."""
        if self._cache is None:
            self._blob_t.copy_(self.vec.state_blob())
            self._cache = self._host_state
        return self._cache

    def _read(self, field, t=None):
        """One state real as a Python float: ship field [t, 0] or env field [0].  A float32 handle's
        double-float fields (env.LO_FIELDS) are read as hi + lo, the value the kernel's decisions use."""
        st = self._state()
        idx = (0,) if t is None else (t, 0)
        v = float(st[field][idx])
        lo = LO_FIELDS.get(field)
        if self._rs == 4 and lo is not None and lo in st:
            v += float(st[lo][idx])
        return v

    def _write(self, field, t, value):
        """Write one ship's state field (the reference's attribute assignment) to the device.  A float32
        handle's double-float field is written as hi = float32(value), lo = value - hi, the other ship's
        hi + lo kept as they are."""
        st = self._state()
        v = st[field].copy()
        v[t, 0] = value
        upd = {field: v}
        lo = LO_FIELDS.get(field)
        if lo is not None and lo in st:
            vl = st[lo].copy()
            vl[t, 0] = float(value) - float(np.float32(value)) if self._rs == 4 else 0.0
            upd[lo] = vl
        self.vec.set_state(upd)
        self._cache = None
        if field == "stop" and t == 1:
            self._obs_stop_pre = bool(value)

    @property
    def sampling_distance_travelled(self):
        return self._read("sampling_dist")

    @property
    def eps_distance_travelled(self):
        return float(self._state()["eps_dist"][0])

    # the single-ship legacy driver reads RL_env.ship_model / auto_pilot (test_beds/main_ast.py:327, 373,
    # 430): the ship under test's
    @property
    def ship_model(self):
        return self.test.ship_model

    @property
    def auto_pilot(self):
        return self.test.auto_pilot


def _scenario_from_assets(vals, map_, cap):
    """Scenario (reset values) and the live state dictionary of the assets."""
    routes = np.zeros((1, 2, cap, 2))
    n_wpt = np.zeros((1, 2), dtype=np.int32)
    init = np.zeros((1, 2, len(_lib.INIT_FIELDS)))
    live = {k: np.zeros((2, 1)) for k in ("north", "east", "yaw", "surge", "sway", "yaw_rate", "shaft_speed",
                                          "ship_speed_i", "shaft_speed_i", "heading_i", "heading_prev", "e_ct_int")}
    live.update({k: np.zeros((2, 1), dtype=np.int32) for k in ("next_wpt", "n_wpt", "ticks", "stop")})
    live["wpt_north"] = np.zeros((2, cap, 1))
    live["wpt_east"] = np.zeros((2, cap, 1))
    mm = "ship_model.ship_machinery_model."
    for t, v in enumerate(vals):
        r0 = _route_of(v["auto_pilot.navigate.init_route"])
        if not 2 <= len(r0) <= cap:
            raise ValueError(f"ship {t}: route of {len(r0)} waypoints (wpt_capacity {cap})")
        routes[0, t, :len(r0)] = r0
        n_wpt[0, t] = len(r0)
        simpl = (mm + "thrust") in v
        shaft = float(v[mm + ("thrust" if simpl else "omega")])
        init[0, t, :6] = [float(v["ship_model.init_" + f]) for f in POSE_FIELDS]
        init[0, t, 6] = shaft
        init[0, t, 7] = float(v["desired_forward_speed"])
        init[0, t, 8] = float(v["throttle_controller.ship_speed_controller.error_i"])
        init[0, t, 9] = 0.0 if simpl else float(v["throttle_controller.shaft_speed_controller.error_i"])
        for f, k in zip(POSE_FIELDS, ("north", "east", "yaw", "surge", "sway", "yaw_rate")):
            live[k][t, 0] = float(v["ship_model." + f])
        live["shaft_speed"][t, 0] = shaft
        live["ship_speed_i"][t, 0] = init[0, t, 8]
        live["shaft_speed_i"][t, 0] = init[0, t, 9]
        hc = "auto_pilot.heading_controller.ship_heading_controller."
        live["heading_i"][t, 0] = float(v[hc + "error_i"])
        live["heading_prev"][t, 0] = float(v[hc + "prev_error"])
        live["e_ct_int"][t, 0] = float(v["auto_pilot.navigate.e_ct_int"])
        live["next_wpt"][t, 0] = int(v["auto_pilot.next_wpt"])
        rn, re_ = list(v["auto_pilot.navigate.north"]), list(v["auto_pilot.navigate.east"])
        if len(rn) > cap or (float(rn[-1]), float(re_[-1])) != (float(r0[-1, 0]), float(r0[-1, 1])):
            raise ValueError(f"ship {t}: the live route must end at the route's final waypoint and fit wpt_capacity")
        live["n_wpt"][t, 0] = len(rn)
        live["wpt_north"][t, :len(rn) - 1, 0] = rn[:-1]
        live["wpt_east"][t, :len(re_) - 1, 0] = re_[:-1]
        live["ticks"][t, 0] = int(round(float(v["ship_model.int.time"]) / float(
            v["ship_model.simulation_config.integration_step"])))
        live["stop"][t, 0] = int(bool(v["stop_flag"]))
    return Scenario(routes, n_wpt, init, _polygons_of(map_)), live


def make_gpu_env(ship_config, env_config, sim_config_test, sim_config_obs, machinery_config, throttle_gains,
                 heading_gains, los_params, route_test, route_obs, obstacle_vertices, args,
                 desired_speed=(8.5, 8.5), omega0=400 * np.pi / 30, shaft_speed_i0=114.0, wpt_capacity=32,
                 precision=64, device=None, record=True) -> MultiShipRLEnv:
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
    return MultiShipRLEnv(scenario=scen, params=p, precision=precision, device=device, record=record)
