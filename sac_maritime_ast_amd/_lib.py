"""ctypes binding of libsit.so (the HIP C ABI declared in include/sit.h).

The library is built in-tree by ``__graft_entry__.build()`` (hipcc --offload-arch=gfx950).
There is no fallback: importing the product path without the library raises.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, c_char_p, c_double, c_int32, c_int64, c_size_t, c_uint64, c_void_p

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SIT_LIBRARY", os.path.join(HERE, "libsit.so"))

SIT_OK, SIT_E_INVALID, SIT_E_HIP, SIT_E_NOMEM, SIT_E_STATE = 0, -1, -2, -3, -4
SIT_F32, SIT_F64 = 32, 64
SIT_SG_MOTOR, SIT_SG_GEN, SIT_SG_OFF = 0, 1, 2
SIT_MACH_SHAFT, SIT_MACH_SIMPLIFIED = 0, 1
SIT_DT_REAL, SIT_DT_I32, SIT_DT_U32 = 0, 1, 2
SIT_OBS_DIM = 10
SIT_TRANSITION_DIM = 24
SIT_ACTOR_HIDDEN = 256
SIT_ACTOR_WEIGHTS = SIT_ACTOR_HIDDEN * SIT_OBS_DIM + SIT_ACTOR_HIDDEN + SIT_ACTOR_HIDDEN ** 2 + SIT_ACTOR_HIDDEN + 2 * SIT_ACTOR_HIDDEN + 2
SIT_LOG_KEYS, SIT_LOG_ROWS = 27, 62
INIT_FIELDS = ("north", "east", "yaw", "surge", "sway", "yaw_rate", "shaft_speed", "desired_speed",
               "ship_speed_i", "shaft_speed_i")

ST_TEST_ENDPOINT, ST_TEST_HORIZON, ST_TEST_TERRAIN = 1 << 0, 1 << 1, 1 << 2
ST_TEST_MECHANICAL, ST_TEST_NAVIGATION, ST_TEST_BLACKOUT = 1 << 3, 1 << 4, 1 << 5
ST_OBS_ENDPOINT, ST_OBS_HORIZON, ST_OBS_TERRAIN = 1 << 6, 1 << 7, 1 << 8
ST_OBS_IW_TERMINAL, ST_OBS_NAVIGATION, ST_COLLISION = 1 << 9, 1 << 10, 1 << 11
ST_TEST_DONE, ST_OBS_DONE, ST_ROUTE_OVERFLOW = 1 << 12, 1 << 13, 1 << 31
ST_NO_STEP = 1 << 30
SIT_POLICY_READY, SIT_POLICY_WAITING = 1, 2

_D = c_double
PARAM_FIELDS = [
    ("dead_weight_tonnage", _D), ("coefficient_of_deadweight_to_displacement", _D), ("bunkers", _D),
    ("ballast", _D), ("length_of_ship", _D), ("width_of_ship", _D),
    ("added_mass_coefficient_in_surge", _D), ("added_mass_coefficient_in_sway", _D),
    ("added_mass_coefficient_in_yaw", _D), ("mass_over_linear_friction_coefficient_in_surge", _D),
    ("mass_over_linear_friction_coefficient_in_sway", _D), ("mass_over_linear_friction_coefficient_in_yaw", _D),
    ("nonlinear_friction_coefficient_in_surge", _D), ("nonlinear_friction_coefficient_in_sway", _D),
    ("nonlinear_friction_coefficient_in_yaw", _D),
    ("current_velocity_component_from_north", _D), ("current_velocity_component_from_east", _D),
    ("wind_speed", _D), ("wind_direction", _D),
    ("rho_air", _D), ("front_height", _D), ("side_height", _D), ("cx", _D), ("cy", _D), ("cn", _D),
    ("integration_step", _D),
    ("hotel_load", _D), ("main_engine_capacity", _D), ("electrical_capacity", _D),
    ("shaft_generator_state", c_int32), ("machinery_model", c_int32),
    ("rated_speed_main_engine_rpm", _D), ("linear_friction_main_engine", _D),
    ("linear_friction_hybrid_shaft_generator", _D), ("gear_ratio_between_main_engine_and_propeller", _D),
    ("gear_ratio_between_hybrid_shaft_generator_and_propeller", _D), ("propeller_inertia", _D),
    ("propeller_speed_to_torque_coefficient", _D), ("propeller_diameter", _D),
    ("propeller_speed_to_thrust_force_coefficient", _D), ("rudder_angle_to_sway_force_coefficient", _D),
    ("rudder_angle_to_yaw_force_coefficient", _D), ("max_rudder_angle_degrees", _D),
    ("kp_ship_speed", _D), ("ki_ship_speed", _D), ("kp_shaft_speed", _D), ("ki_shaft_speed", _D),
    ("heading_kp", _D), ("heading_kd", _D), ("heading_ki", _D),
    ("radius_of_acceptance", _D), ("lookahead_distance", _D), ("los_integral_gain", _D),
    ("integrator_windup_limit", _D),
    ("theta", _D), ("sampling_frequency", c_int32), ("collision_bias", c_int32),
    ("e_tolerance", _D), ("arrival_radius", _D), ("shaft_rpm_max", _D), ("minimum_ship_distance", _D),
    ("bias_throttle_scale", _D), ("bias_throttle_max", _D), ("bias_rudder_degrees", _D),
    ("fuel_me_a", _D), ("fuel_me_b", _D), ("fuel_me_c", _D), ("fuel_dg_a", _D), ("fuel_dg_b", _D),
    ("fuel_dg_c", _D), ("thrust_force_dynamic_time_constant", _D),
]


class SitParams(ctypes.Structure):
    _fields_ = PARAM_FIELDS

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in PARAM_FIELDS if not k.startswith("_")}


class RolloutArgs(ctypes.Structure):
    _fields_ = [
        ("n_steps", c_int32), ("auto_reset", c_int32), ("seed", c_uint64), ("env_id_offset", c_int64),
        ("action_ne", c_void_p), ("sac_update", c_void_p), ("init", c_void_p),
        ("next_state", c_void_p), ("reward", c_void_p), ("done", c_void_p), ("status", c_void_p),
        ("action_out", c_void_p), ("done_count", c_void_p),
        ("transitions", c_void_p), ("transition_count", c_void_p), ("transition_capacity", c_int32),
        ("mask_horizon", c_int32),
        ("policy_action", c_void_p), ("policy_ready", c_void_p), ("request_env", c_void_p),
        ("request_noise", c_void_p), ("request_obs", c_void_p), ("request_count", c_void_p),
        ("request_capacity", c_int32),
        ("env_steps", c_void_p), ("log", c_void_p), ("request_age", c_void_p),
        ("actor_weights", c_void_p), ("actor_deterministic", c_int32), ("actor_served", c_void_p),
    ]


class SitError(RuntimeError):
    pass


# every entry point of include/sit.h: name -> (restype, argtypes)
SIGNATURES = {
    "sit_abi_version": (c_int32, []),
    "sit_params_size": (c_size_t, []),
    "sit_rollout_args_size": (c_size_t, []),
    "sit_params_default": (None, [POINTER(SitParams)]),
    "sit_create": (c_int32, [POINTER(SitParams), c_int32, c_int32, c_int32, POINTER(c_void_p)]),
    "sit_destroy": (None, [c_void_p]),
    "sit_last_error": (c_char_p, [c_void_p]),
    "sit_precision": (c_int32, [c_void_p]),
    "sit_n_env": (c_int32, [c_void_p]),
    "sit_step_kernel": (c_char_p, [c_void_p]),
    "sit_debug_flags": (c_int32, [c_void_p]),
    "sit_debug_build": (c_int32, []),
    "sit_role_fallbacks": (c_int32, [c_void_p, c_int32]),
    "sit_load_map": (c_int32, [c_void_p, c_int32, c_void_p, c_void_p]),
    "sit_load_routes": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "sit_load_initial": (c_int32, [c_void_p, c_void_p]),
    "sit_map_info": (c_int32, [c_void_p, c_void_p, c_int32]),
    "sit_policy_apply": (c_int32, [c_void_p, c_int32, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_int32,
                                   c_void_p, c_void_p, c_void_p, c_void_p]),
    "sit_policy_actor": (c_int32, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "sit_probe_map": (c_int32, [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "sit_selftest_f64": (c_int32, [c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_int32, c_void_p]),
    "sit_restart": (c_int32, [c_void_p, c_void_p]),
    "sit_reset": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p]),
    "sit_init_step": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "sit_step": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_void_p, c_void_p]),
    "sit_step_host": (c_int32, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_void_p]),
    "sit_rollout": (c_int32, [c_void_p, POINTER(RolloutArgs), c_void_p]),
    "sit_state_nfields": (c_int32, []),
    "sit_state_field": (c_int32, [c_void_p, c_int32, POINTER(c_char_p), POINTER(c_size_t),
                                  POINTER(c_int32), POINTER(c_int64)]),
    "sit_state_bytes": (c_int32, [c_void_p, POINTER(c_size_t)]),
    "sit_get_state": (c_int32, [c_void_p, c_void_p, c_void_p]),
    "sit_set_state": (c_int32, [c_void_p, c_void_p, c_void_p]),
}

_lib = None


def load():
    """Load libsit.so (once).  Raises ImportError if the HIP library has not been built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"HIP library {LIB_PATH} is missing; build it with "
                          "`python -c 'import __graft_entry__ as g; g.build()'` (hipcc, gfx950)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None)
        if fn is None:        # diagnostic builds of older revisions (A/B timing) lack newer entries
            continue
        fn.restype = res
        fn.argtypes = args
    if lib.sit_abi_version() != 1:
        raise ImportError("libsit.so ABI version mismatch")
    if lib.sit_params_size() != ctypes.sizeof(SitParams):
        raise ImportError(f"sit_params layout mismatch: C {lib.sit_params_size()} vs "
                          f"ctypes {ctypes.sizeof(SitParams)} bytes")
    if lib.sit_rollout_args_size() != ctypes.sizeof(RolloutArgs):
        raise ImportError(f"sit_rollout_args layout mismatch: C {lib.sit_rollout_args_size()} vs "
                          f"ctypes {ctypes.sizeof(RolloutArgs)} bytes")
    _lib = lib
    return lib


def check(rc, handle=None):
    if rc != SIT_OK:
        msg = load().sit_last_error(handle)
        raise SitError(f"sit error {rc}: {msg.decode() if msg else ''}")
    return rc


def default_params() -> SitParams:
    p = SitParams()
    load().sit_params_default(ctypes.byref(p))
    return p
