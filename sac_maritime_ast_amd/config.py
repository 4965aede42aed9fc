"""Configuration: build ``sit_params`` from the reference's own configuration objects.

The reference configures a ship with NamedTuples (ship_model.py:20-53, ship_engine.py:17-138,
controllers.py:16-38, LOS_guidance.py:15-19) plus env ``args`` (test_beds/test_policy.py:39-42).
``params_from_reference`` accepts those objects (or any object with the same attribute names),
so a user of the reference passes the configs they already have.
"""
from __future__ import annotations

import math

from . import _lib

_SG = {"MOTOR": _lib.SIT_SG_MOTOR, "GEN": _lib.SIT_SG_GEN}


def params(**overrides) -> _lib.SitParams:
    """Defaults of test_beds/test_policy.py:94-226 (PTI mode), with keyword overrides."""
    p = _lib.default_params()
    for k, v in overrides.items():
        if not hasattr(p, k):
            raise KeyError(f"unknown sit_params field {k!r}")
        setattr(p, k, v)
    return p


def params_from_reference(ship_config=None, environment_config=None, simulation_config=None,
                          machinery_config=None, throttle_gains=None, heading_gains=None,
                          los_parameters=None, args=None, **overrides) -> _lib.SitParams:
    """sit_params from reference-style configuration objects (duck-typed NamedTuples).

    A ``SimplifiedPropulsionMachinerySystemConfiguration`` (ship_engine.py:148-157; recognised by its
    thrust_force_dynamic_time_constant) selects SIT_MACH_SIMPLIFIED; ``throttle_gains`` may then be
    the kp / ki of ThrottleFromSpeedSetPointSimplifiedPropulsion (controllers.py:160-169), which
    become kp_ship_speed / ki_ship_speed.
    """
    p = params()
    if ship_config is not None:
        for f in ("dead_weight_tonnage", "coefficient_of_deadweight_to_displacement", "bunkers", "ballast",
                  "length_of_ship", "width_of_ship", "added_mass_coefficient_in_surge",
                  "added_mass_coefficient_in_sway", "added_mass_coefficient_in_yaw",
                  "mass_over_linear_friction_coefficient_in_surge",
                  "mass_over_linear_friction_coefficient_in_sway", "mass_over_linear_friction_coefficient_in_yaw"):
            setattr(p, f, float(getattr(ship_config, f)))
        # the reference spells these with a double underscore (ship_model.py:33-35)
        for axis in ("surge", "sway", "yaw"):
            v = getattr(ship_config, f"nonlinear_friction_coefficient__in_{axis}", None)
            if v is None:
                v = getattr(ship_config, f"nonlinear_friction_coefficient_in_{axis}")
            setattr(p, f"nonlinear_friction_coefficient_in_{axis}", float(v))
    if environment_config is not None:
        for f in ("current_velocity_component_from_north", "current_velocity_component_from_east",
                  "wind_speed", "wind_direction"):
            setattr(p, f, float(getattr(environment_config, f)))
    if simulation_config is not None:
        p.integration_step = float(simulation_config.integration_step)
    if machinery_config is not None:
        mc = machinery_config
        for f in ("hotel_load", "rated_speed_main_engine_rpm", "linear_friction_main_engine",
                  "linear_friction_hybrid_shaft_generator", "gear_ratio_between_main_engine_and_propeller",
                  "gear_ratio_between_hybrid_shaft_generator_and_propeller", "propeller_inertia",
                  "propeller_speed_to_torque_coefficient", "propeller_diameter",
                  "propeller_speed_to_thrust_force_coefficient", "rudder_angle_to_sway_force_coefficient",
                  "rudder_angle_to_yaw_force_coefficient", "max_rudder_angle_degrees"):
            if hasattr(mc, f):      # the simplified configuration has no shaft fields
                setattr(p, f, float(getattr(mc, f)))
        if hasattr(mc, "thrust_force_dynamic_time_constant"):
            p.machinery_model = _lib.SIT_MACH_SIMPLIFIED
            p.thrust_force_dynamic_time_constant = float(mc.thrust_force_dynamic_time_constant)
        modes = getattr(mc.machinery_modes, "list_of_modes", mc.machinery_modes)
        mode = modes[int(mc.machinery_operating_mode)]
        p.main_engine_capacity = float(mode.main_engine_capacity)
        p.electrical_capacity = float(mode.electrical_capacity)
        p.shaft_generator_state = _SG.get(str(mode.shaft_generator_state), _lib.SIT_SG_OFF)
        for tag, f in (("me", "specific_fuel_consumption_coefficients_me"),
                       ("dg", "specific_fuel_consumption_coefficients_dg")):
            co = getattr(mc, f, None)
            if co is not None:
                setattr(p, f"fuel_{tag}_a", float(co.a))
                setattr(p, f"fuel_{tag}_b", float(co.b))
                setattr(p, f"fuel_{tag}_c", float(co.c))
    if throttle_gains is not None:
        if hasattr(throttle_gains, "kp_ship_speed"):
            for f in ("kp_ship_speed", "ki_ship_speed", "kp_shaft_speed", "ki_shaft_speed"):
                setattr(p, f, float(getattr(throttle_gains, f)))
        else:                       # (kp, ki) of the simplified-propulsion throttle
            p.kp_ship_speed, p.ki_ship_speed = float(throttle_gains.kp), float(throttle_gains.ki)
    if heading_gains is not None:
        p.heading_kp, p.heading_kd, p.heading_ki = (float(heading_gains.kp), float(heading_gains.kd),
                                                    float(heading_gains.ki))
    if los_parameters is not None:
        p.radius_of_acceptance = float(los_parameters.radius_of_acceptance)
        p.lookahead_distance = float(los_parameters.lookahead_distance)
        p.los_integral_gain = float(los_parameters.integral_gain)
        p.integrator_windup_limit = float(los_parameters.integrator_windup_limit)
    if args is not None:
        p.sampling_frequency = int(getattr(args, "sampling_frequency", p.sampling_frequency))
        p.theta = float(getattr(args, "theta", p.theta))
    for k, v in overrides.items():
        setattr(p, k, v)
    return p


def shaft_speed_max(p: _lib.SitParams) -> float:
    """ShipMachineryModel.shaft_speed_max (ship_engine.py:325)."""
    return 1.1 * (p.rated_speed_main_engine_rpm * math.pi / 30) * p.gear_ratio_between_main_engine_and_propeller
