"""The scalar drop-in ``compat.MultiShipRLEnv`` — the reference's own ``reset()/init_step()/
step(converted_action, SAC_update, init)`` surface (RLEnv/MSRL_Env.py:42-116, 147-217, 404-446)
— built through ``compat.make_gpu_env`` from reference-style configuration objects (the
NamedTuples of test_beds/test_policy.py:94-226 as SimpleNamespace), replaying the reference's
recorded episodes step by step (``-m gpu``).

Checked per step: the exact Python types the reference returns (list of 10 float, float, bool,
str), the status strings character for character, and the values within 1e-9 relative
(float64, per-field floors)."""
import math
from types import SimpleNamespace

import numpy as np
import pytest

from helpers import OBS_SCALE, env_oracle, env_state_from, golden, params_for, rel_err
from oracle import sit_oracle as so

pytestmark = pytest.mark.gpu

sit = pytest.importorskip("sac_maritime_ast_amd")
from sac_maritime_ast_amd.compat import MultiShipRLEnv, make_gpu_env  # noqa: E402
from sac_maritime_ast_amd.scenario import ISLANDS  # noqa: E402

DEV = "cuda:0"
SG_NAME = {so.SG_MOTOR: "MOTOR", so.SG_GEN: "GEN", so.SG_OFF: "OFF"}


def reference_configs(p):
    """The reference's configuration objects (duck-typed) holding the values of dict p."""
    ship = SimpleNamespace(**{k: p[k] for k in (
        "dead_weight_tonnage", "coefficient_of_deadweight_to_displacement", "bunkers", "ballast", "length_of_ship",
        "width_of_ship", "added_mass_coefficient_in_surge", "added_mass_coefficient_in_sway",
        "added_mass_coefficient_in_yaw", "mass_over_linear_friction_coefficient_in_surge",
        "mass_over_linear_friction_coefficient_in_sway", "mass_over_linear_friction_coefficient_in_yaw")},
        # the reference spells these with a double underscore (ship_model.py:33-35)
        nonlinear_friction_coefficient__in_surge=p["nonlinear_friction_coefficient_in_surge"],
        nonlinear_friction_coefficient__in_sway=p["nonlinear_friction_coefficient_in_sway"],
        nonlinear_friction_coefficient__in_yaw=p["nonlinear_friction_coefficient_in_yaw"])
    env = SimpleNamespace(**{k: p[k] for k in ("current_velocity_component_from_north",
                                               "current_velocity_component_from_east", "wind_speed",
                                               "wind_direction")})
    mode = SimpleNamespace(main_engine_capacity=p["main_engine_capacity"], electrical_capacity=p["electrical_capacity"],
                           shaft_generator_state=SG_NAME[int(p["shaft_generator_state"])])
    mc = SimpleNamespace(hotel_load=p["hotel_load"], machinery_modes=SimpleNamespace(list_of_modes=[mode]),
                         machinery_operating_mode=0,
                         specific_fuel_consumption_coefficients_me=SimpleNamespace(
                             a=p["fuel_me_a"], b=p["fuel_me_b"], c=p["fuel_me_c"]),
                         specific_fuel_consumption_coefficients_dg=SimpleNamespace(
                             a=p["fuel_dg_a"], b=p["fuel_dg_b"], c=p["fuel_dg_c"]),
                         **{k: p[k] for k in (
                             "rated_speed_main_engine_rpm", "linear_friction_main_engine",
                             "linear_friction_hybrid_shaft_generator", "gear_ratio_between_main_engine_and_propeller",
                             "gear_ratio_between_hybrid_shaft_generator_and_propeller", "propeller_inertia",
                             "propeller_speed_to_torque_coefficient", "propeller_diameter",
                             "propeller_speed_to_thrust_force_coefficient", "rudder_angle_to_sway_force_coefficient",
                             "rudder_angle_to_yaw_force_coefficient", "max_rudder_angle_degrees")})
    thr = SimpleNamespace(**{k: p[k] for k in ("kp_ship_speed", "ki_ship_speed", "kp_shaft_speed", "ki_shaft_speed")})
    hdg = SimpleNamespace(kp=p["heading_kp"], kd=p["heading_kd"], ki=p["heading_ki"])
    los = SimpleNamespace(radius_of_acceptance=p["radius_of_acceptance"], lookahead_distance=p["lookahead_distance"],
                          integral_gain=p["los_integral_gain"], integrator_windup_limit=p["integrator_windup_limit"])
    args = SimpleNamespace(sampling_frequency=p["sampling_frequency"], theta=p["theta"])
    return ship, env, mc, thr, hdg, los, args


def sim_config(pose, dt=0.5):
    return SimpleNamespace(initial_north_position_m=pose[0], initial_east_position_m=pose[1],
                           initial_yaw_angle_rad=pose[2], initial_forward_speed_m_per_s=pose[3],
                           initial_sideways_speed_m_per_s=pose[4], initial_yaw_rate_rad_per_s=pose[5],
                           integration_step=dt)


def env_from_fixture(d):
    p = params_for(d["mode"])
    ship, envc, mc, thr, hdg, los, args = reference_configs(p)
    routes, n_wpt = d["routes"], d["n_wpt"]
    route_test = routes[0, :int(n_wpt[0])].tolist()
    route_obs = routes[1, :int(n_wpt[1])].tolist()
    return make_gpu_env(ship, envc, sim_config(d["pose"][0]), sim_config(d["pose"][1]), mc, thr, hdg, los,
                        route_test, route_obs, ISLANDS, args, wpt_capacity=routes.shape[1], device=DEV)


def test_make_gpu_env_maps_reference_configs():
    """Every sit_params field set from the reference-style objects equals the oracle's value."""
    d = golden("env_blackout_pto")            # a non-default machinery mode (PTO)
    env = env_from_fixture(d)
    got = env.vec.params.as_dict()
    for k, v in params_for(d["mode"]).items():
        if k in got:
            assert got[k] == pytest.approx(v, rel=1e-15, abs=0), k


@pytest.mark.parametrize("name", ["env_nominal", "env_collision", "env_obs_arrival"])
def test_compat_replays_reference_episode(name):
    d = golden(name)
    env = env_from_fixture(d)
    assert isinstance(env, MultiShipRLEnv)
    s0 = env.reset()
    assert isinstance(s0, np.ndarray) and s0.dtype == np.float32 and s0.shape == (10,)
    assert np.array_equal(s0, d["reset_state"].astype(np.float32))       # Q15
    assert env.AB_segment_length == pytest.approx(math.hypot(*(d["routes"][1, int(d["n_wpt"][1]) - 1]
                                                               - d["routes"][1, 0])) / 7, rel=1e-15)
    # start from the reference's recorded state before step 0, then drive the episode(s) through
    # the scalar API only (reset + init_step at the recorded episode boundaries)
    env.vec.set_state(env_state_from(d, "pre_", 0, env_oracle(d)))
    resets = set(int(r) for r in d["resets"])
    T = len(d["reward"])
    for i in range(T):
        if i in resets and i > 0:
            env.reset()
            env.init_step()
        ns, r, done, status = env.step((d["action_n"][i], d["action_e"][i]), bool(d["sac_update"][i]),
                                       bool(d["init"][i]))
        assert type(ns) is list and len(ns) == 10 and all(type(x) is float for x in ns), i
        assert type(r) is float and type(done) is bool and type(status) is str, i
        assert status == str(d["status"][i]), f"{name} step {i}: {status!r} vs {str(d['status'][i])!r}"
        assert done == bool(d["done"][i]), f"{name} step {i}: done"
        assert rel_err(np.array(ns), d["next_state"][i], OBS_SCALE).max() <= 1e-9, f"{name} step {i}"
        assert rel_err(r, d["reward"][i], 1.0) <= 1e-9, f"{name} step {i}: reward"
    assert env.sampling_distance_travelled == pytest.approx(float(d["post_sampling_dist"][T - 1]), rel=1e-9, abs=1e-9)


def test_seed_matches_reference_contract():
    """seed() seeds np_random (gymnasium seeding) and leaves the dynamics untouched."""
    d = golden("env_collision")
    outs = []
    for seed in (1, 2):
        env = env_from_fixture(d)
        env.seed(seed)
        env.reset()
        env.init_step()
        outs.append([env.step((d["action_n"][i], d["action_e"][i]), bool(d["sac_update"][i]), bool(d["init"][i]))
                     for i in range(min(20, len(d["reward"])))])
    assert outs[0] == outs[1]
    e1, e2 = env_from_fixture(d), env_from_fixture(d)
    e1.seed(7)
    e2.seed(7)
    assert e1.np_random.random() == e2.np_random.random()


# ------------------------------------------------------------------------------------------
# the reference's own constructor: MultiShipRLEnv(assets, map, ship_draw, time_since_last_ship_drawing, args)
# ------------------------------------------------------------------------------------------
from ref_assets import apply_setup, fixture_assets, polygon_obstacle, route_state  # noqa: E402
from ref_assets import args as ref_args  # noqa: E402
from sac_maritime_ast_amd.trajectory import LOG_KEYS, REWARD_SERIES  # noqa: E402

REF_CASES = ["env_nominal", "env_collision", "env_obs_arrival", "env_test_arrival", "env_mechanical",
             "env_blackout_pto", "env_reset_persist", "env_test_terrain", "env_many_inserts"]
VIEW_REAL = {"north": "ship_model.north", "east": "ship_model.east", "yaw": "ship_model.yaw_angle",
             "surge": "ship_model.forward_speed", "sway": "ship_model.sideways_speed",
             "yaw_rate": "ship_model.yaw_rate", "shaft_speed": "ship_model.ship_machinery_model.omega",
             "ship_speed_i": "throttle_controller.ship_speed_controller.error_i",
             "shaft_speed_i": "throttle_controller.shaft_speed_controller.error_i",
             "heading_i": "auto_pilot.heading_controller.ship_heading_controller.error_i",
             "heading_prev": "auto_pilot.heading_controller.ship_heading_controller.prev_error",
             "e_ct_int": "auto_pilot.navigate.e_ct_int"}


def _attr(obj, path):
    for p in path.split("."):
        obj = getattr(obj, p)
    return obj


def _check_views(env, d, prefix, i, where):
    """The drop-in's test / obs views against the reference's recorded objects (row i)."""
    for t, view in enumerate((env.test, env.obs)):
        for k, path in VIEW_REAL.items():
            want = float(d[prefix + k][i][t])
            got = _attr(view, path)
            assert type(got) is float, f"{where}: {path} type"
            assert abs(got - want) <= 1e-9 * max(abs(want), SCALE_VIEW.get(k, 1.0)), f"{where}: ship {t} {path}"
        assert view.auto_pilot.next_wpt == int(d[prefix + "next_wpt"][i][t]), f"{where}: next_wpt"
        assert view.ship_model.int.time == d[prefix + "ticks"][i][t] * 0.5, f"{where}: int.time"
        assert view.stop_flag == bool(d[prefix + "stop"][i][t]), f"{where}: stop_flag"
        n, e = route_state(d, prefix, i)[t]
        assert view.auto_pilot.navigate.north == n and view.auto_pilot.navigate.east == e, f"{where}: route"


SCALE_VIEW = dict(north=1e4, east=1e4, yaw=np.pi, surge=10.0, sway=10.0, yaw_rate=0.1, shaft_speed=100.0,
                  ship_speed_i=1e3, shaft_speed_i=1e5, heading_i=10.0, heading_prev=np.pi, e_ct_int=1e2)


@pytest.mark.parametrize("name", REF_CASES)
def test_reference_constructor_drives_episode(name):
    """The reference's harness procedure on the drop-in, from step 0 with no state injected: build it
    from ShipAssets / PolygonObstacle objects (stand-ins carrying the reference objects' recorded
    attributes, tests/ref_assets.py), reset(), init_step(), the fixture's attribute set-up (the
    reference's objects were mutated the same way: ``env.test.ship_model.north = ...``), then
    step() with the recorded actions (reset() + init_step() at the recorded restarts).  Per step:
    exact Python types, status strings, values within 1e-9; the views equal the reference's objects
    before step 0 and after every step; simulation_results, reward_results, integrator_term and
    time_list equal the reference's records."""
    d = golden(name)
    test, obs = fixture_assets(d)
    env = MultiShipRLEnv([test, obs], polygon_obstacle(), False, 30, ref_args(), device=DEV,
                         wpt_capacity=d["routes"].shape[1])
    assert env.AB_segment_length == pytest.approx(float(d["ab_len"]), rel=1e-15)
    assert env.AB_alpha == pytest.approx(float(d["ab_alpha"]), rel=1e-15, abs=1e-15)
    s0 = env.reset()
    assert isinstance(s0, np.ndarray) and s0.dtype == np.float32 and np.array_equal(s0, d["reset_state"].astype(np.float32))
    env.init_step()
    apply_setup(env, name)
    _check_views(env, d, "pre_", 0, f"{name} before step 0")
    resets = set(int(r) for r in d["resets"])
    T = len(d["reward"])
    start = 0
    for i in range(T):
        if i in resets and i > 0:
            env.reset()
            env.init_step()
            start = i
        ns, r, done, status = env.step((d["action_n"][i], d["action_e"][i]), bool(d["sac_update"][i]),
                                       bool(d["init"][i]))
        assert type(ns) is list and len(ns) == 10 and all(type(x) is float for x in ns), i
        assert type(r) is float and type(done) is bool and type(status) is str, i
        assert status == str(d["status"][i]), f"{name} step {i}: {status!r} vs {str(d['status'][i])!r}"
        assert done == bool(d["done"][i]), f"{name} step {i}: done"
        assert rel_err(np.array(ns), d["next_state"][i], OBS_SCALE).max() <= 1e-9, f"{name} step {i}"
        assert rel_err(r, d["reward"][i], 1.0) <= 1e-9, f"{name} step {i}: reward"
        if i % 97 == 0 or i == T - 1:
            _check_views(env, d, "post_", i, f"{name} after step {i}")
    assert env.sampling_distance_travelled == pytest.approx(float(d["post_sampling_dist"][T - 1]), rel=1e-9, abs=1e-9)
    # the reference's records since the last reset
    for t, key in ((0, "log_test"), (1, "log_obs")):
        res = env.assets[t].ship_model.simulation_results
        got = np.array([res[k] for k in LOG_KEYS]).T
        assert got.shape == d[key][start:].shape, f"{name} {key} rows"
        err = np.abs(got - d[key][start:]) / np.maximum(np.abs(d[key][start:]), 1.0)
        assert err.max() <= 1e-9, f"{name} {key}: {err.max():.3e}"
        assert np.allclose(env.assets[t].integrator_term, d["post_e_ct_int"][start:, t], rtol=1e-9, atol=1e-9)
        assert env.assets[t].time_list == [float(x) for x in (d["post_ticks"][start:, t] - 1) * 0.5]
    rr = np.array([env.reward_results[a][b] for a, b in REWARD_SERIES]).T
    err = np.abs(rr - d["log_reward"][start:]) / np.maximum(np.abs(d["log_reward"][start:]), 1.0)
    assert err.max() <= 1e-9, f"{name} reward_results: {err.max():.3e}"


def test_reference_constructor_float32_and_space_api():
    """The float32 drop-in on the reference's objects (the benchmark's precision) within 1e-5 of the
    reference's nominal episode for its first 300 steps, and the gymnasium Box surface
    (seed / sample / contains) the legacy driver uses (test_beds/main_ast.py:259-260)."""
    d = golden("env_nominal")
    env = MultiShipRLEnv(fixture_assets(d), polygon_obstacle(), False, 30, ref_args(), device=DEV, precision=32,
                         wpt_capacity=d["routes"].shape[1], record=False)
    env.reset()
    env.init_step()
    for i in range(300):
        ns, r, done, status = env.step((d["action_n"][i], d["action_e"][i]), bool(d["sac_update"][i]),
                                       bool(d["init"][i]))
        assert status == str(d["status"][i]) and done == bool(d["done"][i])
        assert rel_err(np.array(ns), d["next_state"][i], OBS_SCALE).max() <= 1e-5, f"step {i}"
    env.action_space.seed(3)
    a = env.action_space.sample()
    assert a.shape == (1,) and env.action_space.contains(a)
    assert env.observation_space.shape == (10,)
    assert env.ship_model.int.time == env.test.ship_model.int.time == 300 * 0.5


def test_float32_attribute_write_keeps_double_float_parts():
    """On a float32 drop-in, the reference-style attribute assignment of one ship's double-float field
    (``test.ship_model.north = x``) writes that ship's value as hi + lo = x (to the 48 bits two float32
    parts hold) and leaves the other
    ship's hi and lo untouched; the getters read hi + lo (the value the kernel's decisions use)."""
    d = golden("env_nominal")
    env = MultiShipRLEnv(fixture_assets(d), polygon_obstacle(), False, 30, ref_args(), device=DEV, precision=32,
                         wpt_capacity=d["routes"].shape[1], record=False)
    env.reset()
    env.init_step()
    for i in range(50):     # the integrators carry nonzero low parts after a few steps
        env.step((d["action_n"][i], d["action_e"][i]), bool(d["sac_update"][i]), bool(d["init"][i]))
    before = {k: v.cpu().numpy().copy() for k, v in env.vec.get_state().items()}
    assert np.any(before["north_lo"] != 0)
    x = 1234.567890123
    env.test.ship_model.north = x
    after = {k: v.cpu().numpy() for k, v in env.vec.get_state().items()}
    assert after["north"][1, 0] == before["north"][1, 0] and after["north_lo"][1, 0] == before["north_lo"][1, 0]
    # (hi + lo of two float32 values carries 48 bits: x to ~1e-12 m)
    assert abs(float(after["north"][0, 0]) + float(after["north_lo"][0, 0]) - x) <= 1e-11
    assert abs(env.test.ship_model.north - x) <= 1e-11 and after["north"][0, 0] == np.float32(x)
    assert env.obs.ship_model.north == float(before["north"][1, 0]) + float(before["north_lo"][1, 0])
    comb = env.vec.get_state(combined=True)
    assert env.sampling_distance_travelled == float(comb["sampling_dist"][0].item())


@pytest.mark.parametrize("record", [True, False])
def test_drop_in_step_kernel(record):
    """Which step kernel the scalar drop-in runs (sit_step_kernel): a recording env (the default; its
    step returns the trajectory-log row that builds simulation_results) runs the one-wave logged
    k_env_steps; record=False runs the two-wave k_env_steps_sync with the map read through the caches
    (DESIGN.md §4.1a).  Both through the one host-array call, sit_step_host."""
    d = golden("env_nominal")
    env = MultiShipRLEnv(fixture_assets(d), polygon_obstacle(), False, 30, ref_args(), device=DEV,
                         wpt_capacity=d["routes"].shape[1], record=record)
    env.reset()
    env.init_step()
    env.step((float(d["action_n"][0]), float(d["action_e"][0])), bool(d["sac_update"][0]), bool(d["init"][0]))
    name = env.vec.lib.sit_step_kernel(env.vec.handle).decode()
    if record:
        assert name.startswith("k_env_steps<double,kExplicit,") and ",log," in name, name
        assert len(env.test.ship_model.simulation_results["time [s]"]) == 1
    else:
        assert name.startswith("k_env_steps_sync<double,kExplicit,map=global"), name
        assert env.test.ship_model.simulation_results == {}
