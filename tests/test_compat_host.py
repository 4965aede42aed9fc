"""Host logic of the scalar drop-in's reference-form constructor (compat.MultiShipRLEnv(assets, map,
ship_draw, time_since_last_ship_drawing, args), RLEnv/MSRL_Env.py:42-116), on CPU: the attribute
paths it reads exist on the reference's own objects (tests/golden/asset_paths.json, recorded from
them), and the configuration and state it derives from them are the reference's values."""
import math

import numpy as np
import pytest

from helpers import MAP, params_for
from oracle import sit_oracle as so
from ref_assets import asset_paths, fixture_assets, polygon_obstacle, tree

compat = pytest.importorskip("sac_maritime_ast_amd.compat")


def test_paths_exist_on_reference_objects():
    ap = asset_paths()
    assert ap["paths"] == list(compat.ASSET_PATHS)
    for mode, case in ap["cases"].items():
        for snap in ("constructed", "stepped"):
            for who in ("test", "obs"):
                missing = [p for p, v in case[snap][who].items() if v is None]
                assert not missing, f"{mode} {snap} {who}: {missing}"


@pytest.mark.parametrize("mode,row", [("PTI", None), ("PTO", (so.SG_GEN, 2160e3, 0.0))])
def test_params_from_reference_objects(mode, row):
    """Every sit_params field derived from the reference's objects equals the value the reference
    configures (the oracle's DEFAULT_PARAMS, test_beds/test_policy.py:94-226), exactly."""
    case = asset_paths()["cases"][mode]["constructed"]
    assets = [tree(case["test"]), tree(case["obs"])]
    vals = [compat.read_asset(a) for a in assets]
    p = compat.params_from_assets(vals[0], vals[1], tree({"sampling_frequency": 7, "theta": 2}))
    got = p.as_dict()
    want = params_for(row)
    for k, v in want.items():
        if k in got:
            assert got[k] == v, f"{k}: {got[k]!r} vs {v!r}"


def test_live_state_from_stepped_reference_objects():
    """After reset / init_step / three steps with an IW inserted, the state read from the reference's
    objects: pose, shaft speed, integrals, waypoint index, the grown route, time and stop flags."""
    case = asset_paths()["cases"]["PTI"]["stepped"]
    vals = [compat.read_asset(tree(case[w])) for w in ("test", "obs")]
    scen, live = compat._scenario_from_assets(vals, MAP, 16)
    for t, w in enumerate(("test", "obs")):
        v = case[w]
        for f, k in zip(compat.POSE_FIELDS, ("north", "east", "yaw", "surge", "sway", "yaw_rate")):
            assert live[k][t, 0] == v["ship_model." + f]
            assert scen.init[0, t, compat.POSE_FIELDS.index(f)] == v["ship_model.init_" + f]
        assert live["shaft_speed"][t, 0] == v["ship_model.ship_machinery_model.omega"]
        assert live["ship_speed_i"][t, 0] == v["throttle_controller.ship_speed_controller.error_i"]
        assert live["shaft_speed_i"][t, 0] == v["throttle_controller.shaft_speed_controller.error_i"]
        hc = "auto_pilot.heading_controller.ship_heading_controller."
        assert live["heading_i"][t, 0] == v[hc + "error_i"] and live["heading_prev"][t, 0] == v[hc + "prev_error"]
        assert live["e_ct_int"][t, 0] == v["auto_pilot.navigate.e_ct_int"]
        assert live["next_wpt"][t, 0] == v["auto_pilot.next_wpt"]
        rn = v["auto_pilot.navigate.north"]
        assert live["n_wpt"][t, 0] == len(rn)
        assert list(live["wpt_north"][t, :len(rn) - 1, 0]) == rn[:-1]
        assert live["ticks"][t, 0] * 0.5 == v["ship_model.int.time"]
        assert live["stop"][t, 0] == int(v["stop_flag"])
        r0 = np.asarray(v["auto_pilot.navigate.init_route"])
        assert np.array_equal(scen.routes[0, t, :len(r0)], r0) and scen.n_wpt[0, t] == len(r0)
    assert live["n_wpt"][1, 0] == 3                  # the inserted IW (update_route at index -1)


def test_polygon_obstacle_and_degrees():
    polys = compat._polygons_of(polygon_obstacle())
    assert len(polys) == len(MAP)
    for p, m in zip(polys, MAP):
        assert np.array_equal(p, np.asarray(m, dtype=np.float64))
    assert all(np.array_equal(a, b) for a, b in zip(compat._polygons_of(MAP), polys))
    for deg in (30.0, 35.0, 12.5, 1.0 / 3.0):
        assert compat._degrees_of(deg * np.pi / 180) * math.pi / 180 == deg * np.pi / 180


def test_mismatched_ships_rejected():
    case = asset_paths()["cases"]["PTI"]["constructed"]
    obs = dict(case["obs"])
    obs["ship_model.ship_config.bunkers"] = 1.0
    vals = [compat.read_asset(tree(case["test"])), compat.read_asset(tree(obs))]
    with pytest.raises(ValueError, match="bunkers"):
        compat.params_from_assets(vals[0], vals[1])
    bad = dict(case["test"])
    del bad["auto_pilot.navigate.ra"]
    with pytest.raises(AttributeError, match="navigate.ra"):
        compat.read_asset(tree(bad), "assets[0]")


def test_fixture_assets_match_fixture():
    """The GPU tests' stand-ins for an env fixture carry its poses, routes and machinery mode."""
    from helpers import golden
    d = golden("env_blackout_pto")
    test, obs = fixture_assets(d)
    vals = [compat.read_asset(test), compat.read_asset(obs)]
    p = compat.params_from_assets(vals[0], vals[1])
    assert p.shaft_generator_state == so.SG_GEN and p.main_engine_capacity == float(d["mode"][1])
    scen, live = compat._scenario_from_assets(vals, MAP, 40)
    assert np.array_equal(scen.init[0, :, :6], d["pose"])
    assert np.array_equal(scen.routes[0], d["routes"][:, :40])
