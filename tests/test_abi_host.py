"""CPU checks of the C-ABI library and the host-side package (no compute calls: no GPU here)."""
import ctypes
import os
import re
from types import SimpleNamespace

import numpy as np
import pytest

from helpers import ROOT
from oracle import sit_oracle as so

sit = pytest.importorskip("sac_maritime_ast_amd")
from sac_maritime_ast_amd import _lib, config, scenario, status_string  # noqa: E402


def header_functions():
    src = open(os.path.join(ROOT, "include", "sit.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(sit_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    names = header_functions()
    assert len(names) >= 20
    raw = ctypes.CDLL(_lib.LIB_PATH)
    missing = [n for n in names if not hasattr(raw, n)]
    assert not missing, f"missing exports: {missing}"
    assert set(names) == set(_lib.SIGNATURES), "ctypes signatures out of sync with include/sit.h"
    assert lib.sit_abi_version() == 1


def test_params_layout_and_defaults_match_oracle():
    lib = _lib.load()
    assert lib.sit_params_size() == ctypes.sizeof(_lib.SitParams)
    d = config.params().as_dict()
    for k, v in so.DEFAULT_PARAMS.items():
        assert d[k] == pytest.approx(v, rel=0, abs=0), k


def test_create_without_device_fails_cleanly_or_succeeds():
    """sit_create needs a HIP device; on a GPU-less host it must return an error, not crash."""
    lib = _lib.load()
    h = ctypes.c_void_p()
    p = config.params()
    rc = lib.sit_create(ctypes.byref(p), 4, 8, 32, ctypes.byref(h))
    if rc == 0:
        lib.sit_destroy(h)
    else:
        assert rc in (_lib.SIT_E_HIP, _lib.SIT_E_NOMEM)
        assert lib.sit_last_error(None)


def test_create_rejects_bad_arguments():
    lib = _lib.load()
    h = ctypes.c_void_p()
    p = config.params()
    assert lib.sit_create(ctypes.byref(p), 0, 8, 32, ctypes.byref(h)) == _lib.SIT_E_INVALID
    assert b"n_env" in lib.sit_last_error(None)
    assert lib.sit_create(ctypes.byref(p), 4, 8, 16, ctypes.byref(h)) == _lib.SIT_E_INVALID
    assert lib.sit_create(ctypes.byref(p), 4, 1, 32, ctypes.byref(h)) == _lib.SIT_E_INVALID


def test_status_strings_match_oracle():
    rng = np.random.default_rng(0)
    for bits in [0, *rng.integers(0, 1 << 14, 500)]:
        assert status_string(int(bits)) == so.status_string(int(bits))


def test_params_from_reference_style_objects():
    ship = SimpleNamespace(dead_weight_tonnage=3850000, coefficient_of_deadweight_to_displacement=0.7,
                           bunkers=200000, ballast=200000, length_of_ship=80, width_of_ship=16,
                           added_mass_coefficient_in_surge=0.4, added_mass_coefficient_in_sway=0.4,
                           added_mass_coefficient_in_yaw=0.4, mass_over_linear_friction_coefficient_in_surge=130,
                           mass_over_linear_friction_coefficient_in_sway=18,
                           mass_over_linear_friction_coefficient_in_yaw=90,
                           nonlinear_friction_coefficient__in_surge=2500,
                           nonlinear_friction_coefficient__in_sway=4000, nonlinear_friction_coefficient__in_yaw=400)
    mode = SimpleNamespace(main_engine_capacity=2160e3, electrical_capacity=0.0, shaft_generator_state="GEN")
    mc = SimpleNamespace(hotel_load=200000, machinery_modes=SimpleNamespace(list_of_modes=[mode]),
                         machinery_operating_mode=0, rated_speed_main_engine_rpm=1000,
                         linear_friction_main_engine=68, linear_friction_hybrid_shaft_generator=57,
                         gear_ratio_between_main_engine_and_propeller=0.6,
                         gear_ratio_between_hybrid_shaft_generator_and_propeller=0.6, propeller_inertia=6000,
                         propeller_speed_to_torque_coefficient=7.5, propeller_diameter=3.1,
                         propeller_speed_to_thrust_force_coefficient=1.7,
                         rudder_angle_to_sway_force_coefficient=50e3, rudder_angle_to_yaw_force_coefficient=500e3,
                         max_rudder_angle_degrees=30)
    p = config.params_from_reference(ship_config=ship, machinery_config=mc,
                                     args=SimpleNamespace(sampling_frequency=9, theta=1.5))
    assert p.nonlinear_friction_coefficient_in_surge == 2500
    assert p.shaft_generator_state == _lib.SIT_SG_GEN and p.main_engine_capacity == 2160e3
    assert p.sampling_frequency == 9 and p.theta == 1.5
    assert config.shaft_speed_max(p) == pytest.approx(69.11503837897544)
    assert p.machinery_model == _lib.SIT_MACH_SHAFT


def test_params_from_reference_simplified_machinery():
    """A SimplifiedPropulsionMachinerySystemConfiguration (ship_engine.py:148-157) selects the
    SimplifiedMachineryModel; the (kp, ki) of ThrottleFromSpeedSetPointSimplifiedPropulsion
    (controllers.py:160-169) become the ship-speed PI gains."""
    mode = SimpleNamespace(main_engine_capacity=0.0, electrical_capacity=1020e3, shaft_generator_state="MOTOR")
    mc = SimpleNamespace(hotel_load=200000, machinery_modes=SimpleNamespace(list_of_modes=[mode]),
                         machinery_operating_mode=0, thrust_force_dynamic_time_constant=45.0,
                         rudder_angle_to_sway_force_coefficient=40e3, rudder_angle_to_yaw_force_coefficient=400e3,
                         max_rudder_angle_degrees=25)
    p = config.params_from_reference(machinery_config=mc, throttle_gains=SimpleNamespace(kp=2.0, ki=0.05))
    assert p.machinery_model == _lib.SIT_MACH_SIMPLIFIED and p.thrust_force_dynamic_time_constant == 45.0
    assert p.kp_ship_speed == 2.0 and p.ki_ship_speed == 0.05
    assert p.rudder_angle_to_sway_force_coefficient == 40e3 and p.max_rudder_angle_degrees == 25
    assert p.propeller_inertia == config.params().propeller_inertia     # shaft fields untouched


def test_scenario_matches_survey():
    sc = scenario.make_scenario(1, jitter=False)
    assert sc.init[0, 0, 2] == pytest.approx(1.4959364790841299, rel=1e-15)
    assert sc.init[0, 1, 2] == pytest.approx(-0.015623728620476831, rel=1e-15)
    big = scenario.make_scenario(4096)
    d = big.init[:, :, :2] - sc.init[:, :, :2]
    assert np.abs(d).max() <= 100.0 and np.abs(big.init[:, :, 2] - sc.init[:, :, 2]).max() <= 0.05
    o = so.OracleEnvs(dict(so.DEFAULT_PARAMS), sc.routes, sc.n_wpt, sc.init, sc.polys)
    assert o.ab_len[0] == pytest.approx(914.3973146174434, rel=1e-14)


def _host_handle(lib, n_env=64, cap=32, precision=32):
    """A handle for the setup calls, or None where sit_create needs a GPU that is absent (the
    sanitizer build, tools/sanitize.sh, backs the setup memory with host memory instead)."""
    h = ctypes.c_void_p()
    p = config.params()
    rc = lib.sit_create(ctypes.byref(p), n_env, cap, precision, ctypes.byref(h))
    if rc != 0:
        return None
    return h


@pytest.mark.parametrize("precision", [32, 64])
def test_setup_calls_host_logic(precision):
    """sit_load_map / sit_load_routes / sit_load_initial / sit_map_info / sit_state_field on the
    scenario of SURVEY §8(d): argument checks, the spatial index build and the blob layout (no
    kernel is launched).  Runs where a handle can be created: the GPU box, and the host-memory
    sanitizer build (tools/sanitize.sh, ASan + UBSan)."""
    lib = _lib.load()
    n_env, cap = 64, 32
    h = _host_handle(lib, n_env, cap, precision)
    if h is None:
        pytest.skip("sit_create needs a HIP device (use the sanitizer build for host-only runs)")
    try:
        sc = scenario.make_scenario(n_env, cap=cap)
        polys = [np.ascontiguousarray(p, dtype=np.float64) for p in sc.polys]
        offs = np.zeros(len(polys) + 1, dtype=np.int32)
        offs[1:] = np.cumsum([len(p) for p in polys])
        verts = np.ascontiguousarray(np.concatenate(polys))
        vp = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        assert lib.sit_load_map(h, len(polys), vp(offs), vp(verts)) == 0, lib.sit_last_error(h)
        bad = offs.copy()
        bad[1] = 2
        assert lib.sit_load_map(h, len(polys), vp(bad), vp(verts)) == _lib.SIT_E_INVALID
        info = np.zeros(6, dtype=np.int64)
        assert lib.sit_map_info(h, vp(info), 6) == 0
        assert info[0] > 0 and info[1] > 1000 and info[2] > 1000 and info[5] >= info[0]
        routes = np.ascontiguousarray(sc.routes, dtype=np.float64)
        n_wpt = np.ascontiguousarray(sc.n_wpt, dtype=np.int32)
        assert lib.sit_load_routes(h, vp(routes), vp(n_wpt)) == 0, lib.sit_last_error(h)
        bad_n = n_wpt.copy()
        bad_n[3, 1] = cap + 1
        assert lib.sit_load_routes(h, vp(routes), vp(bad_n)) == _lib.SIT_E_INVALID
        init = np.ascontiguousarray(sc.init, dtype=np.float64)
        assert lib.sit_load_initial(h, vp(init)) == 0, lib.sit_last_error(h)
        nbytes = ctypes.c_size_t()
        assert lib.sit_state_bytes(h, ctypes.byref(nbytes)) == 0
        end = 0
        for f in range(lib.sit_state_nfields()):
            name, off, dt, cnt = ctypes.c_char_p(), ctypes.c_size_t(), ctypes.c_int32(), ctypes.c_int64()
            assert lib.sit_state_field(h, f, ctypes.byref(name), ctypes.byref(off), ctypes.byref(dt),
                                       ctypes.byref(cnt)) == 0
            assert off.value % 256 == 0 and off.value >= end and cnt.value > 0
            el = (precision // 8) if dt.value == _lib.SIT_DT_REAL else 4
            end = off.value + cnt.value * el
        assert end <= nbytes.value
    finally:
        lib.sit_destroy(h)


def test_jittered_starts_fixture_n4096():
    """The benchmark scenario's jittered starts for N = 4096, committed by
    tests/golden/make_scenario_fixture.py: reproduced bit for bit, also by shards of the
    population (env_offset), within +-100 m and +-0.05 rad of the unjittered starts."""
    d = np.load(os.path.join(ROOT, "tests", "golden", "scenario_jitter_4096.npz"))
    sc = scenario.make_scenario(4096, seed=int(d["seed"]))
    assert np.array_equal(sc.init[:, :, 0], d["start_north"])
    assert np.array_equal(sc.init[:, :, 1], d["start_east"])
    assert np.array_equal(sc.init[:, :, 2], d["start_yaw"])
    half = scenario.make_scenario(2048, seed=int(d["seed"]), env_offset=2048)
    assert np.array_equal(half.init[:, :, :3], sc.init[2048:, :, :3])
    base = scenario.make_scenario(1, jitter=False).init[0]
    assert np.abs(d["start_north"] - base[:, 0]).max() <= 100.0
    assert np.abs(d["start_yaw"] - base[:, 2]).max() <= 0.05
