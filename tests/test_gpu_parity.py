"""GPU parity: the HIP path (libsit.so through the C ABI) against the reference fixtures and the
CPU oracle.  All tests here run on an MI355X (``-m gpu``).

Contract:
  * float64 handle: bit-faithful arithmetic order; teacher-forced and free-running results
    within 1e-9 relative (per-field scale floors), waypoint index / stop flags / done / status
    identical.  The remaining differences are ocml-vs-libm transcendental ulps.
  * float32 handle: teacher-forced one step from float32-rounded states within 1e-5 relative
    (per-field floors); discrete outputs identical except where the oracle's own decision
    margin lies inside the float32 band (counted and bounded).
"""
import json
import os
import sys

import numpy as np
import pytest
import torch

from helpers import (OBS_SCALE, POLYS, SCALE, env_oracle, env_state_all_rows, env_state_from, golden,
                     golden_names, init_rows, params_for, rel_err)
from oracle import sit_oracle as so

pytestmark = pytest.mark.gpu

sit = pytest.importorskip("sac_maritime_ast_amd")
from sac_maritime_ast_amd import VecMultiShipRLEnv, _lib, make_scenario, status_string  # noqa: E402
from sac_maritime_ast_amd.config import params as sit_params  # noqa: E402
from sac_maritime_ast_amd.scenario import Scenario  # noqa: E402

DEV = "cuda:0"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOL64 = 1e-9
ENV_CASES = golden_names("env_")


def gpu_params(mode_row=None, **over):
    p = params_for(mode_row, **over)
    kw = {k: v for k, v in p.items() if k in sit_params().as_dict()}
    return sit_params(**kw)


def fixture_env(d, n_env, precision):
    sc = Scenario(np.repeat(d["routes"][None], n_env, 0), np.repeat(d["n_wpt"][None], n_env, 0).astype(np.int32),
                  init_rows(np.repeat(d["pose"][None], n_env, 0)), POLYS)
    return VecMultiShipRLEnv(scenario=sc, params=gpu_params(d["mode"]), precision=precision, device=DEV)


def np_state(env):
    return {k: v.cpu().numpy() for k, v in env.get_state().items()}


def check_state(got, want, tol, where, int_fields=so.SHIP_INT, real_fields=so.SHIP_REAL):
    for k in int_fields:
        assert np.array_equal(got[k].astype(np.int64), np.asarray(want[k]).astype(np.int64)), f"{where}: {k}"
    for k in real_fields:
        err = rel_err(got[k], want[k], SCALE[k]).max()
        assert err <= tol, f"{where}: {k} rel err {err:.3e}"


# ------------------------------------------------------------------------------------------
# float64: against the reference's own outputs
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ENV_CASES)
def test_f64_teacher_forced_vs_reference(name):
    d = golden(name)
    T = len(d["reward"])
    o = env_oracle(d, n_env=T)
    st = env_state_all_rows(d, "pre_", o)
    env = fixture_env(d, T, 64)
    env.set_state(st)
    act = np.stack([d["action_n"], d["action_e"]], axis=1)
    ns, rew, done, status = env.step(act, d["sac_update"], d["init"])
    ns, rew, done, status = ns.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy(), status.cpu().numpy()
    assert rel_err(ns, d["next_state"], OBS_SCALE).max() <= TOL64
    assert rel_err(rew, d["reward"], 1.0).max() <= TOL64
    assert np.array_equal(done, d["done"].astype(bool))
    for i in range(T):
        assert status_string(int(status[i])) == str(d["status"][i]), f"{name} step {i}"
    post = np_state(env)
    want = {k: d["post_" + k].T for k in so.SHIP_REAL + so.SHIP_INT}
    check_state(post, want, TOL64, name)
    for k in ("sampling_dist", "eps_dist", "prev_pre_north", "prev_pre_east"):
        assert rel_err(post[k], d["post_" + k], SCALE[k]).max() <= TOL64, k


@pytest.mark.parametrize("name", ENV_CASES)
def test_f64_free_running_vs_reference(name):
    """Whole recorded episodes as fused multi-step launches with the recorded actions."""
    d = golden(name)
    T = len(d["reward"])
    env = fixture_env(d, 1, 64)
    assert np.array_equal(env.reset()[0].cpu().numpy(), d["reset_state"].astype(np.float64))
    o = env_oracle(d)
    env.set_state(env_state_from(d, "pre_", 0, o))
    bounds = sorted({0, T, *[int(r) for r in d["resets"] if 0 < r < T]})
    for a, b in zip(bounds[:-1], bounds[1:]):
        if a > 0:
            env.reset()
            env.init_step()
        acts = {"action_ne": np.stack([d["action_n"][a:b], d["action_e"][a:b]], 1)[:, None, :],
                "sac_update": d["sac_update"][a:b, None], "init": d["init"][a:b, None]}
        out = env.rollout(b - a, actions=acts, auto_reset=False)
        ns = out["next_state"][:, 0].cpu().numpy()
        assert rel_err(ns, d["next_state"][a:b], OBS_SCALE).max() <= TOL64, f"{name} [{a},{b})"
        assert rel_err(out["reward"][:, 0].cpu().numpy(), d["reward"][a:b], 1.0).max() <= TOL64
        st = out["status"][:, 0].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        for i in range(b - a):
            assert status_string(int(st[i])) == str(d["status"][a + i]), f"{name} step {a + i}"


# ------------------------------------------------------------------------------------------
# float64: synthetic-sampler rollouts against the oracle, auto-reset included (4096 envs = 8192
# ships, a superset of C2's 4096 ships; and 256 envs over long episodes)
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n_env,steps", [(4096, 300), (256, 2500)])
def test_f64_synthetic_rollout_vs_oracle(n_env, steps):
    sc = make_scenario(n_env, cap=32)
    env = VecMultiShipRLEnv(scenario=sc, precision=64, device=DEV)
    env.reset()
    env.init_step()
    o = so.OracleEnvs(dict(so.DEFAULT_PARAMS), sc.routes, sc.n_wpt, sc.init, sc.polys)
    o.reset()
    o.init_step()
    chunk = 100
    for k0 in range(0, steps, chunk):
        out = env.rollout(chunk, seed=25450)
        r = o.rollout(chunk, seed=25450)
        where = f"steps [{k0},{k0 + chunk})"
        assert rel_err(out["next_state"].cpu().numpy(), r["next_state"], OBS_SCALE).max() <= TOL64, where
        assert rel_err(out["reward"].cpu().numpy(), r["reward"], 1.0).max() <= TOL64, where
        assert np.array_equal(out["done"].cpu().numpy().astype(bool), r["done"]), where
        assert np.array_equal(out["status"].cpu().numpy().astype(np.int64) & 0xFFFFFFFF,
                              r["status"].astype(np.int64)), where
        act = out["action"].cpu().numpy()
        assert np.array_equal(np.isnan(act[..., 2]), np.isnan(r["action"][..., 2])), where
        assert rel_err(act[..., :2], r["action"][..., :2], 1e4).max() <= TOL64, where
        assert np.array_equal(out["done_count"].cpu().numpy(), r["done"].sum(axis=1)), where
    check_state(np_state(env), o.get_state(), 1e-8, "final state",
                int_fields=so.SHIP_INT + ("ep_step", "event", "episodes"))


# ------------------------------------------------------------------------------------------
# float32: teacher-forced one step against the oracle
# ------------------------------------------------------------------------------------------
def test_f32_teacher_forced_vs_oracle():
    n_env = 4096
    sc = make_scenario(n_env, cap=32)
    # realistic pre-states: a float64 rollout, snapshotted at several depths
    env64 = VecMultiShipRLEnv(scenario=sc, precision=64, device=DEV)
    env64.reset()
    env64.init_step()
    env32 = VecMultiShipRLEnv(scenario=sc, precision=32, device=DEV)
    o = so.OracleEnvs(dict(so.DEFAULT_PARAMS), sc.routes, sc.n_wpt, sc.init, sc.polys)
    worst = {}
    n_disc = 0
    for depth in range(6):
        env64.rollout(250, seed=11 + depth)
        st = np_state(env64)
        st32 = {k: (v.astype(np.float32).astype(np.float64) if v.dtype == np.float64 else v) for k, v in st.items()}
        o.set_state(st32)
        env32.set_state(st32)
        rng = np.random.default_rng(depth)
        sac = rng.random(n_env) < 0.1
        ang = rng.uniform(-np.pi / 6, np.pi / 6, n_env)
        act = np.stack([st32["north"][1] + o.ab_len * np.cos(o.ab_alpha + ang),
                        st32["east"][1] + o.ab_len * np.sin(o.ab_alpha + ang)], 1)
        act = act.astype(np.float32).astype(np.float64)
        init = np.zeros(n_env, bool)
        ns_r, rew_r, done_r, st_r = o.step(act, sac, init)
        ns, rew, done, stat = env32.step(act, sac, init)
        ns, rew, done, stat = ns.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy(), stat.cpu().numpy()
        e = rel_err(ns, ns_r, OBS_SCALE)
        worst["next_state"] = max(worst.get("next_state", 0), e.max())
        # reward: terms up to 2000 plus O(1) shaping; tolerance 1e-5 * max(|r|, 1)
        e = rel_err(rew, rew_r, 1.0)
        worst["reward"] = max(worst.get("reward", 0), e.max())
        n_disc += int(((done != done_r) | (stat != st_r)).sum())
        post = np_state(env32)
        ref = o.get_state()
        for k in so.SHIP_REAL:
            worst[k] = max(worst.get(k, 0), rel_err(post[k], ref[k], SCALE[k]).max())
        for k in ("next_wpt", "n_wpt", "stop"):
            assert np.array_equal(post[k], ref[k]), f"depth {depth}: {k}"
    print("f32 teacher-forced worst:", {k: f"{v:.2e}" for k, v in worst.items()}, "discrete mismatches:", n_disc)
    for k, v in worst.items():
        assert v <= 1e-5, f"{k}: {v:.3e}"
    assert n_disc == 0, f"{n_disc} done/status mismatches"


# ------------------------------------------------------------------------------------------
# API behaviour
# ------------------------------------------------------------------------------------------
def test_state_roundtrip_and_masks():
    sc = make_scenario(300, cap=16)
    env = VecMultiShipRLEnv(scenario=sc, precision=64, device=DEV)
    env.reset()
    env.init_step()
    env.rollout(50, seed=3)
    blob = env.state_blob()
    out1 = env.rollout(20, seed=4)
    env.load_state_blob(blob)
    out2 = env.rollout(20, seed=4)
    assert torch.equal(out1["next_state"], out2["next_state"])
    # masked reset touches only masked envs; shaft speed and integrators persist (Q6)
    before = np_state(env)
    mask = np.zeros(300, bool)
    mask[::3] = True
    init_obs = env.reset(mask).cpu().numpy()
    after = np_state(env)
    assert np.array_equal(after["north"][:, ~mask], before["north"][:, ~mask])
    assert np.allclose(after["north"][:, mask], sc.init[mask, :, 0].T)
    for k in ("shaft_speed", "ship_speed_i", "shaft_speed_i", "heading_i", "heading_prev"):
        assert np.array_equal(after[k], before[k]), k
    assert np.all(after["next_wpt"][:, mask] == 1) and np.all(after["e_ct_int"][:, mask] == 0)
    assert np.allclose(init_obs[:, 0], sc.init[:, 0, 0].astype(np.float32))


def test_route_overflow_flag():
    """Insertions beyond the route capacity are dropped and flagged (SIT_ST_ROUTE_OVERFLOW)."""
    sc = make_scenario(64, cap=5)            # obstacle route 2 waypoints -> room for 3 IWs
    env = VecMultiShipRLEnv(scenario=sc, precision=64, device=DEV)
    env.reset()
    env.init_step()
    st = np_state(env)
    act = np.stack([st["north"][1] + 500.0, st["east"][1]], 1)
    flags = []
    for i in range(5):
        _, _, _, status = env.step(act, np.ones(64, bool), np.full(64, i == 0))
        flags.append(status.cpu().numpy())
    nw = np_state(env)["n_wpt"][1]
    assert np.all(nw == 5)
    for i in range(3):
        assert not (flags[i] & (1 << 31)).any()
    assert (flags[3] & (1 << 31)).all() and (flags[4] & (1 << 31)).all()


def test_done_count_and_large_batch_sanity():
    """C3 size: 65 536 ships (32 768 envs) fused rollout; finite outputs, done_count = sum(done)."""
    env = VecMultiShipRLEnv(n_env=32768, precision=32, device=DEV)
    env.reset()
    env.init_step()
    out = env.rollout(500, seed=1)
    torch.cuda.synchronize()
    assert torch.isfinite(out["next_state"]).all()
    assert torch.isfinite(out["reward"]).all()
    assert torch.equal(out["done_count"].to(torch.int64), out["done"].to(torch.int64).sum(1))


def test_f64_replay_transitions_vs_oracle():
    """Sampling-event transitions (memory.push of test_beds/main_ast.py:385-396) written by the
    kernel match the oracle's, as a set (the kernel appends with atomics)."""
    n_env = 1024
    sc = make_scenario(n_env, cap=32)
    env = VecMultiShipRLEnv(scenario=sc, precision=64, device=DEV)
    env.reset()
    env.init_step()
    o = so.OracleEnvs(dict(so.DEFAULT_PARAMS), sc.routes, sc.n_wpt, sc.init, sc.polys)
    o.reset()
    o.init_step()
    total = 0
    for _ in range(8):
        out = env.rollout(150, seed=99, transition_capacity=8192, mask_horizon=600)
        r = o.rollout(150, seed=99, mask_horizon=600)
        cnt = int(out["transition_count"].item())
        want = r["transitions"]
        assert cnt == len(want)
        total += cnt
        if cnt == 0:
            continue
        got = out["transitions"][:cnt].cpu().numpy()
        key = lambda a: np.lexsort((a[:, 12], a[:, 23]))  # noqa: E731
        got, want = got[key(got)], want[key(want)]
        assert np.array_equal(got[:, 23], want[:, 23])
        assert np.array_equal(got[:, 22], want[:, 22])
        cols = np.r_[0:10, 12:22]
        assert rel_err(got[:, cols], want[:, cols], np.r_[OBS_SCALE, OBS_SCALE]).max() <= TOL64
        assert rel_err(got[:, 10:12], want[:, 10:12], 1.0).max() <= TOL64
    assert total > 2 * n_env


def test_misaligned_output_rejected():
    """Rows are written with paired stores: a next_state pointer off the 2-real alignment is
    refused with SIT_E_INVALID (and nothing is launched), an aligned one is accepted."""
    n = 64
    env = VecMultiShipRLEnv(scenario=make_scenario(n), precision=32, device=DEV)
    env.reset()
    env.init_step()
    a = torch.zeros((n, 2), dtype=torch.float32, device=DEV)
    flags = torch.zeros((n,), dtype=torch.uint8, device=DEV)
    buf = torch.zeros((n * 10 + 1,), dtype=torch.float32, device=DEV)
    rew = torch.zeros((n,), dtype=torch.float32, device=DEV)
    with pytest.raises(_lib.SitError, match="aligned"):
        env._call("sit_step", a.data_ptr(), flags.data_ptr(), flags.data_ptr(), buf.data_ptr() + 4,
                  rew.data_ptr(), None, None, None, env._stream())
    env._call("sit_step", a.data_ptr(), flags.data_ptr(), flags.data_ptr(), buf.data_ptr(),
              rew.data_ptr(), None, None, None, env._stream())
    torch.cuda.synchronize()
    assert torch.isfinite(buf[:n * 10]).all()


def test_f32_sampler_iw_vs_oracle():
    """The float32 handle's synthetic sampler: IW points of sampling events from float32 states
    within 1e-5 relative of the oracle's float64 IW for the same state and draw."""
    n_env = 4096
    sc = make_scenario(n_env, cap=32)
    env64 = VecMultiShipRLEnv(scenario=sc, precision=64, device=DEV)
    env64.reset()
    env64.init_step()
    env64.rollout(137, seed=5)
    st = np_state(env64)
    st32 = {k: (v.astype(np.float32).astype(np.float64) if v.dtype == np.float64 else v) for k, v in st.items()}
    # force a sampling event in every env: episode step 0 (init event)
    st32["ep_step"] = np.zeros_like(st32["ep_step"])
    env32 = VecMultiShipRLEnv(scenario=sc, precision=32, device=DEV)
    env32.set_state(st32)
    o = so.OracleEnvs(dict(so.DEFAULT_PARAMS), sc.routes, sc.n_wpt, sc.init, sc.polys)
    o.set_state(st32)
    act_r, sac_r, _, ang_r = o.sampler_actions(25450)
    out = env32.rollout(1, seed=25450, auto_reset=False)
    a = out["action"][0].cpu().numpy().astype(np.float64)
    assert np.array_equal(a[:, 3] > 0.5, sac_r)
    assert np.abs(a[:, 2] - ang_r).max() <= 1e-6
    err = np.abs(a[:, :2] - act_r) / np.maximum(np.abs(act_r), 1e4)
    assert err.max() <= 1e-5, f"IW rel err {err.max():.3e}"


def test_f32_action_rows_nan_without_sample():
    """The float32 step kernels run with finite math: the action row's angle must
    still be NaN exactly on the rows without a sampling event, and finite on the others."""
    n_env = 2048
    env = VecMultiShipRLEnv(scenario=make_scenario(n_env, cap=48), precision=32, device=DEV)
    env.reset()
    env.init_step()
    out = env.rollout(300, seed=11)
    a = out["action"].cpu().numpy()
    sac = a[..., 3] > 0.5
    assert sac.any() and (~sac).any()
    assert np.isnan(a[..., 2][~sac]).all()
    assert np.isfinite(a[..., 2][sac]).all() and np.abs(a[..., 2][sac]).max() <= np.pi / 6 + 1e-6


# ------------------------------------------------------------------------------------------
# trajectory logs (simulation_results rows, fuel model, reward_results terms)
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ENV_CASES)
def test_f64_trajectory_log_vs_reference(name):
    """The rollout's log (log=True) of recorded episodes against the reference's own
    simulation_results of both ships and its reward_results running sums."""
    from sac_maritime_ast_amd.trajectory import reward_results, simulation_results
    d = golden(name)
    T = len(d["reward"])
    env = fixture_env(d, 1, 64)
    env.reset()
    o = env_oracle(d)
    env.set_state(env_state_from(d, "pre_", 0, o))
    bounds = sorted({0, T, *[int(r) for r in d["resets"] if 0 < r < T]})
    logs = []
    for a, b in zip(bounds[:-1], bounds[1:]):
        if a > 0:
            env.reset()
            env.init_step()
        acts = {"action_ne": np.stack([d["action_n"][a:b], d["action_e"][a:b]], 1)[:, None, :],
                "sac_update": d["sac_update"][a:b, None], "init": d["init"][a:b, None]}
        logs.append(env.rollout(b - a, actions=acts, auto_reset=False, log=True)["log"].cpu().numpy())
    log = np.concatenate(logs)
    for ship, key in ((0, "log_test"), (1, "log_obs")):
        got = np.stack(list(simulation_results(log, 0, ship).values()), axis=1)
        err = np.abs(got - d[key]) / np.maximum(np.abs(d[key]), 1.0)
        assert err.max() <= 1e-9, f"{name} {key}: rel err {err.max():.3e} at {np.unravel_index(err.argmax(), err.shape)}"
    starts = np.zeros(T, bool)
    starts[[r for r in d["resets"] if 0 <= r < T]] = True
    rr = reward_results(log, 0, starts)
    got = np.stack([rr[a][b] for a, b in (("test_ship", "reward_e_ct"), ("test_ship", "reward_near_col"),
                                          ("test_ship", "total_non_terminal"), ("obs_ship", "reward_base"),
                                          ("obs_ship", "reward_e_ct"), ("obs_ship", "reward_near_col"),
                                          ("obs_ship", "total_non_terminal"), ("shared", "total_non_terminal"))], 1)
    err = np.abs(got - d["log_reward"]) / np.maximum(np.abs(d["log_reward"]), 1.0)
    assert err.max() <= 1e-9, f"{name} reward_results: rel err {err.max():.3e}"


def test_f64_synthetic_rollout_log_vs_oracle():
    n_env, steps = 512, 400
    sc = make_scenario(n_env, cap=32)
    env = VecMultiShipRLEnv(scenario=sc, precision=64, device=DEV)
    env.reset()
    env.init_step()
    o = so.OracleEnvs(dict(so.DEFAULT_PARAMS), sc.routes, sc.n_wpt, sc.init, sc.polys)
    o.reset()
    o.init_step()
    o.start_log()
    out = env.rollout(steps, seed=77, log=True)
    o.rollout(steps, seed=77)
    log = out["log"].cpu().numpy()
    ref_ship = np.array(o.log["ship"])                 # [K, 2, 27, n]
    ref = np.concatenate([ref_ship[:, 0], ref_ship[:, 1], np.array(o.log["reward"])], axis=1)
    err = np.abs(log - ref) / np.maximum(np.abs(ref), 1.0)
    assert err.max() <= 1e-9, f"log rel err {err.max():.3e} at {np.unravel_index(err.argmax(), err.shape)}"
    st = np_state(env)
    for k in ("fuel_me", "fuel_el", "fuel"):
        assert rel_err(st[k], o.s[k], 1.0).max() <= 1e-9, k


def test_f32_rollout_log_sanity():
    n_env = 4096
    env = VecMultiShipRLEnv(scenario=make_scenario(n_env, cap=32), precision=32, device=DEV)
    env.reset()
    env.init_step()
    out = env.rollout(200, seed=3, log=True)
    log = out["log"]
    assert torch.isfinite(log).all()
    # the log's pose is the pre-integration state: row k+1's north equals next_state row k's north
    # for the ship under test when no reset happened in between
    ns = out["next_state"]
    same = ~out["done"][:-1].bool()
    assert torch.equal(log[1:, 1][same], ns[:-1, :, 0][same])


# ------------------------------------------------------------------------------------------
# float32: the benchmarked instantiation (k_env_steps<float, kSynth, LDS map, no log>, device
# fast-math) — one fused step from float32 states at six depths of an episode
# ------------------------------------------------------------------------------------------
def f32_rounded(st):
    return {k: (v.astype(np.float32).astype(np.float64) if v.dtype == np.float64 else v) for k, v in st.items()}


def test_f32_synthetic_rollout_step_vs_oracle():
    """rollout(1) in synthetic-sampler mode with auto-reset — the kernel and flags the bench times —
    from float32-rounded states of 4096 envs at six episode depths, against OracleEnvs.rollout(1)
    on the same state: next_state, reward, IW actions and the post-state within 1e-5 relative
    (per-field floors); done, status, sampling events, waypoint index, route length, stop flags,
    episode counters and the replay transitions' discrete fields identical."""
    n_env = 4096
    sc = make_scenario(n_env, cap=32)
    env64 = VecMultiShipRLEnv(scenario=sc, precision=64, device=DEV)
    env64.reset()
    env64.init_step()
    env32 = VecMultiShipRLEnv(scenario=sc, precision=32, device=DEV)
    o = so.OracleEnvs(dict(so.DEFAULT_PARAMS), sc.routes, sc.n_wpt, sc.init, sc.polys)
    worst, n_done, n_sac = {}, 0, 0

    def upd(k, v):
        worst[k] = max(worst.get(k, 0.0), float(v))
    for depth in range(6):
        env64.rollout(300, seed=21 + depth)
        st32 = f32_rounded(np_state(env64))
        o.set_state(st32)
        env32.set_state(st32)
        seed = 900 + depth
        r = o.rollout(1, seed=seed, mask_horizon=600)
        out = env32.rollout(1, seed=seed, transition_capacity=2 * n_env, mask_horizon=600)
        ns, rew = out["next_state"][0].cpu().numpy(), out["reward"][0].cpu().numpy()
        upd("next_state", rel_err(ns, r["next_state"][0], OBS_SCALE).max())
        upd("reward", rel_err(rew, r["reward"][0], 1.0).max())
        done = out["done"][0].cpu().numpy().astype(bool)
        stat = out["status"][0].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        assert np.array_equal(done, r["done"][0]), f"depth {depth}: done"
        assert np.array_equal(stat, r["status"][0].astype(np.int64)), f"depth {depth}: status"
        n_done += int(done.sum())
        act = out["action"][0].cpu().numpy().astype(np.float64)
        sac = r["action"][0, :, 3] > 0.5
        n_sac += int(sac.sum())
        assert np.array_equal(act[:, 3] > 0.5, sac), f"depth {depth}: sampling events"
        upd("iw", rel_err(act[sac, :2], r["action"][0, sac, :2], 1e4).max() if sac.any() else 0.0)
        post, ref = np_state(env32), o.get_state()
        for k in so.SHIP_REAL:
            upd(k, rel_err(post[k], ref[k], SCALE[k]).max())
        for k in ("sampling_dist", "eps_dist", "prev_pre_north", "prev_pre_east", "iw_north", "iw_east"):
            upd(k, rel_err(post[k], ref[k], SCALE[k]).max())
        for k in so.SHIP_INT + ("ep_step", "event", "episodes"):
            assert np.array_equal(post[k].astype(np.int64), ref[k].astype(np.int64)), f"depth {depth}: {k}"
        cnt = int(out["transition_count"].item())
        got, want = out["transitions"][:cnt].cpu().numpy().astype(np.float64), r["transitions"]
        assert cnt == len(want), f"depth {depth}: transitions {cnt} vs {len(want)}"
        if cnt:
            got, want = got[np.argsort(got[:, 23])], want[np.argsort(want[:, 23])]
            assert np.array_equal(got[:, 23], want[:, 23]) and np.array_equal(got[:, 22], want[:, 22])
            assert np.abs(got[:, 10] - want[:, 10]).max() <= 1e-6      # the SAC action in [-1, 1]
            cols = np.r_[0:10, 12:22]
            upd("transitions", rel_err(got[:, cols], want[:, cols], np.r_[OBS_SCALE, OBS_SCALE]).max())
    print("f32 benchmarked-kernel step worst:", {k: f"{v:.2e}" for k, v in worst.items()},
          f"done {n_done}, sampling events {n_sac}")
    bad = {k: f"{v:.2e}" for k, v in worst.items() if v > 1e-5}
    assert not bad, bad
    assert n_sac > 0


def test_f32_free_running_within_storage_bound():
    """float32 free-running against float64 from identical starts, 4096 envs x 2000
    steps of the synthetic sampler with auto-reset, one step per launch (tools/f32_drift.py), and the
    same episodes as the bench runs them (fused 200-step launches), bit for bit equal to the one-step
    run.  A third run, the float64 kernel with its state rounded to float32 after every step, isolates what float32
    state STORAGE alone costs.  Per env the runs are compared until the first step whose discrete
    outcome differs (done, status, sampling event, waypoint index, route length, stop flags, episode
    step, sampler counter).  Gated: before divergence the next_state deviation (per-field floors) is
    within north_star's 1e-5 and below what plain float32 storage alone costs (the float32 handle keeps
    its integrators as double-float values); at most 0.1 % of envs diverge (measured: none).  Every divergence is attributed
    (f32_drift.measure(attribute=True)): re-run in float64 from the float32 run's own pre-step state,
    the step takes the float32 decision (the state's float32 drift decided it), or, where it takes the
    float64 one, the flip is a hull-in-terrain decision whose exact (float64) predicate at the stored
    float32 post-step position IS the float32 decision, with a hull corner closer to the shore than the
    two runs' positions differ (the float32 rounding of the position moved it, not the predicate's
    arithmetic)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import f32_drift
    rep = f32_drift.measure(4096, 2000, 77, log=False, attribute=True, fused_chunk=200)
    rec = os.environ.get("SIT_TEST_RECORD_DIR")
    if rec:
        with open(os.path.join(rec, "f32_flip_attribution.json"), "w") as f:
            json.dump(rep, f, indent=1)
    # the benchmarked instantiation (fused 200-step launches, LDS-staged map, transitions written) gives
    # the one-step run's outputs and states bit for bit, so every bound below holds for it
    fz = rep["fused"]
    assert fz["kernel"].startswith("k_env_steps_sync<float") and "map=LDS" in fz["kernel"], fz["kernel"]
    assert fz["envs_differing_from_one_step_run"] == 0
    att = rep["f32_flip_attribution"]
    assert att["envs"] == rep["f32"]["envs_diverged"] and att["neither"] == 0
    for f in att["flips"]:
        if f["exact_from_f32_state_takes"] == "f32 decision":
            continue
        assert f["hull"], f"env {f['env']} step {f['step']}: float32 arithmetic flipped {f['flipped']}"
        t = 1 if (f["status_bits_f32"] ^ f["status_bits_f64"]) & _lib.ST_OBS_TERRAIN else 0
        h = f["hull"][f"ship{t}"]
        got32 = bool(f["status_bits_f32"] & (_lib.ST_OBS_TERRAIN if t else _lib.ST_TEST_TERRAIN))
        assert h["hull_in_terrain_exact_at_f32_position"] == got32, f"env {f['env']}: hull predicate"
        assert min(h["min_corner_boundary_distance_m_f32"], h["min_corner_boundary_distance_m_f64"]) \
            <= h["position_difference_m"], f"env {f['env']}: not a position knife edge"
    f32, s32 = rep["f32"], rep["s32"]
    print(f"f32 vs f64 free-running: {f32['envs_diverged']} envs diverged (earliest step "
          f"{f32['earliest_divergence_step']}), next_state max {f32['next_state_max']:.2e} p99 "
          f"{f32['next_state_p99']:.2e}; float32 storage alone: {s32['envs_diverged']} diverged, max "
          f"{s32['next_state_max']:.2e}")
    # north_star's 1e-5 before any decision moves; the double-float integrators (csrc/sit_device.h
    # comp_add) took float32 below what float32 state storage alone costs (round 4, plain float32 sums:
    # 38 envs diverged, max 9.95e-6; round 5: 9 envs, max 3.5e-6, profiles/r05_f32_flip_attribution.json)
    assert f32["next_state_max"] <= 1e-5
    assert f32["next_state_max"] <= s32["next_state_max"]
    # round 6, every integrator double-float: 0 of 4 096 envs diverge (round 5: 8); a margin of 0.1 %
    assert f32["envs_diverged"] <= 4
    # every real state field of both ships (pose, velocities, shaft speed, the PI / PID / LOS integrals, the
    # previous heading error) within the same 1e-5 before divergence.  (The heading PID integral, the time
    # integral of the heading error, follows the trajectory; it read 1.43e-5 until round 6 carried surge, sway,
    # yaw rate and shaft speed as double-float values too: 7.0e-6, with 0 of 4 096 envs diverging,
    # profiles/r06_heading_i_storage_attribution.json)
    sp = f32["state_per_field_max"]
    worst = max(sp, key=sp.get)
    assert sp[worst] <= 1e-5, (worst, sp)


# ------------------------------------------------------------------------------------------
# sharding: envs are independent units keyed by global env id
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("precision", [64, 32])
def test_two_shards_equal_one_handle(precision):
    """Two handles with env_id_offset 0 and n reproduce one 2n-env handle bit for bit (the path the
    multi-GPU bench runs on every rank), including the replay transitions."""
    n, steps = 1024, 400
    outs = []
    for parts in (((0, 2 * n),), ((0, n), (n, n))):
        res = []
        for off, cnt in parts:
            env = VecMultiShipRLEnv(scenario=make_scenario(cnt, cap=48, env_offset=off), precision=precision,
                                    device=DEV)
            env.reset()
            env.init_step()
            o = env.rollout(steps, seed=31, env_id_offset=off, transition_capacity=4 * cnt)
            tr = o["transitions"][:int(o["transition_count"].item())].cpu().numpy()
            res.append((o["next_state"].cpu().numpy(), o["reward"].cpu().numpy(), o["status"].cpu().numpy(),
                        tr[np.lexsort((tr[:, 12], tr[:, 23]))]))
        outs.append(res)
    (ns, rw, st, tr), = outs[0]
    cat = [np.concatenate([r[i] for r in outs[1]], axis=1) for i in range(3)]
    assert np.array_equal(ns, cat[0]) and np.array_equal(rw, cat[1]) and np.array_equal(st, cat[2])
    tr2 = np.concatenate([r[3] for r in outs[1]])
    tr2 = tr2[np.lexsort((tr2[:, 12], tr2[:, 23]))]
    assert np.array_equal(tr, tr2, equal_nan=True)


# ------------------------------------------------------------------------------------------
# the float64 helpers of the knife-edge decisions, as compiled in both translation units
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("fast_tu", [1, 0])
def test_ieee_f64_helpers_bitwise(fast_tu):
    rng = np.random.default_rng(5)
    n = 1 << 16
    a = np.concatenate([rng.uniform(-1e4, 1e4, n).astype(np.float32).astype(np.float64),
                        rng.uniform(0, 1, n) * 10.0 ** rng.integers(-300, 300, n),
                        [0.0, -0.0, 1e-310, 5e-324, 2.0 ** -767, 1e308, 4e4, 1000.0]])
    b = np.concatenate([rng.uniform(-1e4, 1e4, n).astype(np.float32).astype(np.float64),
                        rng.uniform(0.5, 2, n) * 10.0 ** rng.integers(-300, 300, n),
                        [1.0, 3.0, 7.0, 1e-310, 3.0, 1e-308, 200.0, 1000.0]])
    with np.errstate(all="ignore"):
        want = [a / b, np.sqrt(np.abs(a)), a * a + b * b, (a + b) - a, a * b + b * a]
    lib = _lib.load()
    for op, w in enumerate(want):
        x = np.abs(a) if op == 1 else a
        ta, tb = torch.from_numpy(x).to(DEV), torch.from_numpy(b).to(DEV)
        out = torch.empty_like(ta)
        _lib.check(lib.sit_selftest_f64(op, len(x), ta.data_ptr(), tb.data_ptr(), out.data_ptr(), fast_tu, None))
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        fin = np.isfinite(w)
        bad = np.nonzero(got[fin].view(np.int64) != w[fin].view(np.int64))[0]
        assert bad.size == 0, f"op {op}: {bad.size} results differ, e.g. a={x[fin][bad[:3]]} b={b[fin][bad[:3]]}"


@pytest.mark.parametrize("fast_tu", [1, 0])
def test_device_transcendentals_vs_reference_libm(fast_tu):
    """sin, cos and atan2 as the float64 path computes them (device math library) against the
    functions the reference calls (Python's math module, LOS_guidance.py:110-113), on angles and leg
    vectors of the map's scale: at most 2 ulp apart, and the count of exact matches reported (a
    knife-edge decision that hinges on the last bit of these can differ only where they do; glibc
    2.35's atan2 is itself not correctly rounded)."""
    import math
    rng = np.random.default_rng(9)
    n = 1 << 15
    ang = np.concatenate([rng.uniform(-np.pi, np.pi, n), rng.uniform(-30, 30, n)])
    scale = 10.0 ** rng.integers(0, 4, 2 * n)        # leg vectors with 0-3 decimals, like route points
    dy = np.round(rng.uniform(-1e4, 1e4, 2 * n) * scale) / scale
    dx = np.round(rng.uniform(-1e4, 1e4, 2 * n) * scale) / scale
    lib = _lib.load()
    report = {}
    for op, (a, b, fn) in {5: (ang, ang, math.sin), 6: (ang, ang, math.cos), 7: (dy, dx, math.atan2)}.items():
        ta, tb = torch.from_numpy(a).to(DEV), torch.from_numpy(b).to(DEV)
        out = torch.empty_like(ta)
        _lib.check(lib.sit_selftest_f64(op, len(a), ta.data_ptr(), tb.data_ptr(), out.data_ptr(), fast_tu, None))
        torch.cuda.synchronize()
        got = out.cpu().numpy()
        want = np.array([fn(x, y) if op == 7 else fn(x) for x, y in zip(a, b)])
        ulps = np.abs(got.view(np.int64) - want.view(np.int64))
        report[fn.__name__] = (int((ulps == 0).sum()), len(a), int(ulps.max()))
        assert ulps.max() <= 2, f"{fn.__name__}: {int(ulps.max())} ulp"
    print("device vs reference libm (exact, total, max ulp):", report)


# measured bound of the float32 step's sine / cosine (v_sin / v_cos of t - rint(t), t = x / 2 pi;
# csrc/sit_device.h xsincos) against float64 sin / cos of the same float32 argument
F32_TRIG_ABS_BOUND = 4e-7


def test_f32_fast_trig_accuracy():
    """The float32 step's heading / IW-direction sine and cosine (xsincos in the fast-math TU:
    ship_model.py:248-250, the kinematics of both ships every step; LOS_guidance.py:110-113 and the
    IW direction) against float64 sin / cos of the same float32 argument, over both ships' heading
    ranges: |psi| <= 0.1 densely (the obstacle ship starts at psi = -0.0156), [-pi, pi] and unwrapped
    headings to +-50 rad (the reference does not wrap, Q4).  Asserts the maximum absolute error; reports
    it, the error relative to |sin psi| where |sin psi| >= 1e-3, and, near psi = 0, the error in units
    of the float32 ulp of psi.  Also the float32 atan (the LOS course) and atan2 (the leg angle) in
    ulps of their float64 value."""
    rng = np.random.default_rng(11)
    dense = np.linspace(-0.1, 0.1, 400_001)
    tiny = np.concatenate([-np.logspace(-9, -1, 4000), np.logspace(-9, -1, 4000), [0.0, -0.0156, -0.0156123]])
    sets = {"|psi|<=0.1": np.concatenate([dense, tiny]), "[-pi,pi]": rng.uniform(-np.pi, np.pi, 1 << 18),
            "+-50 rad": rng.uniform(-50, 50, 1 << 18)}
    lib = _lib.load()

    def run(op, a, b=None):
        ta = torch.from_numpy(a).to(DEV)
        tb = torch.from_numpy(a if b is None else b).to(DEV)
        out = torch.empty_like(ta)
        _lib.check(lib.sit_selftest_f64(op, len(a), ta.data_ptr(), tb.data_ptr(), out.data_ptr(), 1, None))
        torch.cuda.synchronize()
        return out.cpu().numpy()
    report = {}
    worst = 0.0
    for name, x in sets.items():
        x = x.astype(np.float32).astype(np.float64)      # the float32 argument, exactly
        s, c = run(9, x), run(10, x)
        es, ec = np.abs(s - np.sin(x)), np.abs(c - np.cos(x))
        big = np.abs(np.sin(x)) >= 1e-3
        r = {"max_abs_sin": float(es.max()), "max_abs_cos": float(ec.max()),
             "max_rel_sin_where_|sin|>=1e-3": float((es[big] / np.abs(np.sin(x[big]))).max())}
        if name == "|psi|<=0.1":
            nz = np.abs(x) > 0
            ulp = np.spacing(np.abs(x[nz]).astype(np.float32)).astype(np.float64)
            r["max_sin_err_in_ulps_of_psi"] = float((es[nz] / ulp).max())
        report[name] = r
        worst = max(worst, r["max_abs_sin"], r["max_abs_cos"])
    xs = rng.uniform(-20, 20, 1 << 16).astype(np.float32).astype(np.float64)
    ua = np.abs(run(11, xs) - np.arctan(xs)) / np.spacing(np.abs(np.arctan(xs)).astype(np.float32)).astype(np.float64)
    dy = rng.uniform(-1e4, 1e4, 1 << 16).astype(np.float32).astype(np.float64)
    dx = rng.uniform(-1e4, 1e4, 1 << 16).astype(np.float32).astype(np.float64)
    w = np.arctan2(dy, dx)
    ub = np.abs(run(12, dy, dx) - w) / np.spacing(np.abs(w).astype(np.float32)).astype(np.float64)
    report["atan_f32_max_ulp"], report["atan2_f32_max_ulp"] = float(ua.max()), float(ub.max())
    print("float32 step trig vs float64:", report)
    rec = os.environ.get("SIT_TEST_RECORD_DIR")
    if rec:
        with open(os.path.join(rec, "f32_trig_accuracy.json"), "w") as f:
            json.dump(report, f, indent=1)
    assert worst <= F32_TRIG_ABS_BOUND, f"float32 sin/cos error {worst:.3e} > {F32_TRIG_ABS_BOUND}"
    assert report["atan_f32_max_ulp"] <= 4 and report["atan2_f32_max_ulp"] <= 4


# ------------------------------------------------------------------------------------------
# the two-wave kernel (k_env_steps_sync, sit_sync.h) against the one-wave-per-ship kernel
# ------------------------------------------------------------------------------------------
def _rollouts(env, blob, kernel, launches, steps, monkeypatch):
    """Rollouts from `blob` with the step kernel selected at handle creation (SIT_STEP_KERNEL)."""
    if kernel == "classic":
        monkeypatch.setenv("SIT_STEP_KERNEL", "classic")
    else:
        monkeypatch.delenv("SIT_STEP_KERNEL", raising=False)
    env = VecMultiShipRLEnv(scenario=env.scenario, params=env.params, precision=env.precision, device=DEV)
    monkeypatch.delenv("SIT_STEP_KERNEL", raising=False)
    env.load_state_blob(blob)
    res = []
    for i in range(launches):
        # capacity for one event per env-step: nothing is dropped (which records an overflowing buffer
        # keeps depends on the order of the atomics; PTO / MEC blackouts restart episodes every few steps)
        o = env.rollout(steps, seed=41, transition_capacity=steps * env.n_env, mask_horizon=700)
        cnt = int(o["transition_count"].item())
        assert cnt <= steps * env.n_env
        tr = o["transitions"][:cnt].cpu().numpy()
        # per env in step order: one wave writes an env's records, each step's slots allocated after the
        # previous step's (a stable sort by env id keeps that order; records of repeated episode starts
        # can tie on every value column)
        res.append({k: o[k].cpu().numpy() for k in ("next_state", "reward", "done", "status", "action", "done_count")}
                   | {"transitions": tr[np.argsort(tr[:, 23], kind="stable")]})
    name = env.lib.sit_step_kernel(env.handle).decode()
    assert name.startswith("k_env_steps_sync<" if kernel == "sync" else "k_env_steps<"), name
    st = np_state(env)
    torch.cuda.synchronize()
    return res, st


# configurations the sync kernel serves by default besides the reference's PTI / MOTOR shaft model:
# the simplified machinery, the collision bias off, and the blackout paths of the PTO (GEN) and MEC
# (OFF) machinery modes (mode rows of the reference fixtures env_blackout_pto / env_mec_nominal)
SYNC_CONFIGS = {
    "default": lambda: gpu_params(),
    "simplified": lambda: gpu_params(machinery_model=so.MACH_SIMPLIFIED, thrust_force_dynamic_time_constant=30.0),
    "no_bias": lambda: gpu_params(collision_bias=0),
    "pto": lambda: gpu_params(golden("env_blackout_pto")["mode"]),
    "mec": lambda: gpu_params(golden("env_mec_nominal")["mode"]),
}


@pytest.mark.parametrize("config", list(SYNC_CONFIGS))
@pytest.mark.parametrize("precision", [64, 32])
def test_sync_kernel_equals_classic(precision, config, monkeypatch):
    """k_env_steps_sync (the default kernel of every synthetic-sampler and policy rollout with
    auto-reset) against k_env_steps from the same state (after a 600-step warm-up, so episodes are
    desynchronised) on 2000 envs (a partial last block), in each configuration it serves.
    float64: 3 launches x 700 steps with the rarely-hit paths in them (terrain / IW terminations,
    route insertions, stop paths): every output and the final state identical to 1e-9 relative
    (observed: bit for bit), done / status / done counts / transition counts exactly.  float32: the
    two kernels are separately scheduled fast-math code whose float32 roundings may differ, so
    free-running trajectories can drift apart; over 4 launches x 50 steps the discrete outputs are
    identical and the reals within 1e-5 relative against the contract's per-field floors."""
    n_env = 2000
    launches, steps = (3, 700) if precision == 64 else (4, 50)
    env = VecMultiShipRLEnv(scenario=make_scenario(n_env, cap=48), params=SYNC_CONFIGS[config](),
                            precision=precision, device=DEV)
    env.reset()
    env.init_step()
    env.rollout(600, seed=40)
    blob = env.state_blob()
    a, sa = _rollouts(env, blob, "classic", launches, steps, monkeypatch)
    b, sb = _rollouts(env, blob, "sync", launches, steps, monkeypatch)
    tol = TOL64 if precision == 64 else 1e-5
    floors = {"next_state": OBS_SCALE, "reward": 1.0, "action": np.array([1e4, 1e4, np.pi, 1.0]),
              "transitions": np.r_[OBS_SCALE, 1.0, 1.0, OBS_SCALE, 1.0, 1.0]}
    n_terr, worst = 0, {}
    bitwise = True
    for i, (x, y) in enumerate(zip(a, b)):
        for k in ("done", "status", "done_count"):
            assert np.array_equal(x[k], y[k]), f"launch {i}: {k} differs"
        assert x["transitions"].shape == y["transitions"].shape, f"launch {i}: transition count"
        for k in ("next_state", "reward", "action", "transitions"):
            bitwise &= np.array_equal(x[k], y[k], equal_nan=True)
            assert np.array_equal(np.isnan(x[k]), np.isnan(y[k])), f"launch {i}: {k} NaN pattern"
            err = np.nan_to_num(rel_err(x[k], y[k], floors[k])) if x[k].size else np.zeros(1)
            worst[k] = max(worst.get(k, 0.0), float(err.max()))
            assert err.max() <= tol, f"launch {i}: {k} rel err {err.max():.3e}"
        n_terr += int(((x["status"] & (_lib.ST_TEST_TERRAIN | _lib.ST_OBS_TERRAIN |
                                       _lib.ST_OBS_IW_TERMINAL)) != 0).sum())
    for k in so.SHIP_INT:
        assert np.array_equal(sa[k], sb[k]), f"final state {k}"
    for k in so.SHIP_REAL:
        err = rel_err(sb[k], sa[k], SCALE[k]).max()
        worst[k] = float(err)
        assert err <= tol, f"final state {k} rel err {err:.3e}"
    print(f"sync vs classic f{precision} {config}: {n_terr} terrain/IW terminations, bitwise {bitwise}, "
          f"worst {dict((k, f'{v:.1e}') for k, v in worst.items())}")
    assert n_terr > 0 or precision == 32, "the case exercises no terrain / IW termination"


def test_c4_last_shard_full_size():
    """The last of config C4's eight shards at its full per-GPU size, as bench.py --gpus 8 runs it on
    rank 7: envs [7 x 32 768, 8 x 32 768) (scenario and sampler keyed by global env id), one
    40 000-step float32 launch with the replay transitions at the bench's capacity.  No record is
    dropped, the done counts equal the done rows, the outputs are finite, and the shard's first 64
    envs step exactly as a 64-env handle of the same global ids."""
    n, off, K = 32768, 7 * 32768, 40000
    env = VecMultiShipRLEnv(scenario=make_scenario(n, cap=48, env_offset=off), precision=32, device=DEV)
    env.reset()
    env.init_step()
    cap = max(n, n * K // 192)                        # bench.py bench_rollout's capacity
    out = env.rollout(K, seed=25450, env_id_offset=off, transition_capacity=cap)
    torch.cuda.synchronize()
    cnt = int(out["transition_count"].item())
    assert 0 < cnt <= cap, f"{cnt} transitions for capacity {cap}"
    assert torch.equal(out["done_count"].to(torch.int64), out["done"].to(torch.int64).sum(1))
    assert int(out["done_count"].sum().item()) > n     # every env ended at least one episode
    assert bool(torch.isfinite(out["reward"]).all())
    for k0 in range(0, K, 10000):                     # (in slices: the full array is 52 GB)
        assert bool(torch.isfinite(out["next_state"][k0:k0 + 10000]).all())
    tr = out["transitions"][:cnt]
    ids = tr[:, 23].to(torch.int64)
    assert int(ids.min()) >= off and int(ids.max()) < off + n
    head = {k: out[k][:200, :64].cpu().numpy() for k in ("next_state", "reward", "status")}
    del out
    small = VecMultiShipRLEnv(scenario=make_scenario(64, cap=48, env_offset=off), precision=32, device=DEV)
    small.reset()
    small.init_step()
    o = small.rollout(200, seed=25450, env_id_offset=off)
    for k in head:
        assert np.array_equal(o[k].cpu().numpy(), head[k]), k


@pytest.mark.parametrize("kernel", ["sync", "classic"])
@pytest.mark.parametrize("precision", [64, 32])
def test_launch_partition_invariance(precision, kernel, monkeypatch):
    """One 300-step launch equals 300 one-step launches bit for bit (synthetic sampler, auto-reset):
    everything a launch keeps in registers across steps (the route leg cache, the sampler's next draw,
    the next heading's sine and cosine) is rebuilt from the state at the next launch with the same
    values, and the one-step launches' IW-test cache (iw_key_*, keyed by the IW point) returns what the
    test would.  The one-step launches read the map through the caches instead of LDS."""
    if kernel == "classic":
        monkeypatch.setenv("SIT_STEP_KERNEL", "classic")
    n_env, steps = 512, 300
    outs = []
    for k in (steps, 1):
        env = VecMultiShipRLEnv(scenario=make_scenario(n_env, cap=48), precision=precision, device=DEV)
        env.reset()
        env.init_step()
        rows = {q: [] for q in ("next_state", "reward", "done", "status", "action")}
        for _ in range(steps // k):
            o = env.rollout(k, seed=13, transition_capacity=0)
            for q in rows:
                rows[q].append(o[q].cpu().numpy())
        outs.append(({q: np.concatenate(v) for q, v in rows.items()}, np_state(env), env))
    (a, sa, ea), (b, sb, eb) = outs
    assert ea.lib.sit_step_kernel(ea.handle).decode().startswith("k_env_steps_sync" if kernel == "sync" else "k_env_steps<")
    for q in a:
        assert np.array_equal(a[q], b[q], equal_nan=True), q
    for q in sa:
        if not q.startswith("iw_key"):   # the single-step launches' IW-test cache (not model state)
            assert np.array_equal(sa[q], sb[q]), q
    iw = int(((a["status"] & _lib.ST_OBS_IW_TERMINAL) != 0).sum())
    print(f"launch partition f{precision} {kernel}: {iw} IW terminations, identical")


def test_state_restore_across_maps_retests_iw():
    """A state blob saved on one map and restored on a handle with another map: the restored handle
    re-tests the IW against its own map (sit_set_state clears the single-step IW-test cache,
    iw_key_*) instead of reusing the other map's answer.  The IW lies in open water on the reference
    map and inside an extra island on the second map."""
    n_env = 64
    sc = make_scenario(n_env, cap=32)
    obs_n, obs_e = sc.init[:, 1, 0], sc.init[:, 1, 1]
    iw = np.stack([obs_n + 400.0, obs_e], 1)           # 400 m north of the obstacle's start: open water
    c_n, c_e = float(iw[:, 0].mean()), float(iw[:, 1].mean())
    half = 150.0 + float(np.ptp(iw[:, 0]) + np.ptp(iw[:, 1]))
    island = np.array([[c_e - half, c_n - half], [c_e + half, c_n - half], [c_e + half, c_n + half],
                       [c_e - half, c_n + half]])        # (east, north) vertices around every IW
    sc_b = Scenario(sc.routes, sc.n_wpt, sc.init, list(sc.polys) + [island])
    outs = []
    for scen in (sc, sc_b):
        e = VecMultiShipRLEnv(scenario=scen, precision=64, device=DEV)
        e.reset()
        e.init_step()
        outs.append(e)
    a, b = outs
    ones, zeros = np.ones(n_env, np.uint8), np.zeros(n_env, np.uint8)
    _, _, _, st0 = a.step(iw, ones, ones)
    _, _, _, st1 = a.step(iw, zeros, zeros)
    assert not ((st0 | st1) & _lib.ST_OBS_IW_TERMINAL).any(), "the IW should be in open water on map A"
    assert (np_state(a)["iw_key_flags"] & 1).all(), "map A's IW test was not cached"
    b.load_state_blob(a.state_blob())
    _, _, _, st2 = b.step(iw, zeros, zeros)
    assert ((st2 & _lib.ST_OBS_IW_TERMINAL) != 0).all(), "the restored handle reused map A's IW test"


@pytest.mark.parametrize("steps", [1, 16])
@pytest.mark.parametrize("precision", [64, 32])
def test_sync_kernel_equals_classic_explicit_no_reset(precision, steps, monkeypatch):
    """Explicit actions without auto-reset (the drop-in's sit_step / rollout(actions=...)): the two-wave
    kernel against k_env_steps from the same desynchronised state, over 2000 envs and 96 steps in
    launches of `steps` (1: the map read through the caches with the IW-test cache; 16: the LDS map).
    IWs near the obstacle ship, inserted at random steps (1 %), many into terrain.  Final stop flags,
    next waypoint and route length identical; outputs within 1e-9 (f64) / 1e-5 (f32) against the
    per-field floors, done and status identical."""
    n_env, total = 2000, 96
    base = VecMultiShipRLEnv(scenario=make_scenario(n_env, cap=48), precision=precision, device=DEV)
    base.reset()
    base.init_step()
    base.rollout(600, seed=40)
    blob = base.state_blob()
    st = np_state(base)
    rng = np.random.default_rng(5)
    ang = rng.uniform(-np.pi, np.pi, (total, n_env))
    dist = rng.uniform(200.0, 1500.0, (total, n_env))
    act = np.stack([st["north"][1] + dist * np.cos(ang), st["east"][1] + dist * np.sin(ang)], -1)
    sac = (rng.random((total, n_env)) < 0.01).astype(np.uint8)
    init = np.zeros((total, n_env), np.uint8)
    res = {}
    for kernel in ("classic", "sync"):
        if kernel == "classic":
            monkeypatch.setenv("SIT_STEP_KERNEL", "classic")
        env = VecMultiShipRLEnv(scenario=base.scenario, precision=precision, device=DEV)
        monkeypatch.delenv("SIT_STEP_KERNEL", raising=False)
        env.load_state_blob(blob)
        rows = {q: [] for q in ("next_state", "reward", "done", "status")}
        for k0 in range(0, total, steps):
            sl = slice(k0, k0 + steps)
            o = env.rollout(steps, auto_reset=False, actions={"action_ne": act[sl], "sac_update": sac[sl],
                                                              "init": init[sl]}, transition_capacity=0)
            for q in rows:
                rows[q].append(o[q].cpu().numpy())
        name = env.lib.sit_step_kernel(env.handle).decode()
        assert name.startswith("k_env_steps_sync<" if kernel == "sync" else "k_env_steps<"), name
        assert ("map=global" in name) == (steps == 1), name
        res[kernel] = ({q: np.concatenate(v) for q, v in rows.items()}, np_state(env))
    (x, sx), (y, sy) = res["classic"], res["sync"]
    tol = TOL64 if precision == 64 else 1e-5
    for q in ("done", "status"):
        assert np.array_equal(x[q], y[q]), q
    assert rel_err(y["next_state"], x["next_state"], OBS_SCALE).max() <= tol
    assert np.abs(y["reward"] - x["reward"]).max() <= tol * max(1.0, float(np.abs(x["reward"]).max()))
    for q in ("stop", "next_wpt", "n_wpt"):
        assert np.array_equal(sx[q], sy[q]), q
    n_iw = int(((x["status"] & _lib.ST_OBS_IW_TERMINAL) != 0).sum())
    n_stop = int(sx["stop"].sum())
    print(f"explicit no-reset f{precision} K={steps}: {n_iw} IW-terminal rows, {n_stop} stopped ships")
    assert n_iw > 0 and n_stop > 0
