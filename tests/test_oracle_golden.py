"""Pin the CPU oracle (oracle/sit_oracle.py) against the reference's own outputs.

Fixtures come from tests/golden/make_golden.py, which runs the reference simulator
(simulators/ship_in_transit/*) unmodified and the reference env (RLEnv/MSRL_env_ex.py) under
API shims.  Float tolerance: 1e-11 relative with the per-field scale floors of SURVEY §8(d)
(observed: <= 1e-13; differences are libm-vs-numpy transcendental ulps).  Discrete outputs
(waypoint index, stop flags, done, status strings) must be identical.
"""
import numpy as np
import pytest

from helpers import (OBS_SCALE, SCALE, SIM_FIELDS, env_oracle, env_state_all_rows, env_state_from,
                     golden, golden_names, rel_err, sim_oracle, sim_oracle_batch, sim_scale, sim_state_all_rows,
                     sim_state_from)
from oracle import sit_oracle as so

TOL = 1e-11


def _check_fields(got, want, names, tol, where, scale=SCALE):
    for k in names:
        err = rel_err(got[k], want[k], scale.get(k, 1.0)).max()
        assert err <= tol, f"{where}: field {k} rel err {err:.3e}"


@pytest.mark.parametrize("name", ["sim_c1", "sim_k2", "sim_bias", "sim_pto", "sim_mec", "sim_simpl", "sim_simpl_pto"])
def test_sim_trajectory_free_running(name):
    """Whole trajectories of one ship (C1 = sim_c1: 1000 zero-action steps), no teacher forcing.
    sim_simpl*: the SimplifiedMachineryModel (ship_engine.py:398-433) with its throttle
    controller (controllers.py:154-172), composed as make_golden.py documents."""
    d = golden(name)
    o = sim_oracle(d)
    bias = bool(d["bias"])
    scale = sim_scale(d)
    for i in range(len(d["out_rudder"])):
        _check_fields({k: o.s[k][1] for k in SIM_FIELDS}, {k: d["pre_" + k][i] for k in SIM_FIELDS},
                      SIM_FIELDS, TOL, f"{name} step {i}", scale)
        out = o.sim_step(1, bias)
        for k, v in out.items():
            if "out_" + k in d.files:
                err = rel_err(v[0], d["out_" + k][i], scale[k])
                assert err <= TOL, f"{name} step {i}: {k} rel err {err:.3e}"


def test_known_answers_k1_k2():
    """SURVEY §8(a) K1/K2 known-answer values (reference outputs, float64)."""
    d = golden("sim_c1")
    o = sim_oracle(d)
    out = o.sim_step(1)
    assert out["throttle"][0] == pytest.approx(3.72275625, rel=1e-12)
    assert out["d_surge"][0] == pytest.approx(0.02134085128069556, rel=1e-12)
    assert out["d_sway"][0] == pytest.approx(1.4395501405809803e-4, rel=1e-12)
    assert out["d_shaft_speed"][0] == pytest.approx(1.1228801563249238, rel=1e-12)
    assert out["thrust"][0] == pytest.approx(275469.11598875304, rel=1e-12)
    k2 = golden("sim_k2")
    o = sim_oracle(k2)
    o.set_state(sim_state_from(k2, "pre_", 500, o))
    assert k2["pre_north"][500] == pytest.approx(621.8290931380596, rel=1e-12)
    assert int(k2["pre_next_wpt"][500]) == 1
    out = o.sim_step(1)
    assert out["rudder"][0] == pytest.approx(-0.026737999545429776, rel=1e-11)
    assert out["throttle"][0] == pytest.approx(192.3899565258797, rel=1e-11)
    assert out["heading_ref"][0] == pytest.approx(0.6737103277202099, rel=1e-12)
    assert out["e_ct"][0] == pytest.approx(104.67549291706916, rel=1e-12)
    assert out["d_surge"][0] == pytest.approx(0.004254350556551482, rel=1e-10)


def test_sim_teacher_forced_one_step():
    """600 one-step cases incl. knife edges: acceptance circle +-1e-9 m, |e_ct| = lookahead,
    anti-windup limit, negative throttle, unwrapped heading, reversed shaft.  Cases run as one
    batch of envs; odd cases carry the collision bias (run separately)."""
    d = golden("sim_teacher_forced")
    n = len(d["bias"])
    for b in (False, True):
        o = sim_oracle_batch(d, n)
        o.set_state(sim_state_all_rows(d, "pre_", o))
        out = o.sim_step(1, b)
        sel = d["bias"].astype(bool) == b
        st = o.get_state()
        assert np.array_equal(st["next_wpt"][1][sel], d["post_next_wpt"][sel]), "waypoint index"
        _check_fields({k: st[k][1][sel] for k in SIM_FIELDS}, {k: d["post_" + k][sel] for k in SIM_FIELDS},
                      SIM_FIELDS, TOL, f"bias={b}")
        for k, v in out.items():
            if "out_" + k in d.files:
                assert rel_err(v[sel], d["out_" + k][sel], SCALE[k]).max() <= TOL, k


ENV_CASES = golden_names("env_")


@pytest.mark.parametrize("name", ENV_CASES)
def test_env_teacher_forced(name):
    """MultiShipRLEnv.step from every recorded pre-state (one batch: env j = step j): next_state,
    reward, done, status string and the full post-state (ships, controllers, stop flags,
    distances, routes)."""
    d = golden(name)
    T = len(d["reward"])
    o = env_oracle(d, n_env=T)
    o.set_state(env_state_all_rows(d, "pre_", o))
    act = np.stack([d["action_n"], d["action_e"]], axis=1)
    ns, rew, done, st = o.step(act, d["sac_update"], d["init"])
    assert rel_err(ns, d["next_state"], OBS_SCALE).max() <= TOL
    assert rel_err(rew, d["reward"], 1.0).max() <= TOL
    assert np.array_equal(done, d["done"].astype(bool))
    for i in range(T):
        assert so.status_string(int(st[i])) == str(d["status"][i]), f"{name} step {i}"
    post = o.get_state()
    for k in so.SHIP_INT:
        assert np.array_equal(post[k], d["post_" + k].T), k
    for k in so.SHIP_REAL:
        assert rel_err(post[k], d["post_" + k].T, SCALE[k]).max() <= TOL, k
    for k in ("sampling_dist", "eps_dist", "prev_pre_north", "prev_pre_east"):
        assert rel_err(post[k], d["post_" + k], SCALE[k]).max() <= TOL, k
    for i in range(T):
        nw = int(d["post_n_wpt"][i][1]) - 1
        assert np.array_equal(post["wpt_north"][1, :nw, i], d["post_wpt_north"][i][1, :nw]), i


@pytest.mark.parametrize("name", ENV_CASES)
def test_env_free_running(name):
    """Whole episodes from the first recorded state, resets included (Q6 persistence)."""
    d = golden(name)
    o = env_oracle(d)
    assert np.array_equal(o.reset()[0], d["reset_state"])          # Q15: float32 construction state
    o.set_state(env_state_from(d, "pre_", 0, o))
    resets = set(d["resets"].tolist())
    for i in range(len(d["reward"])):
        if i in resets and i > 0:
            o.reset()
            o.init_step()
        st = o.s
        for k in ("north", "east", "yaw", "shaft_speed", "shaft_speed_i", "heading_i"):
            assert rel_err(st[k][:, 0], d["pre_" + k][i], SCALE[k]).max() <= 1e-10, f"{name} {i} {k}"
        assert np.array_equal(st["next_wpt"][:, 0], d["pre_next_wpt"][i])
        ns, rew, done, stt = o.step([[d["action_n"][i], d["action_e"][i]]], [d["sac_update"][i]],
                                    [d["init"][i]])
        assert rel_err(rew[0], d["reward"][i], 1.0) <= 1e-10, f"{name} {i}"
        assert so.status_string(int(stt[0])) == str(d["status"][i]), f"{name} {i}"


def test_nominal_episode_matches_survey_k4():
    """the seeded random-IW episode ends at step 1694, IW in terminal state."""
    d = golden("env_nominal")
    assert len(d["reward"]) == 1694
    assert "Obstacle ship IW sampled in terminal state" in str(d["status"][-1])
    assert d["reward"][-1] == pytest.approx(-999.893291, abs=1e-6)


# ------------------------------------------------------------------------------------------
# trajectory logs: simulation_results (ship_model.py:645-700, fuel model ship_engine.py:256-292)
# and reward_results (MSRL_env_ex.py:926-964), recorded from the reference by make_golden.py
# ------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", [n for n in golden_names("sim_") if n != "sim_teacher_forced"
                                  and not n.startswith("sim_simpl")])   # no reference log for that model
def test_oracle_simulation_log_vs_reference(name):
    d = golden(name)
    o = sim_oracle(d)
    rows = [o.sim_step(1, bias=bool(d["bias"]))["log"][:, 0] for _ in range(len(d["log"]))]
    err = np.abs(np.array(rows) - d["log"]) / np.maximum(np.abs(d["log"]), 1.0)
    assert err.max() <= 1e-10, f"{name}: log rel err {err.max():.3e}"


@pytest.mark.parametrize("name", golden_names("env_"))
def test_oracle_env_logs_vs_reference(name):
    """Teacher-forced env steps: both ships' simulation_results rows (incl. the obstacle's
    store_last_simulation_data on the stop path) and the per-episode reward_results sums."""
    d = golden(name)
    o = env_oracle(d)
    o.reset()
    o.init_step()
    o.start_log()
    n = min(len(d["reward"]), 300)          # long horizons are covered by the simulator logs
    for i in range(n):
        o.set_state(env_state_from(d, "pre_", i, o))
        o.step(np.array([[d["action_n"][i], d["action_e"][i]]]), [d["sac_update"][i] > 0.5], [d["init"][i] > 0.5])
    logs = np.array(o.log["ship"])[:, :, :, 0]
    for t, key in ((0, "log_test"), (1, "log_obs")):
        err = np.abs(logs[:, t] - d[key][:n]) / np.maximum(np.abs(d[key][:n]), 1.0)
        assert err.max() <= 1e-10, f"{name} {key}: rel err {err.max():.3e}"
    terms = np.array(o.log["reward"])[:, :, 0]
    resets = set(d["resets"].tolist())
    acc, cum = np.zeros(len(so.REWARD_TERMS)), []
    for i in range(n):
        if i in resets:
            acc = np.zeros(len(so.REWARD_TERMS))
        acc = acc + terms[i]
        cum.append(acc.copy())
    err = np.abs(np.array(cum) - d["log_reward"][:n]) / np.maximum(np.abs(d["log_reward"][:n]), 1.0)
    assert err.max() <= 1e-12, f"{name} reward_results: rel err {err.max():.3e}"
