"""GPU parity of the policy-driven sampler (config 5 path) against the oracle's synchronous loop.

The HIP kernel's policy mode lets an env wait (rows with status ST_NO_STEP) until the actor has
produced the action of its sampling event; the oracle (OracleEnvs.policy_rollout) runs the
reference's per-step loop (test_beds/main_ast.py:310-412, agent.select_action mode 1) with the
same policy and the same Philox noise.  Per env, the k-th executed GPU step must equal the
oracle's k-th step: float64 within 1e-9 (per-field floors), discrete outputs identical.
"""
import copy

import numpy as np
import pytest
import torch

from helpers import OBS_SCALE
from oracle import sit_oracle as so

pytestmark = pytest.mark.gpu

sit = pytest.importorskip("sac_maritime_ast_amd")
from sac_maritime_ast_amd import VecMultiShipRLEnv, _lib, make_scenario  # noqa: E402
from sac_maritime_ast_amd.samplers import (GaussianPolicy, OverlappedPolicySampler,  # noqa: E402
                                           PolicySampler)

DEV = "cuda:0"
SEED = 4242


def make_policy(dtype, device):
    torch.manual_seed(3)
    pol = GaussianPolicy(hidden=(64, 64))
    with torch.no_grad():   # make the actor's actions span [-1, 1] on this state scale
        pol.net[0].weight.mul_(1e-3)
    return pol.to(dtype=dtype, device=device)


def oracle_policy_fn(pol_cpu):
    def fn(state, noise):
        with torch.no_grad():
            a, _, _, _ = pol_cpu(torch.from_numpy(state), torch.from_numpy(np.asarray(noise)))
        return a[:, 0].numpy()
    return fn


def run_gpu(sampler_list, n_launch):
    """Per env, the executed rows in order: dict of lists of numpy arrays."""
    rows = []
    for _ in range(n_launch):
        outs = sampler_list.launch() if hasattr(sampler_list, "samplers") else [sampler_list.launch()]
        torch.cuda.synchronize()
        rows.append([{k: v.cpu().numpy().copy() for k, v in o.items() if k != "done_count"} for o in outs])
    return rows


def per_env(rows, group, n_env):
    seq = {k: [[] for _ in range(n_env)] for k in ("next_state", "reward", "done", "status", "action")}
    for launch in rows:
        o = launch[group]
        st = o["status"].astype(np.int64) & 0xFFFFFFFF
        for k in range(st.shape[0]):
            for e in np.nonzero((st[k] & _lib.ST_NO_STEP) == 0)[0]:
                seq["next_state"][e].append(o["next_state"][k, e])
                seq["reward"][e].append(o["reward"][k, e])
                seq["done"][e].append(bool(o["done"][k, e]))
                seq["status"][e].append(int(st[k, e]))
                seq["action"][e].append(o["action"][k, e])
    return seq


def compare(seq, ref, n_env, n_steps):
    for e in range(n_env):
        assert len(seq["reward"][e]) >= n_steps, f"env {e}: only {len(seq['reward'][e])} steps executed"
        ns = np.array(seq["next_state"][e][:n_steps])
        err = np.abs(ns - ref["next_state"][:, e]) / np.maximum(np.abs(ref["next_state"][:, e]), OBS_SCALE)
        assert err.max() <= 1e-9, f"env {e}: next_state rel err {err.max():.3e}"
        rw = np.array(seq["reward"][e][:n_steps])
        assert np.abs(rw - ref["reward"][:, e]).max() <= 1e-9 * max(1.0, np.abs(ref["reward"][:, e]).max())
        assert np.array_equal(np.array(seq["done"][e][:n_steps]), ref["done"][:, e]), f"env {e}: done"
        got_st, ref_st = np.array(seq["status"][e][:n_steps]), ref["status"][:, e].astype(np.int64)
        bad = np.nonzero(got_st != ref_st)[0]
        assert bad.size == 0, f"env {e}: status at step {bad[:3]}: {got_st[bad[:3]]} vs {ref_st[bad[:3]]}"
        act = np.array(seq["action"][e][:n_steps])
        sac = ref["action"][:, e, 3] > 0.5
        assert np.array_equal(act[:, 3] > 0.5, sac), f"env {e}: sampling events"
        assert np.allclose(act[sac, :3], ref["action"][sac, e, :3], rtol=1e-10, atol=1e-9), f"env {e}: IW"


def oracle_run(sc, pol, n_steps, env_id_offset=0):
    o = so.OracleEnvs(dict(so.DEFAULT_PARAMS), sc.routes, sc.n_wpt, sc.init, sc.polys)
    o.reset()
    o.init_step()
    return o.policy_rollout(n_steps, SEED, oracle_policy_fn(pol), env_id_offset=env_id_offset)


@pytest.mark.parametrize("capacity", [None, 8])
def test_f64_policy_mode_matches_synchronous_loop(capacity):
    n_env, chunk, n_launch = 64, 16, 40
    sc = make_scenario(n_env, cap=32, seed=11)
    env = VecMultiShipRLEnv(scenario=sc, precision=64, device=DEV)
    env.reset()
    env.init_step()
    pol = make_policy(torch.float64, DEV)
    sm = PolicySampler(env, pol, chunk=chunk, seed=SEED, request_capacity=capacity, transition_capacity=2 * n_env)
    rows = run_gpu(sm, n_launch)
    seq = per_env(rows, 0, n_env)
    done_steps = min(len(r) for r in seq["reward"])
    executed = int(sm.env_steps.item())
    assert executed == sum(len(r) for r in seq["reward"])
    assert done_steps >= 200, done_steps
    ref = oracle_run(sc, make_policy(torch.float64, "cpu"), done_steps)
    compare(seq, ref, n_env, done_steps)
    # the actor saw sampling events of every env (init events at least)
    assert int(sm.served.item()) >= n_env
    # replay transitions of the policy's events: per env in event order (an env takes at most one
    # sampling event per launch: it waits for the actor at the next one), the action column holding
    # the policy's squashed action in [-1, 1] as in synthetic mode (memory.push, main_ast.py:395)
    gpu = [[] for _ in range(n_env)]
    for launch in rows:
        o = launch[0]
        tr = o["transitions"][:int(o["transition_count"][0])]
        for rec in tr:
            gpu[int(rec[23])].append(rec)
    want = ref["transitions"]
    assert len(want) >= n_env
    for e in range(n_env):
        w = want[want[:, 23] == e]
        g = np.array(gpu[e][:len(w)])
        assert len(g) == len(w), f"env {e}: {len(g)} transitions vs {len(w)}"
        assert np.array_equal(g[:, 22], w[:, 22]), f"env {e}: masks"
        assert np.abs(g[:, 10]).max() <= 1.0
        scale = np.r_[OBS_SCALE, 1.0, 1.0, OBS_SCALE]
        err = np.abs(g[:, :22] - w[:, :22]) / np.maximum(np.abs(w[:, :22]), scale)
        assert err.max() <= 1e-9, f"env {e}: transition rel err {err.max():.3e}"


def test_f64_overlapped_groups_match():
    n_env, chunk, n_launch = 32, 16, 30
    sc_all = make_scenario(2 * n_env, cap=32, seed=12)
    groups = []
    for g in range(2):
        sl = slice(g * n_env, (g + 1) * n_env)
        from sac_maritime_ast_amd.scenario import Scenario
        sc = Scenario(sc_all.routes[sl], sc_all.n_wpt[sl], sc_all.init[sl], sc_all.polys)
        env = VecMultiShipRLEnv(scenario=sc, precision=64, device=DEV)
        env.reset()
        env.init_step()
        groups.append((sc, PolicySampler(env, make_policy(torch.float64, DEV), chunk=chunk, seed=SEED,
                                         env_id_offset=g * n_env)))
    ov = OverlappedPolicySampler([s for _, s in groups])
    rows = run_gpu(ov, n_launch)
    ref = None
    for g, (sc, _) in enumerate(groups):
        seq = per_env(rows, g, n_env)
        n = min(len(r) for r in seq["reward"])
        assert n >= 150, n
        ref = oracle_run(sc, make_policy(torch.float64, "cpu"), n, env_id_offset=g * n_env)
        compare(seq, ref, n_env, n)


def test_f32_policy_mode_sanity():
    n_env = 4096
    env = VecMultiShipRLEnv(scenario=make_scenario(n_env, cap=48), precision=32, device=DEV)
    env.reset()
    env.init_step()
    sm = PolicySampler(env, make_policy(torch.float32, DEV), chunk=32, seed=SEED, request_capacity=1024)
    stepped = 0
    for _ in range(20):
        out = sm.launch()
        st = out["status"].to(torch.int64) & 0xFFFFFFFF
        live = (st & _lib.ST_NO_STEP) == 0
        stepped += int(live.sum().item())
        assert torch.isfinite(out["next_state"][live]).all()
        assert torch.isfinite(out["reward"][live]).all()
    assert stepped == int(sm.env_steps.item())
    assert stepped > 0.8 * 20 * 32 * n_env


def make_policy256(device):
    torch.manual_seed(5)
    pol = GaussianPolicy(hidden=(256, 256))
    with torch.no_grad():
        pol.net[0].weight.mul_(1e-3)
    return pol.to(dtype=torch.float32, device=device)


@pytest.mark.parametrize("precision,deterministic", [(32, False), (32, True), (64, False)])
def test_fused_actor_matches_torch_float64(precision, deterministic):
    """sit_policy_actor (the whole 10-256-256-2 actor + squashed head + scatter in one kernel)
    against the same policy evaluated in float64 PyTorch on the queued rows: |action| error
    <= 1e-5 (float32 actor); the other request-counter slot is cleared and `served` advanced by the
    kernel."""
    n_env = 2048
    env = VecMultiShipRLEnv(scenario=make_scenario(n_env, cap=48, seed=7), precision=precision, device=DEV)
    env.reset()
    env.init_step()
    pol = make_policy256(DEV)
    ref_pol = copy.deepcopy(pol).double()
    sm = PolicySampler(env, pol, chunk=32, seed=SEED, request_capacity=1024, deterministic=deterministic)
    assert sm.fused
    io = sm.io
    checked = 0
    for it in range(6):
        io["request_count"].zero_()
        sm._counts[1].fill_(7)              # the other slot: cleared by the actor
        env.rollout(sm.chunk, seed=sm.seed, env_id_offset=0, out=sm.out, policy_io=io)
        torch.cuda.synchronize()
        count = min(int(io["request_count"].item()), io["request_env"].numel())
        obs = io["request_obs"][:count].double().clone()
        noise = io["request_noise"][:count].double().clone()
        envs = io["request_env"][:count].long().clone()
        served0 = int(sm.served.item())
        io["policy_ready"].zero_()
        sm.act()
        torch.cuda.synchronize()
        assert int(sm._counts[1].item()) == 0
        assert int(sm.served.item()) == served0 + count
        with torch.no_grad():
            ref = ref_pol(obs, noise, deterministic=deterministic)[0][:, 0]
        got = io["policy_action"][envs].double()
        assert torch.all(io["policy_ready"][envs] == 1)
        if count:
            err = (got - ref).abs().max().item()
            assert err <= 1e-5, f"launch {it}: fused actor max |err| {err:.3e} over {count} rows"
            assert ref.abs().max().item() > (1e-3 if deterministic else 0.05)   # not all ~0
        checked += count
    assert checked >= n_env


def test_fused_actor_policy_mode_sanity():
    """C5 configuration on a small population: fused actor, graph capture, overlapped groups."""
    n_env = 4096
    samplers = []
    for g in range(2):
        env = VecMultiShipRLEnv(scenario=make_scenario(n_env, cap=48, seed=9, env_offset=g * n_env), precision=32,
                                device=DEV)
        env.reset()
        env.init_step()
        samplers.append(PolicySampler(env, make_policy256(DEV), chunk=32, seed=SEED, env_id_offset=g * n_env,
                                      request_capacity=n_env // 4))
    assert all(s.fused for s in samplers)
    ov = OverlappedPolicySampler(samplers).capture(4)
    before = [int(s.env_steps.item()) for s in samplers]
    for _ in range(5):
        outs = ov.replay()
    torch.cuda.synchronize()
    for s, b, out in zip(samplers, before, outs):
        stepped = int(s.env_steps.item()) - b
        assert stepped > 0.8 * 5 * 4 * 32 * n_env
        st = out["status"].to(torch.int64) & 0xFFFFFFFF
        live = (st & _lib.ST_NO_STEP) == 0
        assert torch.isfinite(out["next_state"][live]).all()
        assert int(s.served.item()) > n_env
