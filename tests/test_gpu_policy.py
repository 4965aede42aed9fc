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
    clear = torch.full((1,), 7, dtype=torch.int32, device=DEV)
    for it in range(6):
        env.rollout(sm.chunk, seed=sm.seed, env_id_offset=0, out=sm.out, policy_io=io)
        torch.cuda.synchronize()
        count = min(int(io["request_count"].item()), io["request_env"].numel())
        obs = io["request_obs"][:count].double().clone()
        noise = io["request_noise"][:count].double().clone()
        envs = io["request_env"][:count].long().clone()
        served0 = int(sm.served.item())
        io["policy_ready"].zero_()
        if it == 0:     # the ABI's optional clear_count store
            with torch.cuda.device(env.device):
                env._call("sit_policy_actor", int(sm._rows.numel()), sm._w.data_ptr(), io["request_obs"].data_ptr(),
                          io["request_noise"].data_ptr(), io["request_env"].data_ptr(),
                          io["request_count"].data_ptr(), int(bool(deterministic)), io["policy_action"].data_ptr(),
                          io["policy_ready"].data_ptr(), sm.served.data_ptr(), clear.data_ptr(), env._stream())
        else:
            sm.act()
        torch.cuda.synchronize()
        assert int(clear.item()) == 0
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


# ------------------------------------------------------------------------------------------
# float32 policy mode: the instantiation config C5 times (k_env_steps_sync<float, kPolicy>)
# ------------------------------------------------------------------------------------------
def _f32_rounded(st):
    return {k: (v.astype(np.float32).astype(np.float64) if v.dtype == np.float64 else v) for k, v in st.items()}


def _np_state(env):
    return {k: v.cpu().numpy() for k, v in env.get_state().items()}


def _policy_io(n_env, cap, dtype):
    io = {"policy_action": torch.zeros(n_env + 1, dtype=dtype, device=DEV),
          "policy_ready": torch.zeros(n_env + 1, dtype=torch.int32, device=DEV),
          "request_env": torch.full((cap,), -1, dtype=torch.int32, device=DEV),
          "request_noise": torch.zeros(cap, dtype=dtype, device=DEV),
          "request_obs": torch.zeros((cap, _lib.SIT_OBS_DIM), dtype=dtype, device=DEV),
          "request_count": torch.zeros(1, dtype=torch.int32, device=DEV),
          "request_age": torch.zeros(n_env, dtype=torch.int32, device=DEV),
          "env_steps": torch.zeros(1, dtype=torch.int64, device=DEV)}
    return io


def _rel(a, b, scale):
    a, b = np.asarray(a, dtype=np.float64), np.asarray(b, dtype=np.float64)
    return np.abs(a - b) / np.maximum(np.abs(b), scale)


SCALE_F = dict(north=1e4, east=1e4, yaw=np.pi, surge=10.0, sway=10.0, yaw_rate=0.1, shaft_speed=100.0,
               ship_speed_i=1e3, shaft_speed_i=1e5, heading_i=10.0, heading_prev=np.pi, e_ct_int=1e2,
               last_rpm=1e3, last_e_ct=1e3, last_power_me=1e3, sampling_dist=1e4, eps_dist=1e4,
               prev_pre_north=1e4, prev_pre_east=1e4, iw_north=1e4, iw_east=1e4)


def test_f32_policy_mode_step_vs_oracle():
    """One policy-mode step of the float32 kernel C5 runs, from float32-rounded states of 4096 envs at
    six episode depths, against the oracle's synchronous loop (OracleEnvs.policy_rollout, the loop of
    test_beds/main_ast.py:337-396) on the same state and actions.  At each depth a quarter of the envs
    are put at a sampling event (episode start or sampling distance >= AB_len); two thirds of those
    hold a ready action (policy_ready, an action in [-1, 1]) and step, the others wait for the policy.
    Stepping envs: next_state, reward, IW and post-state within 1e-5 relative (per-field floors);
    done, status, waypoint index, route length, stop flags, counters and replay transitions' discrete
    fields identical.  Waiting envs: ST_NO_STEP rows with done 0, state untouched, and their request
    (env id, observation, the event's normal draw) queued."""
    n_env = 4096
    sc = make_scenario(n_env, cap=32, seed=31)
    env64 = VecMultiShipRLEnv(scenario=sc, precision=64, device=DEV)
    env64.reset()
    env64.init_step()
    env32 = VecMultiShipRLEnv(scenario=sc, precision=32, device=DEV)
    o = so.OracleEnvs(dict(so.DEFAULT_PARAMS), sc.routes, sc.n_wpt, sc.init, sc.polys)
    worst, n_live_ev, n_wait = {}, 0, 0

    def upd(k, v):
        worst[k] = max(worst.get(k, 0.0), float(v))
    for depth in range(6):
        env64.rollout(300, seed=50 + depth)
        st = _f32_rounded(_np_state(env64))
        rng = np.random.default_rng(depth)
        # put a quarter of the envs at a sampling event (a third of those at an episode start)
        ev = rng.random(n_env) < 0.25
        start = ev & (rng.random(n_env) < 0.33)
        st["ep_step"] = np.where(start, 0, st["ep_step"])
        run = ev & ~start & (st["stop"][1] == 0)
        st["sampling_dist"] = np.where(run, np.float32(o.ab_len * 1.0001), st["sampling_dist"]).astype(np.float64)
        st["sampling_dist"] = st["sampling_dist"].astype(np.float32).astype(np.float64)
        need = (st["ep_step"] == 0) | ((st["sampling_dist"] >= o.ab_len) & (st["stop"][1] == 0))
        ready = need & (rng.random(n_env) < 0.67)
        wait = need & ~ready
        act = rng.uniform(-1, 1, n_env).astype(np.float32)
        o.set_state(st)
        env32.set_state(st)
        io = _policy_io(n_env, n_env, torch.float32)
        io["policy_action"][:n_env] = torch.from_numpy(act).to(DEV)
        io["policy_ready"][:n_env] = torch.from_numpy(ready.astype(np.int32)).to(DEV)
        seed = 700 + depth
        out = env32.rollout(1, seed=seed, policy_io=io, transition_capacity=2 * n_env, mask_horizon=600)
        assert "kPolicy" in env32.lib.sit_step_kernel(env32.handle).decode()
        post = _np_state(env32)
        live = ~wait

        def policy_fn(state, noise):
            return act[np.nonzero(need)[0]].astype(np.float64)
        r = o.policy_rollout(1, seed, policy_fn, mask_horizon=600)
        ref = o.get_state()
        # stepping envs
        ns, rew = out["next_state"][0].cpu().numpy(), out["reward"][0].cpu().numpy()
        upd("next_state", _rel(ns[live], r["next_state"][0][live], OBS_SCALE).max())
        upd("reward", _rel(rew[live], r["reward"][0][live], 1.0).max())
        done = out["done"][0].cpu().numpy().astype(bool)
        stat = out["status"][0].cpu().numpy().astype(np.int64) & 0xFFFFFFFF
        assert np.array_equal(done[live], r["done"][0][live]), f"depth {depth}: done"
        assert np.array_equal(stat[live], r["status"][0][live].astype(np.int64)), f"depth {depth}: status"
        a = out["action"][0].cpu().numpy().astype(np.float64)
        sac = r["action"][0, :, 3] > 0.5
        assert np.array_equal(a[live, 3] > 0.5, sac[live]), f"depth {depth}: sampling events"
        ev_live = live & sac
        n_live_ev += int(ev_live.sum())
        upd("iw", _rel(a[ev_live, :2], r["action"][0, ev_live, :2], 1e4).max() if ev_live.any() else 0.0)
        for k in so.SHIP_REAL:
            upd(k, _rel(post[k][:, live], ref[k][:, live], SCALE_F[k]).max())
        for k in so.ENV_REAL:
            upd(k, _rel(post[k][live], ref[k][live], SCALE_F[k]).max())
        for k in so.SHIP_INT:
            assert np.array_equal(post[k][:, live], ref[k][:, live].astype(post[k].dtype)), f"depth {depth}: {k}"
        for k in so.ENV_INT:
            assert np.array_equal(post[k][live].astype(np.int64), ref[k][live].astype(np.int64)), f"depth {depth}: {k}"
        # the consumed action slots are cleared, the unused ones keep their flag, the waiting envs
        # are marked SIT_POLICY_WAITING
        rd = io["policy_ready"][:n_env].cpu().numpy()
        want_rd = np.where(wait, _lib.SIT_POLICY_WAITING, (ready & ~need).astype(np.int32) * _lib.SIT_POLICY_READY)
        assert np.array_equal(rd, want_rd), f"depth {depth}: policy_ready"
        # replay transitions of the stepping envs' events (per env id; the kernel appends with atomics)
        cnt = int(out["transition_count"].item())
        got = out["transitions"][:cnt].cpu().numpy().astype(np.float64)
        want = r["transitions"]
        want = want[live[want[:, 23].astype(np.int64)]]
        assert cnt == len(want), f"depth {depth}: transitions {cnt} vs {len(want)}"
        if cnt:
            got, want = got[np.argsort(got[:, 23])], want[np.argsort(want[:, 23])]
            assert np.array_equal(got[:, 23], want[:, 23]) and np.array_equal(got[:, 22], want[:, 22])
            assert np.abs(got[:, 10] - want[:, 10]).max() <= 1e-7         # the policy's action
            cols = np.r_[0:10, 12:22]
            upd("transitions", _rel(got[:, cols], want[:, cols], np.r_[OBS_SCALE, OBS_SCALE]).max())
        # waiting envs: no step, state untouched, request queued
        n_wait += int(wait.sum())
        assert np.all(stat[wait] == _lib.ST_NO_STEP) and not done[wait].any(), f"depth {depth}: waiting rows"
        for k in so.SHIP_REAL + so.SHIP_INT:
            assert np.array_equal(post[k][:, wait], st[k][:, wait].astype(post[k].dtype)), f"depth {depth}: {k} moved"
        for k in so.ENV_REAL + so.ENV_INT:
            assert np.array_equal(post[k][wait], st[k][wait].astype(post[k].dtype)), f"depth {depth}: {k} moved"
        q = int(io["request_count"].item())
        assert q == int(wait.sum()), f"depth {depth}: {q} requests for {int(wait.sum())} waiting envs"
        renv = io["request_env"][:q].cpu().numpy()
        # the admission queues the waiting envs in env-id order (all of them: capacity = n_env)
        assert np.array_equal(renv, np.nonzero(wait)[0]), f"depth {depth}: request env ids"
        assert not io["request_age"].any(), f"depth {depth}: admitted envs keep an age"
        robs = io["request_obs"][:q].cpu().numpy().astype(np.float64)
        assert np.array_equal(robs, st["last_obs"].T[renv]), f"depth {depth}: request observations"
        noise = so.sampler_normal(seed, renv.astype(np.uint64), st["event"][renv])
        assert np.abs(io["request_noise"][:q].cpu().numpy() - noise).max() <= 1e-6 * max(1.0, np.abs(noise).max())
        assert int(io["env_steps"].item()) == int(live.sum())
    print("f32 policy-mode step worst:", {k: f"{v:.2e}" for k, v in worst.items()},
          f"events stepped {n_live_ev}, envs waiting {n_wait}")
    bad = {k: f"{v:.2e}" for k, v in worst.items() if v > 1e-5}
    assert not bad, bad
    assert n_live_ev > 1000 and n_wait > 500


def _executed_rows(outs_list, n_env):
    """Per env, the executed (status without ST_NO_STEP) rows of a list of launch outputs."""
    seq = [[] for _ in range(n_env)]
    for o in outs_list:
        st = o["status"].astype(np.int64) & 0xFFFFFFFF
        live = (st & _lib.ST_NO_STEP) == 0
        for k in range(st.shape[0]):
            for e in np.nonzero(live[k])[0]:
                seq[e].append((o["next_state"][k, e], o["reward"][k, e], int(st[k, e])))
    return seq


def test_f32_c5_size_fused_actor_graph_replay():
    """Config C5 at its configured size: 65 536 ships (2 groups x 16 384 envs) on two streams, the fused
    256x256 actor, 16 launches per HIP graph, as bench.py --mode policy runs it.  Properties: the
    executed rows account for the device env-step counter, ST_NO_STEP rows carry done 0, outputs are
    finite, the policy served every
    group more than once per env; and batching independence: the first 512 envs of group 0, run as a
    512-env handle with the same global ids and policy, execute bit-identical rows."""
    n, G, chunk, per_graph = 16384, 2, 32, 16
    pol = make_policy256(DEV)
    samplers = []
    for g in range(G):
        env = VecMultiShipRLEnv(scenario=make_scenario(n, cap=48, seed=25450, env_offset=g * n), precision=32,
                                device=DEV)
        env.reset()
        env.init_step()
        samplers.append(PolicySampler(env, pol, chunk=chunk, seed=SEED, env_id_offset=g * n,
                                      request_capacity=n // 4, transition_capacity=per_graph * chunk * n // 64))
    assert all(s.fused for s in samplers)
    ov = OverlappedPolicySampler(samplers).capture(per_graph)
    assert "k_env_steps_sync<float,kPolicy" in samplers[0].env.lib.sit_step_kernel(samplers[0].env.handle).decode()
    before = [int(s.env_steps.item()) for s in samplers]
    rows_g0 = []
    for rep in range(3):
        outs = ov.replay()
        torch.cuda.synchronize()
        for s, out in zip(samplers, outs):
            st = out["status"].to(torch.int64) & 0xFFFFFFFF
            live = (st & _lib.ST_NO_STEP) == 0
            assert torch.isfinite(out["next_state"][live]).all() and torch.isfinite(out["reward"][live]).all()
            assert not out["done"][~live].any()
            # the graph's launches append their replay transitions to one buffer: at least the last
            # launch's sampling events, none dropped
            ev = (out["action"][..., 3] > 0.5) & live
            cnt = int(out["transition_count"].item())
            assert int(ev.sum().item()) <= cnt <= s.transition_capacity, (int(ev.sum().item()), cnt)
    stepped = [int(s.env_steps.item()) - b for s, b in zip(samplers, before)]
    for s in stepped:
        assert s > 0.8 * 3 * per_graph * chunk * n, stepped
    for s in samplers:
        assert int(s.served.item()) > n
    # batching independence (eager launches; the graph's launches are the same kernels): the first
    # 512 envs as part of the 16 384-env handle and as a 512-env handle execute identical rows; each
    # handle's per-env progress obeys the admission's FIFO bound and is reproducible
    m, n_launch = 512, 12
    envs, counts = [], []
    for nn in (n, m):
        env = VecMultiShipRLEnv(scenario=make_scenario(nn, cap=48, seed=25450, env_offset=0), precision=32,
                                device=DEV)
        env.reset()
        env.init_step()
        sm = PolicySampler(env, pol, chunk=chunk, seed=SEED, env_id_offset=0, request_capacity=nn // 4)
        outs, stalled = [], []
        for _ in range(n_launch):
            o = sm.launch()
            torch.cuda.synchronize()
            outs.append({k: o[k][:, :m].cpu().numpy().copy() for k in ("next_state", "reward", "status")})
            st = o["status"].to(torch.int64) & 0xFFFFFFFF
            stalled.append(((st & _lib.ST_NO_STEP) != 0).all(0).cpu().numpy())
        envs.append(_executed_rows(outs, m))
        _assert_fifo_bound(np.stack(stalled), nn, nn // 4)
    big, small = envs
    compared = 0
    for e in range(m):
        k = min(len(big[e]), len(small[e]))
        assert k >= 1, f"env {e}: no rows"
        for i in range(k):
            assert np.array_equal(big[e][i][0], small[e][i][0]) and big[e][i][1] == small[e][i][1] \
                and big[e][i][2] == small[e][i][2], f"env {e} row {i}"
        compared += k
    assert compared > 100000, compared


def _assert_fifo_bound(stalled, n_env, cap):
    """stalled [launch, env]: the env took no step in the launch.  A request made in launch L is
    admitted by round L + ceil(n/cap) - 1 and its action consumed in the next launch, so an env
    takes no step in at most ceil(n/cap) consecutive launches (include/sit.h, sit_rollout_args)."""
    bound = -(-n_env // cap)
    run = np.zeros(stalled.shape[1], dtype=np.int64)
    worst = np.zeros_like(run)
    for row in stalled:
        run = np.where(row, run + 1, 0)
        worst = np.maximum(worst, run)
    assert worst.max() <= bound, f"an env waited {worst.max()} launches in a row (bound {bound})"
    return worst


def _admission_model(ready_after, age_before, cap):
    """The admission rule in numpy: waiting envs (policy_ready == SIT_POLICY_WAITING) age by one round;
    the oldest `cap` (ties by env id; ages of 16 and more share one bucket) are queued in env-id order and
    their age reset; the others keep waiting with their age; envs not waiting have age 0."""
    n = age_before.size
    wait = ready_after[:n] == _lib.SIT_POLICY_WAITING
    age = np.where(wait, np.minimum(age_before.astype(np.int64) + 1, 1 << 30), 0)
    cand = np.nonzero(wait)[0]
    order = cand[np.lexsort((cand, -np.minimum(age[cand], 16)))]
    adm = np.sort(order[:cap])
    age[adm] = 0
    return adm, age


def _run_overflowing(n, cap, chunk, n_launch, pol, check_model):
    """n envs, capacity cap < the demand, eager launches; per launch the admitted queue is checked
    against _admission_model (check_model).  Returns the per-env executed-row counts and the
    [launch, env] fully-stalled matrix."""
    env = VecMultiShipRLEnv(scenario=make_scenario(n, cap=48, seed=77), precision=32, device=DEV)
    env.reset()
    env.init_step()
    sm = PolicySampler(env, pol, chunk=chunk, seed=SEED, request_capacity=cap)
    io = sm.io
    rows = np.zeros(n, dtype=np.int64)
    stalled, overflowed = [], 0
    for _ in range(n_launch):
        age0 = io["request_age"].cpu().numpy().copy()
        env.rollout(chunk, seed=SEED, out=sm.out, want=("next_state", "reward", "done", "status", "action"),
                    policy_io=io)
        torch.cuda.synchronize()
        if check_model:
            ready = io["policy_ready"].cpu().numpy()
            adm, age = _admission_model(ready, age0, cap)
            q = int(io["request_count"].item())
            assert q == adm.size, (q, adm.size)
            assert np.array_equal(io["request_env"][:q].cpu().numpy(), adm)
            assert np.array_equal(io["request_age"].cpu().numpy(), age)
            overflowed += int((ready[:n] == _lib.SIT_POLICY_WAITING).sum()) - q
        sm.act()
        st = sm.out["status"].to(torch.int64) & 0xFFFFFFFF
        live = (st & _lib.ST_NO_STEP) == 0
        rows += live.sum(0).cpu().numpy()
        stalled.append((~live).all(0).cpu().numpy())
    if check_model:
        assert overflowed > 0, "the queue never overflowed"
    assert int(rows.sum()) == int(sm.env_steps.item())
    return rows, np.stack(stalled)


def test_f32_policy_admission_is_deterministic_and_fifo():
    """An overflowing request queue (capacity n/8): the admitted rows of every launch equal the
    admission rule's (oldest request first, ties by env id; _admission_model), two runs from the same
    start execute identical per-env row counts, and no env waits longer than the FIFO bound."""
    n, chunk, n_launch = 4096, 32, 16
    cap = n // 8
    pol = make_policy256(DEV)
    rows1, st1 = _run_overflowing(n, cap, chunk, n_launch, pol, check_model=True)
    rows2, st2 = _run_overflowing(n, cap, chunk, n_launch, pol, check_model=False)
    assert np.array_equal(rows1, rows2), "per-env progress differs between two identical runs"
    assert np.array_equal(st1, st2)
    worst = _assert_fifo_bound(st1, n, cap)
    assert worst.max() >= 2, "the test did not exercise waiting across launches"
    print(f"admission: rows/env min {rows1.min()} mean {rows1.mean():.1f}, longest wait {worst.max()} launches")


def test_f64_intermediate_waypoint_sampler_switches_to_policy():
    """IntermediateWaypointSampler (the reference's empty ast_core sampler): random IWs (mode 0, device
    Philox draws) for the first start_steps env-steps, then the policy (mode 1) — main_ast.py:335-348.
    Per env: the random phase equals OracleEnvs.rollout, the policy phase equals OracleEnvs.policy_rollout
    continued from the same state (float64, 1e-9)."""
    from sac_maritime_ast_amd.samplers import IntermediateWaypointSampler
    n_env, chunk, n_rand, n_pol = 64, 16, 6, 30
    sc = make_scenario(n_env, cap=32, seed=13)
    env = VecMultiShipRLEnv(scenario=sc, precision=64, device=DEV)
    env.reset()
    env.init_step()
    ims = IntermediateWaypointSampler(env, make_policy(torch.float64, DEV), chunk=chunk, seed=SEED,
                                      start_steps=n_rand * chunk * n_env, request_capacity=n_env // 2)
    rand_rows, pol_rows = [], []
    for i in range(n_rand + n_pol):
        out = ims.launch()
        torch.cuda.synchronize()
        snap = {k: v.cpu().numpy().copy() for k, v in out.items() if k != "done_count"}
        (rand_rows if i < n_rand else pol_rows).append([snap])
    assert ims.policy_sampler.served.item() > 0
    o = so.OracleEnvs(dict(so.DEFAULT_PARAMS), sc.routes, sc.n_wpt, sc.init, sc.polys)
    o.reset()
    o.init_step()
    r = o.rollout(n_rand * chunk, SEED)
    got = {k: np.concatenate([l[0][k] for l in rand_rows]) for k in ("next_state", "reward", "done", "status")}
    err = np.abs(got["next_state"] - r["next_state"]) / np.maximum(np.abs(r["next_state"]), OBS_SCALE)
    assert err.max() <= 1e-9, f"random phase rel err {err.max():.3e}"
    assert np.array_equal(got["done"].astype(bool), r["done"])
    assert np.array_equal(got["status"].astype(np.int64) & 0xFFFFFFFF, r["status"].astype(np.int64))
    seq = per_env(pol_rows, 0, n_env)
    n = min(len(x) for x in seq["reward"])
    assert n >= 200, n
    ref = o.policy_rollout(n, SEED, oracle_policy_fn(make_policy(torch.float64, "cpu")))
    compare(seq, ref, n_env, n)


# ------------------------------------------------------------------------------------------
# in-kernel serving (sit_rollout_args.actor_weights): the step kernel evaluates the actor for the
# envs of each block that end the launch waiting (csrc/sit_serve.h)
# ------------------------------------------------------------------------------------------
def _same(a, b):
    """Bitwise equal, NaN where NaN (the route-angle column of non-event rows)."""
    return torch.equal(torch.isnan(a), torch.isnan(b)) and torch.equal(torch.nan_to_num(a), torch.nan_to_num(b))


def _serving_samplers(n, precision, chunk, serves, deterministic=False, seed=77, tcap=0):
    pol = make_policy256(DEV)
    out = []
    for serve in serves:
        env = VecMultiShipRLEnv(scenario=make_scenario(n, cap=48, seed=seed), precision=precision, device=DEV)
        env.reset()
        env.init_step()
        out.append(PolicySampler(env, pol, chunk=chunk, seed=SEED, serve=serve, deterministic=deterministic,
                                 transition_capacity=tcap))
    return pol, out


@pytest.mark.parametrize("precision", [32, 64])
def test_in_kernel_serving_equals_queue_path(precision):
    """In-kernel serving against the request queue at capacity n_env served by sit_policy_actor, from
    the same start: every launch's rows (next_state, reward, done, status, action), the action slots
    and ready flags, the replay transitions, and the served / env-step counters are identical bit for
    bit (include/sit.h: both paths share the actor's per-row arithmetic), and no env ever waits more
    than the launch it stopped in."""
    n, chunk, n_launch = (2000, 32, 12) if precision == 32 else (500, 32, 10)   # (a partial last block)
    _, (k, q) = _serving_samplers(n, precision, chunk, ("kernel", "queue"), tcap=chunk * n // 32)
    assert k.serve == "kernel" and q.serve == "queue"
    assert "request_env" not in k.io
    prev_wait = np.zeros(n, dtype=bool)
    for it in range(n_launch):
        ok, oq = k.launch(), q.launch()
        torch.cuda.synchronize()
        for key in ("done", "status"):
            assert torch.equal(ok[key], oq[key]), f"launch {it}: {key}"
        live = (ok["status"].to(torch.int64) & _lib.ST_NO_STEP) == 0   # (ST_NO_STEP rows are not written)
        for key in ("next_state", "reward", "action"):
            assert _same(ok[key][live], oq[key][live]), f"launch {it}: {key}"
        assert torch.equal(k.io["policy_action"][:n], q.io["policy_action"][:n]), f"launch {it}: actions"
        rk, rq = k.io["policy_ready"][:n].cpu().numpy(), q.io["policy_ready"][:n].cpu().numpy()
        assert np.array_equal(rk, rq), f"launch {it}: ready flags"
        assert not (rk == _lib.SIT_POLICY_WAITING).any()
        ck, cq = int(ok["transition_count"].item()), int(oq["transition_count"].item())
        assert ck == cq, f"launch {it}: transitions {ck} vs {cq}"
        tk = ok["transitions"][:ck].cpu().numpy()
        tq = oq["transitions"][:cq].cpu().numpy()
        tk, tq = tk[np.lexsort(tk.T[::-1])], tq[np.lexsort(tq.T[::-1])]
        assert np.array_equal(tk, tq), f"launch {it}: transition records"
        st = ok["status"].to(torch.int64).cpu().numpy() & 0xFFFFFFFF
        waiting = ((st & _lib.ST_NO_STEP) != 0).all(0)
        assert not (waiting & prev_wait).any(), f"launch {it}: an env waited two launches in a row"
        prev_wait = waiting
    assert int(k.served.item()) == int(q.served.item()) >= n
    assert int(k.env_steps.item()) == int(q.env_steps.item())


@pytest.mark.parametrize("precision,deterministic", [(32, False), (32, True), (64, False)])
def test_in_kernel_serving_actions_match_torch_float64(precision, deterministic):
    """The actions the step kernel serves against the same policy in float64 PyTorch on each served
    env's observation (state last_obs) and its event's normal draw (oracle sampler_normal): |error|
    <= 1e-5; the served counter advances by the envs served (all envs waiting at the end of the
    launch; the ready flags are cleared before each launch so that every env at an event waits)."""
    n = 2048
    pol, (k,) = _serving_samplers(n, precision, 32, ("kernel",), deterministic=deterministic, seed=7)
    ref_pol = copy.deepcopy(pol).double()
    checked = 0
    for it in range(6):
        k.io["policy_ready"].zero_()
        before = int(k.served.item())
        k.launch()
        torch.cuda.synchronize()
        served = np.nonzero(k.io["policy_ready"][:n].cpu().numpy() == _lib.SIT_POLICY_READY)[0]
        assert int(k.served.item()) - before == served.size
        st = _np_state(k.env)
        obs = torch.from_numpy(st["last_obs"].T[served].astype(np.float64)).to(DEV)
        ev = st["event"][served].astype(np.uint32)
        noise = torch.from_numpy(np.asarray(so.sampler_normal(SEED, served.astype(np.uint64), ev))).to(DEV)
        with torch.no_grad():
            ref = ref_pol(obs, noise, deterministic=deterministic)[0][:, 0]
        got = k.io["policy_action"][torch.from_numpy(served).to(DEV)].double()
        if served.size:
            err = (got - ref).abs().max().item()
            assert err <= 1e-5, f"launch {it}: served action max |err| {err:.3e} over {served.size} envs"
            assert ref.abs().max().item() > (1e-3 if deterministic else 0.05)
        checked += served.size
    assert checked >= n


def test_in_kernel_serving_logged_launch_takes_library_queue():
    """A logged policy launch runs the one-wave kernel, which cannot serve in-kernel: the library
    serves it through its own queue (capacity n_env) and sit_policy_actor.  Float64: the logged run's
    done / status rows and ready flags equal the unlogged (in-kernel) run's, launch by launch, its
    reals within 1e-9 (the two step kernels' float64 contract) and its served actions within 1e-6
    (float32 actor on observations equal to 1e-9)."""
    n, chunk = 256, 16
    _, (a, b) = _serving_samplers(n, 64, chunk, ("kernel", "kernel"), seed=21)
    for it in range(8):
        oa = a.env.rollout(chunk, seed=SEED, out=a.out, policy_io=a.io, log=True,
                           want=("next_state", "reward", "done", "status", "action"))
        name = a.env.lib.sit_step_kernel(a.env.handle).decode()
        ob = b.launch()
        torch.cuda.synchronize()
        assert name.startswith("k_env_steps<") and "log" in name, name
        for key in ("done", "status"):
            assert torch.equal(oa[key], ob[key]), f"launch {it}: {key}"
        live = (oa["status"].to(torch.int64) & _lib.ST_NO_STEP) == 0
        for key, floor in (("next_state", torch.tensor(OBS_SCALE, device=DEV)), ("reward", 1.0),
                           ("action", torch.tensor([1e4, 1e4, np.pi, 1.0], device=DEV, dtype=torch.float64))):
            x, y = oa[key][live], ob[key][live]
            assert torch.equal(torch.isnan(x), torch.isnan(y)), f"launch {it}: {key} NaN pattern"
            err = (torch.nan_to_num(x) - torch.nan_to_num(y)).abs() / torch.maximum(
                torch.nan_to_num(y).abs(), torch.as_tensor(floor, device=DEV, dtype=y.dtype).expand_as(y))
            assert err.numel() == 0 or err.max().item() <= 1e-9, f"launch {it}: {key} rel err {err.max().item():.3e}"
        assert (a.io["policy_action"][:n] - b.io["policy_action"][:n]).abs().max().item() <= 1e-6, f"launch {it}"
        assert torch.equal(a.io["policy_ready"][:n], b.io["policy_ready"][:n]), f"launch {it}: ready"
    assert int(a.served.item()) == int(b.served.item()) > 0


def test_f32_c5_size_in_kernel_serving_graph_replay():
    """Config C5 as bench.py runs it by default: 65 536 ships (2 groups x 16 384 envs, two streams), the
    256x256 actor served inside the step kernel, 16 launches per HIP graph.  Properties: executed rows
    account for the device env-step counter, ST_NO_STEP rows carry done 0, outputs are finite, every env
    is served; no env takes no step in two launches in a row; and batching independence: the first 512
    envs of a 16 384-env handle and of a 512-env handle (same global ids and policy) execute identical
    rows, launch by launch."""
    n, G, chunk, per_graph = 16384, 2, 64, 16
    pol = make_policy256(DEV)
    samplers = []
    for g in range(G):
        env = VecMultiShipRLEnv(scenario=make_scenario(n, cap=48, seed=25450, env_offset=g * n), precision=32,
                                device=DEV)
        env.reset()
        env.init_step()
        samplers.append(PolicySampler(env, pol, chunk=chunk, seed=SEED, env_id_offset=g * n,
                                      transition_capacity=per_graph * chunk * n // 64))
    assert all(s.serve == "kernel" for s in samplers)
    ov = OverlappedPolicySampler(samplers).capture(per_graph)
    before = [int(s.env_steps.item()) for s in samplers]
    for rep in range(3):
        outs = ov.replay()
        torch.cuda.synchronize()
        for s, out in zip(samplers, outs):
            st = out["status"].to(torch.int64) & 0xFFFFFFFF
            live = (st & _lib.ST_NO_STEP) == 0
            assert torch.isfinite(out["next_state"][live]).all() and torch.isfinite(out["reward"][live]).all()
            assert not out["done"][~live].any()
            assert not (s.io["policy_ready"][:n] == _lib.SIT_POLICY_WAITING).any()
    stepped = [int(s.env_steps.item()) - b for s, b in zip(samplers, before)]
    for s in stepped:
        assert s > 0.8 * 3 * per_graph * chunk * n, stepped
    for s in samplers:
        assert int(s.served.item()) > n
    m, n_launch = 512, 10
    rows = []
    for nn in (n, m):
        env = VecMultiShipRLEnv(scenario=make_scenario(nn, cap=48, seed=25450, env_offset=0), precision=32,
                                device=DEV)
        env.reset()
        env.init_step()
        sm = PolicySampler(env, pol, chunk=chunk, seed=SEED, env_id_offset=0)
        outs, prev = [], np.zeros(m, dtype=bool)
        for _ in range(n_launch):
            o = sm.launch()
            torch.cuda.synchronize()
            outs.append({k: o[k][:, :m].cpu().numpy().copy() for k in ("next_state", "reward", "status", "done")})
            st = outs[-1]["status"].astype(np.int64) & 0xFFFFFFFF
            waited = ((st & _lib.ST_NO_STEP) != 0).all(0)
            assert not (waited & prev).any(), "an env took no step in two launches in a row"
            prev = waited
        rows.append(outs)
    for i, (x, y) in enumerate(zip(*rows)):
        assert np.array_equal(x["status"], y["status"]) and np.array_equal(x["done"], y["done"]), f"launch {i}"
        live = ((x["status"].astype(np.int64) & _lib.ST_NO_STEP) == 0)
        assert np.array_equal(x["next_state"][live], y["next_state"][live]), f"launch {i}: next_state"
        assert np.array_equal(x["reward"][live], y["reward"][live]), f"launch {i}: reward"


def test_rollout_serving_argument_checks():
    """sit_rollout's policy-mode argument rules (include/sit.h), checked before anything is launched:
    actor_weights need policy mode and policy_ready; without actor_weights every request buffer and a
    positive capacity are required; policy mode and explicit actions are exclusive.  A serving launch
    with the request buffers left NULL is accepted."""
    import ctypes
    n = 128
    env = VecMultiShipRLEnv(scenario=make_scenario(n, cap=32, seed=3), precision=32, device=DEV)
    env.reset()
    env.init_step()
    w = torch.zeros(_lib.SIT_ACTOR_WEIGHTS, dtype=torch.float32, device=DEV)
    act = torch.zeros(n + 1, dtype=torch.float32, device=DEV)
    ready = torch.zeros(n + 1, dtype=torch.int32, device=DEV)
    ns = torch.empty((1, n, _lib.SIT_OBS_DIM), dtype=torch.float32, device=DEV)
    ane = torch.zeros((1, n, 2), dtype=torch.float32, device=DEV)
    u8 = torch.zeros((1, n), dtype=torch.uint8, device=DEV)

    def call(**kw):
        ra = _lib.RolloutArgs()
        ra.n_steps, ra.auto_reset, ra.seed = 1, 1, 1
        ra.next_state = ns.data_ptr()
        for k, v in kw.items():
            setattr(ra, k, v)
        with torch.cuda.device(DEV):
            rc = env.lib.sit_rollout(env.handle, ctypes.byref(ra), env._stream())
        return rc, env.lib.sit_last_error(env.handle)

    rc, msg = call(actor_weights=w.data_ptr())
    assert rc == _lib.SIT_E_INVALID and b"policy mode" in msg
    rc, msg = call(actor_weights=w.data_ptr(), policy_action=act.data_ptr())
    assert rc == _lib.SIT_E_INVALID and b"policy_ready" in msg
    rc, msg = call(policy_action=act.data_ptr(), policy_ready=ready.data_ptr())
    assert rc == _lib.SIT_E_INVALID and b"request_capacity" in msg
    rc, msg = call(policy_action=act.data_ptr(), policy_ready=ready.data_ptr(), actor_weights=w.data_ptr(),
                   action_ne=ane.data_ptr(), sac_update=u8.data_ptr(), init=u8.data_ptr())
    assert rc == _lib.SIT_E_INVALID and b"exclusive" in msg
    rc, msg = call(policy_action=act.data_ptr(), policy_ready=ready.data_ptr(), actor_weights=w.data_ptr())
    torch.cuda.synchronize()
    assert rc == 0, msg
    assert "kPolicy" in env.lib.sit_step_kernel(env.handle).decode()
    # every env started at its episode's first sampling event with no action: served in the same launch
    assert (ready[:n] == _lib.SIT_POLICY_READY).all()


def test_torch_actor_on_its_stream_matches_fused_actor():
    """The PyTorch-ROCm actor as bench.py's c5_torch_actor line runs it — each hidden Linear + ReLU one GEMM
    with the ReLU in its epilogue (samplers._trunk), the head and scatter in sit_policy_apply (which also
    counts the served rows), the actor forked onto a HIP stream of its own after the launch and joined
    before the next — against the fused HIP actor on the same request queue (float32, 1 024 envs): the
    first launch stops every env at its episode's first sampling event, so both queues hold every env;
    the actions agree within 1e-5 and the served counts are equal."""
    n_env = 1024
    pol = make_policy256(DEV)
    out = []
    for fused, stream in ((True, False), (False, True)):
        env = VecMultiShipRLEnv(scenario=make_scenario(n_env, cap=48, seed=5), precision=32, device=DEV)
        env.reset()
        env.init_step()
        sm = PolicySampler(env, pol, chunk=32, seed=SEED, request_capacity=n_env, serve="queue", fused_actor=fused,
                           actor_stream=stream)
        assert sm.fused == fused and (sm.actor_stream is not None) == stream
        sm.launch()
        torch.cuda.synchronize()
        cnt = int(sm.io["request_count"].item())
        out.append((cnt, sm.io["request_env"][:cnt].cpu().numpy(), sm.io["policy_action"][:n_env].cpu().numpy(),
                    sm.io["policy_ready"][:n_env].cpu().numpy(), int(sm.served.item())))
    (c0, e0, a0, r0, s0), (c1, e1, a1, r1, s1) = out
    assert c0 == c1 == n_env and np.array_equal(e0, e1)
    assert s0 == s1 == n_env
    assert np.array_equal(r0, r1) and (r0 == _lib.SIT_POLICY_READY).all()
    err = np.abs(a0.astype(np.float64) - a1.astype(np.float64)).max()
    print(f"PyTorch actor (fused ReLU epilogues, own stream) vs fused HIP actor: max |action| difference {err:.2e}")
    assert err <= 1e-5
