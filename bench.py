#!/usr/bin/env python3
"""Benchmark: env-steps/s of the two-ship SAC-AST environment on MI355X (BASELINE.json metric).

A bench "step" is one MultiShipRLEnv.step (RLEnv/MSRL_Env.py:404-442 + MSRL_env_ex.py:906-980)
of every env: both ships (guidance, control, machinery, 3-DOF hull, Euler) plus reward,
termination and status, with the synthetic random-IW sampler and auto-reset.
Config C3: 65 536 ships = 32 768 two-ship envs per GPU (weak scaling over ranks).  Steps run as
fused launches of --chunk steps; every step's full output (next_state[10], reward, done,
status, IW action) is written to HBM.  Inputs (env state) are resident in HBM before timing.

Multi-GPU: one process per GPU (torchrun); each rank owns an independent env shard (global
env ids offset by rank, no data-path collective) and, once per chunk, the replay transitions
of that chunk's sampling events (the only data the SAC learner consumes, test_beds/main_ast.py:
395-396) are compacted on device and all-gathered over RCCL to every rank (rank 0 = learner).
"""
from __future__ import annotations

import argparse
import glob
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

METRIC = "env-steps/sec at 64k parallel ships, 1/2/4/8 MI355X; fp32 match vs NumPy"
HBM_PEAK_GBS = 8000.0   # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=6000)
    ap.add_argument("--warmup", type=int, default=600)
    ap.add_argument("--n-env", type=int, default=32768, help="two-ship envs per GPU (32768 = 64k ships)")
    ap.add_argument("--chunk", type=int, default=200, help="env steps fused per kernel launch")
    ap.add_argument("--precision", type=int, default=32, choices=(32, 64))
    ap.add_argument("--seed", type=int, default=25450)
    ap.add_argument("--mode", default="rollout", choices=("rollout", "step"),
                    help="rollout: fused K-step launches; step: one sit_step launch per env step")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--launch-trace", action="store_true", help="print every launch's kernel ms to stderr")
    return ap.parse_args()


def algorithmic_bytes_per_launch(n_env, k, rs, mean_nw_obs, mean_nw_test, mode):
    """Bytes a launch must move (no padding, no redundant reloads).  rs = bytes per real."""
    ship_state = 15 * rs + 4 * 4            # 15 reals + next_wpt, n_wpt, ticks, stop
    env_state = 6 * rs + 3 * 4              # sampling/eps dist, prev pos, IW + ep_step, event, episodes
    scen = 2 * 3 * rs + 2 * 8               # per env: end wpt + desired speed per ship, AB len/alpha
    routes = 2 * rs * ((mean_nw_obs - 1) * 2 + (mean_nw_test - 1))   # obs read+write back, test read
    out_step = 15 * rs + 1 + 4              # next_state 10 + reward + IW action 4, done u8, status u32
    if mode == "rollout":
        per_env = 2 * (2 * ship_state + env_state) + scen + routes + k * out_step
    else:  # per-step launch: state in and out every step, explicit action in
        per_env = k * (2 * (2 * ship_state + env_state) + scen + 2 * rs * 3 + 2 * rs + 2 + out_step - 4 * rs)
    return n_env * per_env


def latest_pmc(precision, mode):
    """HBM bytes per launch from the committed rocprofv3 PMC summary of this config, if any."""
    best = None
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json"))):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("precision") == precision and d.get("mode") == mode and d.get("n_env") == 32768:
            best = d
    return best


def cpu_baseline(seconds, seed):
    """The oracle (float64 NumPy restatement, vectorised over envs, 1 core) on a bounded sample of
    the same workload: 2048 envs, synthetic sampler, auto-reset, until ~`seconds` of CPU work."""
    from oracle import sit_oracle as so  # CPU baseline leg only
    from sac_maritime_ast_amd.scenario import make_scenario
    n_env = 2048
    sc = make_scenario(n_env, cap=32)
    o = so.OracleEnvs(dict(so.DEFAULT_PARAMS), sc.routes, sc.n_wpt, sc.init, sc.polys)
    o.reset()
    o.init_step()
    o.rollout(2, seed)
    steps, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        o.rollout(10, seed)
        steps += 10
    dt = time.perf_counter() - t0
    return {"value": n_env * steps / dt, "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"oracle/sit_oracle.py float64 NumPy, {n_env} envs x {steps} steps (synthetic "
                      f"sampler, auto-reset), {dt:.1f} s on 1 host core"}


class TransitionGather:
    """Per chunk: compact sampling-event transitions (state, action a, reward, next_state, mask)
    on device and all-gather them over RCCL (fixed-capacity records)."""

    def __init__(self, n_env, chunk, dtype, device, world, enabled):
        self.world, self.enabled = world, enabled and world > 1
        self.cap = max(1024, n_env * chunk // 64)
        self.rec = torch.zeros((self.cap, 24), dtype=dtype, device=device)
        self.gathered = torch.empty((world, self.cap, 24), dtype=dtype, device=device) if self.enabled else None
        self.prev = None
        self.count = torch.zeros(1, dtype=torch.int64, device=device)
        self.total = 0

    def __call__(self, out, initial_state):
        ns = out["next_state"]
        if self.prev is None:
            self.prev = initial_state.clone()
        state = torch.cat([self.prev[None], ns[:-1]], 0)
        sel = out["action"][..., 3] > 0.5
        idx = sel.nonzero(as_tuple=False)
        k = min(idx.shape[0], self.cap)
        idx = idx[:k]
        t, e = idx[:, 0], idx[:, 1]
        r = self.rec
        r[:k, 0:10] = state[t, e]
        r[:k, 10] = out["action"][t, e, 2]
        r[:k, 11] = out["reward"][t, e]
        r[:k, 12:22] = ns[t, e]
        r[:k, 22] = 1.0 - out["done"][t, e].to(r.dtype)
        r[:k, 23] = float(k)
        self.prev = ns[-1]
        self.total += k
        if self.enabled:
            import torch.distributed as dist
            dist.all_gather_into_tensor(self.gathered, r)


def main():
    args = parse()
    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)
    from sac_maritime_ast_amd import VecMultiShipRLEnv, make_scenario

    n_env = args.n_env
    sc = make_scenario(n_env, cap=48, seed=args.seed + rank)
    env = VecMultiShipRLEnv(scenario=sc, precision=args.precision, device=dev)
    init_obs = env.reset()
    env.init_step()
    chunk = args.chunk if args.mode == "rollout" else 1
    steps = (args.steps // chunk) * chunk
    warm = max(chunk, (args.warmup // chunk) * chunk)
    offset = rank * n_env
    out = {}
    gather = TransitionGather(n_env, chunk, env.dtype, dev, world, not args.no_gather)
    stream = torch.cuda.current_stream(dev)

    # per-step mode: precomputed random IW actions (explicit inputs), one launch per env step
    if args.mode == "step":
        g = torch.Generator(device=dev).manual_seed(args.seed)
        st = env.get_state()
        step_act = torch.stack([st["north"][1], st["east"][1]], 1) + torch.randn(n_env, 2, device=dev,
                                                                                dtype=env.dtype, generator=g) * 500
        step_sac = (torch.rand(n_env, device=dev, generator=g) < 0.005).to(torch.uint8)
        step_init = torch.zeros(n_env, dtype=torch.uint8, device=dev)
        ns = torch.empty((n_env, 10), dtype=env.dtype, device=dev)
        rew = torch.empty((n_env,), dtype=env.dtype, device=dev)
        done = torch.empty((n_env,), dtype=torch.uint8, device=dev)
        stat = torch.empty((n_env,), dtype=torch.int32, device=dev)
        dcount = torch.zeros(1, dtype=torch.int32, device=dev)

        def one(i):
            env._call("sit_step", step_act.data_ptr(), step_sac.data_ptr(), step_init.data_ptr(),
                      ns.data_ptr(), rew.data_ptr(), done.data_ptr(), stat.data_ptr(), dcount.data_ptr(),
                      env._stream())
    else:
        def one(i):
            env.rollout(chunk, seed=args.seed, env_id_offset=offset, out=out)
            if gather.enabled:
                gather(out, init_obs)

    for i in range(warm // chunk):
        one(i)
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    n_launch = steps // chunk
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_launch)]
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(n_launch):
        if args.mode == "rollout":
            ev[i][0].record(stream)
            env.rollout(chunk, seed=args.seed, env_id_offset=offset, out=out)
            ev[i][1].record(stream)
            if gather.enabled:
                gather(out, init_obs)
        else:
            ev[i][0].record(stream)
            one(i)
            ev[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(t.item())
    launch_ms = [a.elapsed_time(b) for a, b in ev]
    kern_ms = float(np.mean(launch_ms))
    if args.launch_trace:
        print("launch_ms " + " ".join(f"{x:.4f}" for x in launch_ms), file=sys.stderr)

    st = env.get_state()
    mean_nw_obs = float(st["n_wpt"][1].double().mean().item())
    mean_nw_test = float(st["n_wpt"][0].double().mean().item())
    rs = 4 if args.precision == 32 else 8
    alg = algorithmic_bytes_per_launch(n_env, chunk, rs, mean_nw_obs, mean_nw_test, args.mode)
    achieved = alg / (kern_ms * 1e-3) / 1e9
    pmc = latest_pmc(args.precision, args.mode)
    env_steps = world * n_env * steps
    result = {
        "metric": METRIC,
        "value": env_steps / elapsed,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": steps,
        "warmup": warm,
        "ms_per_step": elapsed * 1e3 / steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32" if args.precision == 32 else "f64",
        "data": "synthetic (SURVEY §8(d) routes, island map of test_policy.py:189-194, Philox random IWs)",
        "config": {"workload": "C3: 65 536 ships = 32 768 two-ship envs per GPU, random IW actions, auto-reset",
                   "envs_per_gpu": n_env, "ships_per_gpu": 2 * n_env, "fused_steps_per_launch": chunk,
                   "mode": args.mode, "parallelism": f"env-shard x{world}",
                   "ship_steps_per_s": 2 * env_steps / elapsed,
                   "rccl_transition_gather": bool(gather.enabled), "transitions_compacted": gather.total},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS,
                     "traffic": (pmc["hbm_bytes_per_launch"] if pmc else None),
                     "kernel": "k_env_steps", "kernel_ms_per_launch": kern_ms,
                     "algorithmic_bytes_per_launch": alg,
                     "algorithmic_bytes_per_env_step": alg / (n_env * chunk)},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(args.cpu_baseline_seconds, args.seed)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
