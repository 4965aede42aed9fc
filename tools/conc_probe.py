#!/usr/bin/env python3
"""Config C5 throughput of in-kernel serving by chunk length, eager launches, one GPU (the concurrent
server of commit 14a3fac took serve="concurrent"):
   python tools/conc_probe.py [--n-env 32768] [--chunks 64,256,1024] [--seconds 2]
Prints env-steps/s, env_step_fraction and the server's counters per (serve, chunk)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from sac_maritime_ast_amd import VecMultiShipRLEnv, make_scenario  # noqa: E402
from sac_maritime_ast_amd.samplers import GaussianPolicy, PolicySampler  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--n-env", type=int, default=32768)
ap.add_argument("--chunks", default="64,256,1024")
ap.add_argument("--serves", default="kernel")
ap.add_argument("--seconds", type=float, default=2.0)
ap.add_argument("--warm-steps", type=int, default=30720)
args = ap.parse_args()
dev = torch.device("cuda:0")
torch.manual_seed(0)
policy = GaussianPolicy(hidden=(256, 256)).to(dev)
res = []
for serve in args.serves.split(","):
    for chunk in (int(c) for c in args.chunks.split(",")):
        env = VecMultiShipRLEnv(scenario=make_scenario(args.n_env, cap=48, seed=25450), precision=32, device=dev)
        env.reset()
        env.init_step()
        sm = PolicySampler(env, policy, chunk=chunk, seed=25450, serve=serve)
        want = ("reward", "done", "status")
        for _ in range(max(2, args.warm_steps // chunk)):
            sm.launch(want)
        torch.cuda.synchronize()
        s0 = int(sm.env_steps.item())
        t0 = time.perf_counter()
        n_l = 0
        while True:
            sm.launch(want)
            n_l += 1
            if n_l % 8 == 0:
                torch.cuda.synchronize()
                if time.perf_counter() - t0 > args.seconds:
                    break
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        steps = int(sm.env_steps.item()) - s0
        r = {"serve": serve, "chunk": chunk, "env_steps_per_s": steps / dt,
             "env_step_fraction": steps / (args.n_env * chunk * n_l), "launches": n_l,
             "ms_per_launch": 1e3 * dt / n_l}
        print(json.dumps(r), flush=True)
        res.append(r)
        del sm, env
        torch.cuda.empty_cache()
