#!/usr/bin/env python3
"""Standalone timing of sit_policy_actor (no env kernel running beside it): request rows filled
synthetically; 20 launches captured in a HIP graph, HIP events around each replay (run it under
rocprofv3 --kernel-trace --stats for per-kernel durations)."""
import sys

import torch

sys.path.insert(0, ".")
from sac_maritime_ast_amd import VecMultiShipRLEnv, make_scenario  # noqa: E402
from sac_maritime_ast_amd.samplers import GaussianPolicy, PolicySampler  # noqa: E402

dev = "cuda:0"
env = VecMultiShipRLEnv(scenario=make_scenario(16384, cap=48), precision=32, device=dev)
torch.manual_seed(0)
pol = GaussianPolicy(hidden=(256, 256)).to(dev)
sm = PolicySampler(env, pol, chunk=32, request_capacity=4096)
io = sm.io
io["request_obs"].normal_()
io["request_noise"].normal_()
io["request_env"].copy_(torch.randperm(16384, device=dev)[:4096].int())
import ctypes  # noqa: E402
counts = {}
variant = sys.argv[1] if len(sys.argv) > 1 else "fused"
for count in (8, 256, 1400, 4096):
    counts[count] = torch.full((1,), count, dtype=torch.int32, device=dev)
if variant == "noatomics":      # the kernel without the served / count-reset atomics
    def act():
        env._call("sit_policy_actor", 4096, sm._w.data_ptr(), io["request_obs"].data_ptr(),
                  io["request_noise"].data_ptr(), io["request_env"].data_ptr(), io["request_count"].data_ptr(), 0,
                  io["policy_action"].data_ptr(), io["policy_ready"].data_ptr(), None, None, env._stream())
    sm.act = act
elif variant == "torch":        # the unfused path (PyTorch GEMMs + sit_policy_apply)
    sm._w = None
for count in (8, 256, 1400, 4096):
    g = torch.cuda.CUDAGraph()
    io["request_count"].fill_(count)
    sm.act()
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(20):
            io["request_count"].copy_(counts[count])
            sm.act()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for it in range(20):
        ev[0].record()
        g.replay()
        ev[1].record()
        torch.cuda.synchronize()
        ts.append(ev[0].elapsed_time(ev[1]) * 1e3 / 20)
    ts.sort()
    flops = count * 2 * (10 * 256 + 256 * 256 + 256 * 2)
    print(f"rows {count}: median {ts[len(ts) // 2]:.2f} us per act (incl. a 1-element copy), min {ts[0]:.2f} us, "
          f"{flops / (ts[len(ts) // 2] * 1e-6) / 1e12:.2f} TFLOP/s")
