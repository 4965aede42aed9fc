#!/usr/bin/env python3
"""How often the fused step kernel's blocks find their four waves on fewer than four SIMDs
(sit_role_fallbacks) in the bench's own launch shapes: C3 (synthetic sampler, 40 000-step launches)
and C5 (policy mode with in-kernel serving, 64-step launches in HIP-graph replays).  Prints JSON."""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sac_maritime_ast_amd import VecMultiShipRLEnv, _lib, make_scenario  # noqa: E402
from sac_maritime_ast_amd.samplers import GaussianPolicy, PolicySampler  # noqa: E402

lib = _lib.load()
c = ctypes.c_uint64()


def fallbacks():
    _lib.check(lib.sit_role_fallbacks(ctypes.byref(c), 1))
    return int(c.value)


n = 32768
res = {"blocks_per_launch": n // 64}
env = VecMultiShipRLEnv(scenario=make_scenario(n, cap=48), precision=32, device="cuda:0")
env.reset()
env.init_step()
fallbacks()
for _ in range(3):
    env.rollout(4000, seed=3, want=("reward",))
res["c3_launches"] = 3
res["c3_fallback_blocks"] = fallbacks()
torch.manual_seed(0)
env5 = VecMultiShipRLEnv(scenario=make_scenario(n, cap=48), precision=32, device="cuda:0")
env5.reset()
env5.init_step()
sm = PolicySampler(env5, GaussianPolicy().to("cuda:0"), chunk=64, serve="kernel")
for _ in range(40):
    sm.launch()
torch.cuda.synchronize()
fallbacks()
sm.capture(16)
for _ in range(4):
    sm.replay()
torch.cuda.synchronize()
res["c5_launches"] = 64
res["c5_fallback_blocks"] = fallbacks()
print(json.dumps(res))
