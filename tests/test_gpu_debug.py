"""The bounds-checked debug variant of the library (libsit_debug.so, -DSIT_DEBUG; SURVEY §5 "bounds
asserts in a debug kernel variant"): every table index the step kernels compute is checked before
use (route rows, waypoint index, route length, spatial-index entries, edge ids, class-grid words,
mixed-cell records), and the in-kernel serving pass its published row count, served env ids and
LDS extents.  The workload of every kernel variant runs under it with no check failing; a
deliberately corrupted waypoint index and route length are reported (and clamped, so nothing is read
out of bounds).  The debug library runs in a child process (SIT_LIBRARY) so that this test session
keeps the release library."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEBUG_LIB = os.path.join(ROOT, "sac_maritime_ast_amd", "libsit_debug.so")

WORKLOAD = r'''
import json, sys
import numpy as np
import torch
sys.path.insert(0, sys.argv[1])
from sac_maritime_ast_amd import VecMultiShipRLEnv, _lib, make_scenario
from sac_maritime_ast_amd.samplers import GaussianPolicy, PolicySampler
lib = _lib.load()
flags = _lib.ctypes.c_uint32()
def read():
    _lib.check(lib.sit_debug_flags(_lib.ctypes.byref(flags)))
    return int(flags.value)
res = {"debug_build": int(lib.sit_debug_build())}
read()
# float32 synthetic sampler with auto-reset (k_env_steps_sync), replay transitions
env = VecMultiShipRLEnv(scenario=make_scenario(4096, cap=48), precision=32, device="cuda:0")
env.reset(); env.init_step()
for _ in range(3):
    env.rollout(1000, seed=5, transition_capacity=4096 * 8)
res["f32_sync"] = read()
# float64 trajectory log (k_env_steps with the log), explicit sit_step, map probes
e64 = VecMultiShipRLEnv(scenario=make_scenario(512, cap=16), precision=64, device="cuda:0")
e64.reset(); e64.init_step()
e64.rollout(800, seed=6, log=True)
st = e64.get_state()
a = torch.stack([st["north"][1] + 400.0, st["east"][1]], 1)
for i in range(20):
    e64.step(a, torch.ones(512, dtype=torch.uint8), torch.full((512,), int(i == 0), dtype=torch.uint8))
pts = torch.rand((100000, 2), dtype=torch.float64, device="cuda:0") * 12000 - 1000
e64.probe_map(pts)
res["f64_log_step_probe"] = read()
# policy mode (k_env_steps_sync<kPolicy>) with the fused actor
torch.manual_seed(0)
sm = PolicySampler(env, GaussianPolicy().to("cuda:0"), chunk=64, request_capacity=1024)
for _ in range(30):
    sm.launch()
res["f32_policy"] = read()
# policy mode with in-kernel serving (csrc/sit_serve.h: published rows, served env ids, the serving LDS)
# on ragged populations (a partial last block), float32 and float64
for prec, n_r in ((32, 4096 - 37), (64, 512 - 5)):
    er = VecMultiShipRLEnv(scenario=make_scenario(n_r, cap=48), precision=prec, device="cuda:0")
    er.reset(); er.init_step()
    sk = PolicySampler(er, GaussianPolicy().to("cuda:0"), chunk=64, serve="kernel")
    for _ in range(30):
        sk.launch()
    torch.cuda.synchronize()
    res[f"f{prec}_policy_serve"] = read()
    res[f"f{prec}_policy_serve_kernel"] = er.lib.sit_step_kernel(er.handle).decode()
    res[f"f{prec}_served"] = int(sk.served.item())
# corrupted state: the checks fire and clamp (no out-of-bounds access)
st = env.get_state()
st["next_wpt"][1, 0] = 999
env.set_state({"next_wpt": st["next_wpt"]})
env.rollout(1, seed=7)
res["bad_waypoint"] = read()
st = env.get_state()
st["n_wpt"][0, 1] = 1000
env.set_state({"n_wpt": st["n_wpt"]})
env.rollout(1, seed=7)
res["bad_route_len"] = read()
torch.cuda.synchronize()
print(json.dumps(res))
'''


def test_debug_variant_checks_every_kernel():
    if not os.path.exists(DEBUG_LIB):
        pytest.fail("libsit_debug.so is missing: __graft_entry__.build() builds it")
    env = dict(os.environ, SIT_LIBRARY=DEBUG_LIB)
    p = subprocess.run([sys.executable, "-c", WORKLOAD, ROOT], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    print("debug variant:", res)
    assert res["debug_build"] == 1
    for k in ("f32_sync", "f64_log_step_probe", "f32_policy", "f32_policy_serve", "f64_policy_serve"):
        assert res[k] == 0, f"{k}: bounds checks failed: {res[k]:#x}"
    for prec in (32, 64):   # the serving pass ran (inside the sync kernel) and served envs
        assert "k_env_steps_sync" in res[f"f{prec}_policy_serve_kernel"], res
        assert res[f"f{prec}_served"] > 0, res
    assert res["bad_waypoint"] & (1 << 1), res          # kDbgWaypoint
    assert res["bad_route_len"] & (1 << 2), res         # kDbgRouteLen
