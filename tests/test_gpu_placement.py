"""Placement independence of the fused two-wave step kernel (k_env_steps_sync, csrc/sit_sync.h).

Each wave of a fused launch takes its role (D0, D1, P0, P1) from the rank of its (HW_ID SIMD, wave
index) among the block's four (sync_role_of, csrc/sit_device.h): a permutation of the four roles
for every placement, equal to the SIMD when the four waves sit on four SIMDs.  Checked three ways:
* the role function itself over all 4^4 SIMD assignments x both CU tickets, in both translation
  units (sit_selftest_f64 op 8): always a permutation, and the SIMD itself (^ the mirror for the
  second block of a CU) when the SIMDs differ;
* the real kernel with shared-SIMD placements forced (the SIT_TEST_FAKE_SIMDS hook: the waves report
  a given SIMD assignment instead of HW_ID) against the same launch with the hardware's placement:
  rows and state bit for bit, and the fallback counter (sit_role_fallbacks) counts every block;
* a C3-shaped launch beside a kernel that holds wave slots and registers on every CU on another
  stream (tests/csrc/sit_occupy.hip), against a solo run: rows and state bit for bit.  How many
  blocks then found their waves on shared SIMDs is recorded (it depends on the hardware's dispatch).
"""
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest
import torch

from sac_maritime_ast_amd import VecMultiShipRLEnv, _lib, make_scenario

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OCCUPY_LIB = os.path.join(ROOT, "tests", "libsit_occupy.so")
MIRROR = 2     # SIT_SIMD_MIRROR


def _roles(packed):
    return [(packed >> (2 * v)) & 3 for v in range(4)]


@pytest.mark.parametrize("fast_tu", [0, 1])
def test_role_function_is_a_permutation_for_every_placement(fast_tu):
    lib = _lib.load()
    assign = np.repeat(np.arange(256, dtype=np.float64), 2)
    ticket = np.tile(np.array([0.0, 1.0]), 256)
    a = torch.tensor(assign, device="cuda:0")
    b = torch.tensor(ticket, device="cuda:0")
    out = torch.empty_like(a)
    _lib.check(lib.sit_selftest_f64(8, len(assign), a.data_ptr(), b.data_ptr(), out.data_ptr(), fast_tu, None))
    torch.cuda.synchronize()
    got = out.cpu().numpy().astype(np.int64)
    n_dup = 0
    for s, tk, p in zip(assign.astype(int), ticket.astype(int), got):
        simd = [(s >> (2 * v)) & 3 for v in range(4)]
        roles = _roles(int(p))
        assert sorted(roles) == [0, 1, 2, 3], (simd, tk, roles)
        if len(set(simd)) == 4:
            assert roles == [x ^ (MIRROR if tk else 0) for x in simd], (simd, tk, roles)
        else:
            n_dup += 1
    assert n_dup == 2 * (256 - 24)


def _c3_env(n, warm):
    env = VecMultiShipRLEnv(scenario=make_scenario(n, cap=48), precision=32, device="cuda:0")
    env.reset()
    env.init_step()
    if warm:
        env.rollout(warm, seed=11, want=("reward",))      # desynchronised episodes (different phases per env)
    torch.cuda.synchronize()
    return env


def _run(env, blob, k, seed):
    env.load_state_blob(blob)
    out = env.rollout(k, seed=seed, want=("next_state", "reward", "done", "status", "action"))
    return out, env.state_blob()


def _bits(t):
    """Bit patterns of a tensor (the action rows hold NaN where no sample was taken: NaN != NaN)."""
    if t.is_floating_point():
        return t.contiguous().view(torch.int32 if t.dtype == torch.float32 else torch.int64)
    return t


def _same(a, b):
    (oa, sa), (ob, sb) = a, b
    for key in oa:
        assert torch.equal(_bits(oa[key]), _bits(ob[key])), key
    assert torch.equal(sa, sb), "state"


# the child process: a handle created with SIT_TEST_FAKE_SIMDS set runs the same launch as one without
_FAKE = r'''
import json, sys, torch
sys.path.insert(0, sys.argv[1])
from sac_maritime_ast_amd import VecMultiShipRLEnv, _lib, make_scenario
lib = _lib.load()
n = 4096
env = VecMultiShipRLEnv(scenario=make_scenario(n, cap=48), precision=int(sys.argv[2]), device="cuda:0")
env.reset(); env.init_step()
env.rollout(300, seed=3, want=("reward",))
blob = env.state_blob()
out = env.rollout(64, seed=4, want=("next_state", "reward", "done", "status", "action"))
torch.cuda.synchronize()
c = _lib.ctypes.c_uint64()
_lib.check(lib.sit_role_fallbacks(_lib.ctypes.byref(c), 1))
res = {k: v.cpu() for k, v in out.items()}
res["state"] = env.state_blob().cpu()
torch.save(res, sys.argv[3])
print(json.dumps({"fallbacks": int(c.value), "kernel": env.lib.sit_step_kernel(env.handle).decode()}))
'''


@pytest.mark.parametrize("precision", [32, 64])
def test_forced_shared_simd_placements_give_identical_results(precision, tmp_path):
    """Placements the hardware rarely produces, forced: all four waves on one SIMD (roles by wave
    index), two pairs of waves sharing two SIMDs, three on one SIMD.  Every one runs each role exactly
    once per block, so rows and state equal the hardware placement's bit for bit."""
    runs = {}
    for tag, fake in (("hw", None), ("one_simd", 0), ("two_pairs", 0b01010000), ("three_one", 0b11000000),
                      ("reversed_dup", 0b00011011 ^ 0b00000011)):
        env = dict(os.environ)
        env.pop("SIT_TEST_FAKE_SIMDS", None)
        if fake is not None:
            env["SIT_TEST_FAKE_SIMDS"] = str(fake)
        path = str(tmp_path / f"{tag}.pt")
        p = subprocess.run([sys.executable, "-c", _FAKE, ROOT, str(precision), path], env=env, capture_output=True,
                           text=True, timeout=240)
        assert p.returncode == 0, p.stderr[-3000:]
        info = json.loads(p.stdout.strip().splitlines()[-1])
        assert "k_env_steps_sync" in info["kernel"] and "map=LDS" in info["kernel"], info
        runs[tag] = (torch.load(path, weights_only=True), info)
    ref, _ = runs["hw"]
    n_blocks = 4096 // 64
    for tag, (res, info) in runs.items():
        for key in ref:
            assert torch.equal(_bits(res[key]), _bits(ref[key])), (tag, key)
        if tag != "hw":
            # every forced assignment shares a SIMD in every block: each block of both fused launches
            # (the warm-up and the compared one) is counted
            assert info["fallbacks"] == 2 * n_blocks, (tag, info)
        print(tag, info)


def _occupy_lib():
    if not os.path.exists(OCCUPY_LIB):
        pytest.fail("tests/libsit_occupy.so is missing: __graft_entry__.build() builds it")
    lib = ctypes.CDLL(OCCUPY_LIB)
    lib.sit_test_occupy.restype = ctypes.c_int32
    lib.sit_test_occupy.argtypes = [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.c_double, ctypes.c_void_p,
                                    ctypes.c_void_p]
    return lib


def test_c3_launch_beside_cu_occupier_equals_solo_run():
    """A C3-shaped launch (32 768 envs, the benchmarked float32 kernel with the LDS map) while another
    stream's kernel holds wave slots and registers on the CUs, against the same launch alone: rows and
    state bit for bit.  Several occupier shapes (heavy waves reserve 256 VGPRs, so that a SIMD holding
    one has room for one step wave, not two); the occupier must still be running when the step
    launch ends (the two ran concurrently)."""
    occ = _occupy_lib()
    lib = _lib.load()
    n, k = 32768, 200
    env = _c3_env(n, 2000)
    blob = env.state_blob()
    c = ctypes.c_uint64()
    _lib.check(lib.sit_role_fallbacks(ctypes.byref(c), 1))
    solo = _run(env, blob, k, seed=21)
    torch.cuda.synchronize()
    _lib.check(lib.sit_role_fallbacks(ctypes.byref(c), 1))
    record = {"solo_fallback_blocks": int(c.value), "blocks_per_launch": n // 64, "configs": []}
    s_occ = torch.cuda.Stream()
    s_step = torch.cuda.Stream()
    started = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    for blocks, threads, heavy in ((256, 64, 1), (512, 64, 1), (256, 128, 1), (256, 256, 1), (2048, 64, 0),
                                   (768, 64, 1)):
        started.zero_()
        torch.cuda.synchronize()
        with torch.cuda.stream(s_occ):
            assert occ.sit_test_occupy(blocks, threads, heavy, 400.0, ctypes.c_void_p(started.data_ptr()),
                                       ctypes.c_void_p(s_occ.cuda_stream)) == 0
        time.sleep(0.05)                          # the occupier's waves are resident
        t0 = time.perf_counter()
        with torch.cuda.stream(s_step):
            res = _run(env, blob, k, seed=21)
        s_step.synchronize()
        t_step = time.perf_counter() - t0
        concurrent = not s_occ.query()           # the occupier still running when the step ended
        torch.cuda.synchronize()
        _lib.check(lib.sit_role_fallbacks(ctypes.byref(c), 1))
        cfg = {"occupier": {"blocks": blocks, "threads": threads, "heavy": heavy}, "waves_started": int(started.item()),
               "concurrent": concurrent, "step_s": round(t_step, 4), "fallback_blocks": int(c.value)}
        record["configs"].append(cfg)
        print(cfg)
        _same(res, solo)
        assert cfg["waves_started"] == blocks * threads // 64
    # (a shape whose waves leave no room for a step block delays it until the occupier ends; the
    # others run beside it)
    assert sum(c["concurrent"] for c in record["configs"]) >= 3, record
    out = os.environ.get("SIT_PLACEMENT_RECORD")
    if out:
        with open(out, "w") as f:
            json.dump(record, f, indent=1)
