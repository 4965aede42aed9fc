#!/usr/bin/env python3
"""Cycles per role and loop segment of k_env_steps_sync from a -DSIT_DIAG_SYNC build (diagnostic,
never shipped):

    tools/build_variant.py diagsync -DSIT_DIAG_SYNC
    SIT_LIBRARY=build_diag/libsit_diagsync.so python tools/diag_sync.py [--policy]

Runs the bench workload (f32, 32768 envs, synthetic sampler, auto-reset; --policy: one group in policy
mode with the fused actor) and prints, per role (D0 test-ship dynamics, D1 obstacle dynamics, P0 / P1
their position predicates and outputs), shader cycles per wave-step: work before barrier A, the wait
at A, work A -> B, the wait at B, work after B.  The s_memtime stamps cost ~10 % themselves."""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sac_maritime_ast_amd import VecMultiShipRLEnv, _lib, make_scenario  # noqa: E402

SEGS = ["work before A", "wait A", "work A->B", "wait B", "work after B"]
EXTRA = {6: "of which outputs up to the row stores", 7: "of which outputs after the stores"}
ROLES = ["D0 test dynamics", "D1 obstacle dynamics", "P0 test predicates+outputs", "P1 obstacle predicates"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-env", type=int, default=32768)
    ap.add_argument("--chunk", type=int, default=2000)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--policy", action="store_true")
    args = ap.parse_args()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.sit_diag_read_f32.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 64)()
    env = VecMultiShipRLEnv(scenario=make_scenario(args.n_env, cap=48), precision=32, device="cuda:0")
    env.reset()
    env.init_step()
    if args.policy:
        from sac_maritime_ast_amd.samplers import GaussianPolicy, PolicySampler
        torch.manual_seed(0)
        sm = PolicySampler(env, GaussianPolicy().to("cuda:0"), chunk=64, request_capacity=args.n_env // 4)
        run = sm.launch
        for _ in range(600):
            run()
    else:
        def run():
            env.rollout(args.chunk, seed=25450)
        for _ in range(max(1, 40000 // args.chunk)):
            run()
    assert lib.sit_diag_read_f32(buf, 1) == 0
    for _ in range(args.launches if not args.policy else 200):
        run()
    torch.cuda.synchronize()
    assert lib.sit_diag_read_f32(buf, 0) == 0
    c = np.array(buf[:], dtype=np.float64).reshape(2, 32)
    out = {"kernel": env.lib.sit_step_kernel(env.handle).decode(), "roles": {}}
    for r, name in enumerate(ROLES):
        row = c[r >> 1, (r & 1) * 8:(r & 1) * 8 + 8]
        steps = max(row[5], 1.0)
        # segments 6 and 7 (P0's outputs of the previous step) are stamped inside segment 2
        seg = row.copy()
        seg[2] += seg[6] + seg[7]
        out["roles"][name] = {s_: round(seg[i] / steps, 1) for i, s_ in enumerate(SEGS)}
        for k in (6, 7):
            if seg[k]:
                out["roles"][name][EXTRA[k]] = round(seg[k] / steps, 1)
        out["roles"][name]["total"] = round(seg[:5].sum() / steps, 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
