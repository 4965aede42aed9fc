#!/usr/bin/env python3
"""Cycles per role and loop segment of k_env_steps_sync from a -DSIT_DIAG_SYNC build (diagnostic,
never shipped):

    tools/build_variant.py diagsync -DSIT_DIAG_SYNC
    SIT_LIBRARY=build_diag/libsit_diagsync.so python tools/diag_sync.py [--policy]

Runs the bench workload (f32, 32768 envs, synthetic sampler, auto-reset; --policy: one group in policy
mode with the fused actor served in the step kernel, 64 steps per launch; --queue: on the request queue)
and prints, per role (D0 test-ship dynamics, D1 obstacle dynamics, P0 / P1
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
# (The marks pin instruction order inside a basic block only: the compiler still moves work across
# block boundaries — round 5 found the next heading's sincos and dynamics tail after D1's mark 9, so the
# sub-segment D1 6 ("travelled distance") holds them too.  The five segments are exact.)
# sub-segments (part of the segment named first): D 10 = sincos + Euler position (before A), 8 = guidance
# and control, 9 = machinery and kinetics (A->B), 11 = the episode-end decision (after B, the rest is the
# reset); P 8 = cell record + first edge group issued, 9 = boundary distance, 10 = hull test (A->B);
# P0 6 / 7 = the previous step's outputs up to the row stores / after them (A->B)
SUB = {"D": {10: ("work before A", "Euler position"), 8: ("work A->B", "dynamics base + guidance + control"),
             9: ("work A->B", "machinery + kinetics + next heading trig"),
             6: ("work A->B", "D1: travelled distance (or the stop path)"),
             7: ("work A->B", "D1: navigation test + publishing the step"),
             14: ("work A->B", "D1: the next event's draw (synthetic sampler)"),
             11: ("work after B", "episode-end decision")},
       "P": {6: ("work A->B", "P0 outputs up to the row stores"), 7: ("work A->B", "P0 outputs after the stores"),
             8: ("work A->B", "cell record + first edges"), 9: ("work A->B", "boundary distance"),
             10: ("work A->B", "hull test"), 11: ("work A->B", "IW test (P1) / collision (P0)")}}
ONCE = {12: "prologue (per launch)", 13: "epilogue (per launch)", 14: "barrier D + in-kernel serving (per launch)",
        15: "kernel start to the staged map (per launch)"}
ROLES = ["D0 test dynamics", "D1 obstacle dynamics", "P0 test predicates+outputs", "P1 obstacle predicates"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-env", type=int, default=32768)
    ap.add_argument("--chunk", type=int, default=2000)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--policy", action="store_true")
    ap.add_argument("--queue", action="store_true", help="--policy on the request queue (capacity n/4)")
    ap.add_argument("--policy-chunk", type=int, default=64)
    ap.add_argument("--step", action="store_true", help="explicit actions, one launch per step (sit_step)")
    args = ap.parse_args()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.sit_diag_read_f32.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 64)()
    env = VecMultiShipRLEnv(scenario=make_scenario(args.n_env, cap=48), precision=32, device="cuda:0")
    env.reset()
    env.init_step()
    if args.step:
        g = torch.Generator(device="cuda:0").manual_seed(1)
        st = env.get_state()
        act = torch.stack([st["north"][1], st["east"][1]], 1) + torch.randn(args.n_env, 2, device="cuda:0", generator=g) * 500
        sac = (torch.rand(args.n_env, device="cuda:0", generator=g) < 0.005).to(torch.uint8)
        init = torch.zeros(args.n_env, dtype=torch.uint8, device="cuda:0")

        def run():
            env.step(act, sac, init)
        for _ in range(200):
            run()
    elif args.policy:
        from sac_maritime_ast_amd.samplers import GaussianPolicy, PolicySampler
        torch.manual_seed(0)
        sm = PolicySampler(env, GaussianPolicy().to("cuda:0"), chunk=args.policy_chunk,
                           request_capacity=args.n_env // 4 if args.queue else None)
        run = sm.launch
        for _ in range(600):
            run()
    else:
        def run():
            env.rollout(args.chunk, seed=25450)
        for _ in range(max(1, 40000 // args.chunk)):
            run()
    assert lib.sit_diag_read_f32(buf, 1) == 0
    for _ in range(args.launches if not (args.policy or args.step) else 200):
        run()
    torch.cuda.synchronize()
    assert lib.sit_diag_read_f32(buf, 0) == 0
    c = np.array(buf[:], dtype=np.float64).reshape(2, 32)
    out = {"kernel": env.lib.sit_step_kernel(env.handle).decode(), "roles": {}}
    for r, name in enumerate(ROLES):
        row = c[r >> 1, (r & 1) * 16:(r & 1) * 16 + 16]
        steps = max(row[5], 1.0)
        sub = SUB[name[0]]
        seg = {s_: row[i] for i, s_ in enumerate(SEGS)}
        for k, (parent, _) in sub.items():      # a sub-segment's cycles belong to its parent segment
            seg[parent] += row[k]
        res = {s_: round(v / steps, 1) for s_, v in seg.items()}
        for k, (parent, label) in sorted(sub.items()):
            if row[k]:
                res[f"  {parent}: {label}"] = round(row[k] / steps, 1)
        res["total"] = round(sum(seg.values()) / steps, 1)
        launches = max(1, args.launches if not (args.policy or args.step) else 200)
        waves = launches * ((args.n_env + 63) // 64)
        for k, label in ONCE.items():   # per wave and launch
            if k not in sub or args.policy:
                res[label] = round(row[k] / waves, 1)
        out["roles"][name] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
