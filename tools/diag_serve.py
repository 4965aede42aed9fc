#!/usr/bin/env python3
"""Cycles per phase of the in-kernel serving pass (sit_serve.h) from a -DSIT_DIAG_SERVE build
(diagnostic, never shipped):

    tools/build_variant.py diagserve -DSIT_DIAG_SERVE
    SIT_LIBRARY=build_diag/libsit_diagserve.so python tools/diag_serve.py [--chunk 80]

Runs the C5 workload (f32, 32768 envs in one group, policy mode with the fused actor served at the end of
each launch) and prints the passes per launch and block by their row count, the mean duration of a pass
(s_memrealtime, 100 MHz) and the launch time from host events."""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sac_maritime_ast_amd import VecMultiShipRLEnv, _lib, make_scenario  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-env", type=int, default=32768)
    ap.add_argument("--chunk", type=int, default=80)
    ap.add_argument("--warmup", type=int, default=600)
    ap.add_argument("--launches", type=int, default=200)
    args = ap.parse_args()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.sit_diag_read_f32.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 64)()
    env = VecMultiShipRLEnv(scenario=make_scenario(args.n_env, cap=48), precision=32, device="cuda:0")
    env.reset()
    env.init_step()
    from sac_maritime_ast_amd.samplers import GaussianPolicy, PolicySampler
    torch.manual_seed(0)
    sm = PolicySampler(env, GaussianPolicy().to("cuda:0"), chunk=args.chunk)
    for _ in range(args.warmup):
        sm.launch()
    torch.cuda.synchronize()
    assert lib.sit_diag_read_f32(buf, 1) == 0
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.launches):
        sm.launch()
    e1.record()
    torch.cuda.synchronize()
    assert lib.sit_diag_read_f32(buf, 0) == 0
    c = np.array(buf[:], dtype=np.float64).reshape(2, 32)
    passes = {4 * k: int(c[1, k]) for k in range(1, 5) if c[1, k]}
    n_pass = max(sum(passes.values()), 1)
    blocks = args.launches * ((args.n_env + 63) // 64)
    out = {"kernel": env.lib.sit_step_kernel(env.handle).decode(), "chunk": args.chunk, "launches": args.launches,
           "passes_by_rows": passes, "passes_per_block_launch": n_pass / blocks,
           "rows_per_block_launch_upper": sum(r * n for r, n in passes.items()) / blocks}
    out["pass_us_realtime"] = round(c[1, 9] / n_pass / 100.0, 3)       # s_memrealtime runs at 100 MHz
    out["memtime_ticks_per_us"] = round(c[1, 8] / max(c[1, 9], 1) * 100.0, 1)
    out["us_per_launch_host_events"] = round(e0.elapsed_time(e1) * 1e3 / args.launches, 2)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
