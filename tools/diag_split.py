"""Per-role phase cycles of the pipelined step kernel from a SIT_DIAG_SPLIT build (diagnostic only).

    SIT_LIBRARY=build_diag/libsit_dsplit.so python tools/diag_split.py

Runs the bench workload (f32, 32768 envs, synthetic sampler) and prints shader cycles per
wave-step of each role's phases, the redo rate, and how the block's waves sat on the SIMDs."""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sac_maritime_ast_amd import VecMultiShipRLEnv, make_scenario  # noqa: E402
from sac_maritime_ast_amd import _lib  # noqa: E402

PH = {0: ["step (pass 0)", "wait A", "redo", "wait B", "env level + reset", "redo wave-steps", "-", "-"],
      2: ["outputs (P0)", "predicates", "wait A", "wait B", "-", "-", "-", "-"]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-env", type=int, default=32768)
    ap.add_argument("--launches", type=int, default=5)
    ap.add_argument("--chunk", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=40000)
    args = ap.parse_args()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.sit_diag_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 64)()
    env = VecMultiShipRLEnv(scenario=make_scenario(args.n_env, cap=48), precision=32, device="cuda:0")
    env.reset()
    env.init_step()
    for _ in range(max(1, args.warmup // args.chunk)):
        env.rollout(args.chunk, seed=25450)
    torch.cuda.synchronize()
    assert lib.sit_diag_read(buf, 1) == 0
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(args.launches):
        env.rollout(args.chunk, seed=25450)
    ev[1].record()
    torch.cuda.synchronize()
    assert lib.sit_diag_read(buf, 1) == 0
    c = np.array(buf[:], dtype=np.float64).reshape(2, 32)
    waves_per_role = 2 * ((args.n_env + 127) // 128)
    ws = waves_per_role * (args.chunk + 2) * args.launches
    print(f"{args.launches} launches x {args.chunk} steps: {ev[0].elapsed_time(ev[1]) / args.launches:.3f} ms per launch")
    for role, name in enumerate(["D0 test", "D1 obstacle", "P0 test", "P1 obstacle"]):
        row = c[role >> 1, (role & 1) * 8:(role & 1) * 8 + 8]
        names = PH[0 if role < 2 else 2]
        parts = [f"{names[q]} {row[q] / ws:.0f}" for q in range(8) if names[q] != "-" and q != 5]
        extra = f"  redo wave-step fraction {row[5] / ws:.4f}" if role < 2 else ""
        print(f"{name:12s} cycles/wave-step: " + ", ".join(parts) + f"  total {row[[q for q in range(8) if q != 5]].sum() / ws:.0f}" + extra)
    print(f"blocks with one D and one P wave per SIMD: {c[1, 16]:.0f} of {c[1, 17]:.0f}; "
          f"mean SIMD id per wave slot: {np.round(c[1, 18:26] / max(c[1, 17], 1), 2).tolist()}")


if __name__ == "__main__":
    main()
