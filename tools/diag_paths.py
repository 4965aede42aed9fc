"""Predicate path statistics from a SIT_DIAG_PATHS build (diagnostic, never shipped).

    SIT_LIBRARY=build_diag/libsit_diag.so python tools/diag_paths.py [--launches 10]

Runs the bench workload (f32, 32768 envs, fused 200-step rollouts, synthetic sampler) and
prints, per ship type, lane- and wave-level counts of the predicate paths (-DSIT_DIAG_PATHS
build) and/or shader-clock cycles per step phase (-DSIT_DIAG_PHASES build)."""
import argparse
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sac_maritime_ast_amd import VecMultiShipRLEnv, make_scenario  # noqa: E402
from sac_maritime_ast_amd import _lib  # noqa: E402

NAMES = ["dist candidates (lane sum)", "near-shore lanes", "pair scans (lanes)", "hull band trips (lane sum)",
         "mixed far centre (lanes)", "mixed IW (lanes)", "IW band trips (lane sum)", "wave-steps",
         "max dist candidates (wave sum)", "waves with near-shore lane", "waves with pair scan",
         "max hull band trips (wave sum)", "waves with mixed far centre", "waves with mixed IW",
         "max IW band trips (wave sum)"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-env", type=int, default=32768)
    ap.add_argument("--launches", type=int, default=10)
    ap.add_argument("--chunk", type=int, default=200)
    args = ap.parse_args()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.sit_diag_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 64)()
    env = VecMultiShipRLEnv(scenario=make_scenario(args.n_env), precision=32, device="cuda:0")
    env.reset()
    env.init_step()
    env.rollout(args.chunk, seed=25450)          # warm-up launch
    assert lib.sit_diag_read(buf, 1) == 0
    for _ in range(args.launches):
        env.rollout(args.chunk, seed=25450)
    torch.cuda.synchronize()
    assert lib.sit_diag_read(buf, 1) == 0
    c = np.array(buf[:], dtype=np.float64).reshape(2, 32)
    phases = ["own ship (sampler, guidance, dynamics)", "boundary distance", "hull test",
              "IW test, rest, exchange writes", "barrier", "env level (reward, outputs)", "auto reset"]
    wave_steps = args.launches * args.chunk * ((args.n_env + 63) // 64)
    if c[:, 16:23].sum() > 0:
        for t, name in enumerate(("test ship", "obstacle ship")):
            tot = c[t, 16:23].sum()
            print(f"--- {name}: shader-clock cycles per wave-step (total {tot / wave_steps:.0f})")
            for k, nm in enumerate(phases):
                print(f"  {nm:40s} {c[t, 16 + k] / wave_steps:10.1f}  {100 * c[t, 16 + k] / tot:5.1f}%")
    for t, name in enumerate(("test ship", "obstacle ship")):
        ws = c[t, 7]
        if ws == 0:
            continue
        lanes = ws * 64
        print(f"--- {name}: {int(ws)} wave-steps")
        for j, nm in enumerate(NAMES[:15]):
            if j == 7:
                continue
            per = c[t, j] / (lanes if j < 7 else ws)
            print(f"  {nm:34s} {c[t, j]:14.0f}  per {'lane' if j < 7 else 'wave'}-step {per:.4f}")


if __name__ == "__main__":
    main()
