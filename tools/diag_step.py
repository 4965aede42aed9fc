#!/usr/bin/env python3
"""Where a single-step launch (sit_step, K = 1: the drop-in MultiShipRLEnv.step path) spends its time,
from a -DSIT_DIAG_PHASES build (diagnostic, never shipped):

    tools/build_variant.py phases -DSIT_DIAG_PHASES
    SIT_LIBRARY=build_diag/libsit_phases.so python tools/diag_step.py

Runs bench.py --mode step's workload (f32, 32768 envs, explicit random IWs, one launch per step) and
prints, per ship type, the mean shader cycles per wave of the prologue (constants, state, route leg,
map pointers), the step and the epilogue (state write-back), and, for the last launch, the realtime
spread of the waves' starts and ends (100 MHz ticks) against the launch's first start -> last end."""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sac_maritime_ast_amd import VecMultiShipRLEnv, _lib, make_scenario  # noqa: E402

PHASES = ["own ship", "boundary distance", "hull test", "IW test, rest, exchange", "barrier", "env level",
          "auto reset"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n-env", type=int, default=32768)
    ap.add_argument("--launches", type=int, default=200)
    args = ap.parse_args()
    n = args.n_env
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.sit_diag_read_f32.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 64)()
    env = VecMultiShipRLEnv(scenario=make_scenario(n, cap=48), precision=32, device="cuda:0")
    env.reset()
    env.init_step()
    g = torch.Generator(device="cuda:0").manual_seed(1)
    st = env.get_state()
    act = torch.stack([st["north"][1], st["east"][1]], 1) + torch.randn(n, 2, device="cuda:0", generator=g) * 500
    sac = (torch.rand(n, device="cuda:0", generator=g) < 0.005).to(torch.uint8)
    init = torch.zeros(n, dtype=torch.uint8, device="cuda:0")
    for _ in range(200):
        env.step(act, sac, init)
    torch.cuda.synchronize()
    assert lib.sit_diag_read_f32(buf, 1) == 0
    for _ in range(args.launches):
        env.step(act, sac, init)
    torch.cuda.synchronize()
    assert lib.sit_diag_read_f32(buf, 1) == 0
    c = np.array(buf[:], dtype=np.float64).reshape(2, 32)
    env.step(act, sac, init)                      # one more launch for the start / end spread
    torch.cuda.synchronize()
    assert lib.sit_diag_read_f32(buf, 1) == 0
    c1 = np.array(buf[:], dtype=np.float64).reshape(2, 32)
    waves = args.launches * ((n + 63) // 64)
    out = {"kernel": env.lib.sit_step_kernel(env.handle).decode(), "n_env": n, "launches": args.launches}
    for t, name in enumerate(("test ship", "obstacle ship")):
        out[name] = {"mean wave cycles": c[t, 24] / waves, "max wave cycles": c[t, 25],
                     "prologue": c[t, 26] / waves, "epilogue": c[t, 27] / waves,
                     "step phases": {nm: c[t, 16 + k] / waves for k, nm in enumerate(PHASES)}}
    out["last launch ns"] = {"start spread": (c1[:, 29].max() - c1[:, 28].min()) * 10,
                             "end spread": (c1[:, 31].max() - c1[:, 30].min()) * 10,
                             "first start -> last end": (c1[:, 31].max() - c1[:, 28].min()) * 10}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
