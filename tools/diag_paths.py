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
    ap.add_argument("--warmup", type=int, default=200, help="env steps before the measured launches")
    args = ap.parse_args()
    lib = ctypes.CDLL(_lib.LIB_PATH)
    lib.sit_diag_read.argtypes = [ctypes.POINTER(ctypes.c_ulonglong), ctypes.c_int]
    buf = (ctypes.c_ulonglong * 64)()
    env = VecMultiShipRLEnv(scenario=make_scenario(args.n_env), precision=32, device="cuda:0")
    env.reset()
    env.init_step()
    for _ in range(max(1, args.warmup // args.chunk)):   # warm-up launches (steady state)
        env.rollout(args.chunk, seed=25450)
    assert lib.sit_diag_read(buf, 1) == 0
    for _ in range(args.launches):
        env.rollout(args.chunk, seed=25450)
    torch.cuda.synchronize()
    assert lib.sit_diag_read(buf, 1) == 0
    c = np.array(buf[:], dtype=np.float64).reshape(2, 32)
    env.rollout(args.chunk, seed=25450)           # one more launch for the start/end skew
    assert lib.sit_diag_read(buf, 1) == 0
    c1 = np.array(buf[:], dtype=np.float64).reshape(2, 32)
    c[:, 28:32] = c1[:, 28:32]
    if hasattr(lib, "sit_diag_read_waves"):
        nw = 2 * ((args.n_env + 63) // 64)
        wb = (ctypes.c_ulonglong * (4 * nw))()
        assert lib.sit_diag_read_waves(wb, nw) == 0
        w = np.array(wb[:], dtype=np.uint64).reshape(nw, 4)
        np.save(os.environ.get("SIT_WAVE_DUMP", "gpurun_out/waves.npy"), w)
        t0 = w[:, 0].min()
        dur = (w[:, 1] - w[:, 0]).astype(np.float64) * 10e-3   # us
        hw = w[:, 3] & 0xffffffff
        xcc = (w[:, 3] >> 32).astype(np.int64)
        simd = ((hw >> 4) & 3).astype(np.int64)
        cu = ((hw >> 8) & 15).astype(np.int64)
        sh = ((hw >> 12) & 1).astype(np.int64)
        se = ((hw >> 13) & 7).astype(np.int64)
        key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
        skey = key * 4 + simd
        _, per_simd = np.unique(skey, return_counts=True)
        _, per_cu = np.unique(key, return_counts=True)
        share = np.array([per_simd[np.searchsorted(np.unique(skey), k)] for k in skey])
        print(f"--- last launch, {nw} waves: duration us mean {dur.mean():.1f} max {dur.max():.1f}; "
              f"distinct CUs {len(per_cu)}, SIMDs {len(per_simd)}, waves/SIMD max {per_simd.max()}")
        for k in sorted(set(share.tolist())):
            m = share == k
            print(f"  waves sharing a SIMD with {k - 1} others: {m.sum():5d}  duration us mean {dur[m].mean():.1f} max {dur[m].max():.1f}")
        print(f"  waves per CU histogram: {np.bincount(per_cu).tolist()}")
    phases = ["own ship (sampler, guidance, dynamics)", "boundary distance", "hull test",
              "IW test, rest, exchange writes", "barrier", "env level (reward, outputs)", "auto reset"]
    wave_steps = args.launches * args.chunk * ((args.n_env + 63) // 64)
    if c[:, 16:23].sum() > 0:
        for t, name in enumerate(("test ship", "obstacle ship")):
            tot = c[t, 16:23].sum()
            print(f"--- {name}: shader-clock cycles per wave-step (total {tot / wave_steps:.0f})")
            for k, nm in enumerate(phases):
                print(f"  {nm:40s} {c[t, 16 + k] / wave_steps:10.1f}  {100 * c[t, 16 + k] / tot:5.1f}%")
    if c[:, 24].sum() > 0:
        waves = args.launches * ((args.n_env + 63) // 64)
        for t, name in enumerate(("test ship", "obstacle ship")):
            print(f"--- {name}: per-launch wave timing (shader clock; realtime = 100 MHz ticks)")
            print(f"  mean wave cycles / launch            {c[t, 24] / waves:12.0f}")
            print(f"  max wave cycles (any launch)         {c[t, 25]:12.0f}")
            print(f"  mean prologue cycles                 {c[t, 26] / waves:12.0f}")
            print(f"  mean epilogue cycles                 {c[t, 27] / waves:12.0f}")
        print(f"  last launch: start skew {(c[:, 29].max() - c[:, 28].min()) * 10:.0f} ns, "
              f"end skew {(c[:, 31].max() - c[:, 30].min()) * 10:.0f} ns, "
              f"first start -> last end {(c[:, 31].max() - c[:, 28].min()) * 10:.0f} ns")
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
