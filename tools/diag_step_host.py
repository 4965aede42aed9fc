#!/usr/bin/env python3
"""Where the scalar drop-in's per-step time goes: wall time per call (host perf_counter, median of
400 after 50 warm-up) of
  sync        torch.cuda.synchronize() alone (the completion round trip of an idle stream)
  empty       a 1-element torch kernel + synchronize (launch + completion)
  sit_step    sit_step on device arrays (1 env, the K=1 sync kernel) + hipStreamSynchronize
  step_host   sit_step_host (pinned coherent staging, one launch, one synchronisation)
  step_host_s sit_step_host with the state blob copy (what a recording drop-in does)
  compat      compat.MultiShipRLEnv.step (record False / True)
One JSON line."""
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
from sac_maritime_ast_amd import VecMultiShipRLEnv, make_scenario  # noqa: E402


def bench(fn, n=450, warm=50):
    lat = []
    for i in range(n):
        t0 = time.perf_counter()
        fn()
        lat.append(time.perf_counter() - t0)
    v = np.asarray(lat[warm:]) * 1e6
    return {"median_us": float(np.median(v)), "p10_us": float(np.percentile(v, 10)), "p90_us": float(np.percentile(v, 90))}


def main():
    torch.cuda.init()
    dev = "cuda:0"
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    res = {}
    res["sync"] = bench(torch.cuda.synchronize)
    x = torch.zeros(1, device=dev)
    res["empty"] = bench(lambda: (x.add_(1), torch.cuda.synchronize()))
    res["hip_sync_ctypes"] = bench(lambda: hip.hipStreamSynchronize(None))
    for prec in (64, 32):
        env = VecMultiShipRLEnv(scenario=make_scenario(1, cap=32, jitter=False), precision=prec, device=dev)
        env.reset()
        env.init_step()
        dt = np.float64 if prec == 64 else np.float32
        st = env.get_state()
        a_h = np.array([float(st["north"][1, 0]) + 500.0, float(st["east"][1, 0])], dt)
        z = np.zeros(1, np.uint8)
        ns, rw, dn, stt = np.zeros(10, dt), np.zeros(1, dt), np.zeros(1, np.uint8), np.zeros(1, np.uint32)
        blob = np.zeros(env._state_bytes, np.uint8)
        p = lambda a: ctypes.c_void_p(a.ctypes.data)  # noqa: E731
        stream = env._stream()
        args = (env.handle, p(a_h), p(z), p(z), p(ns), p(rw), p(dn), p(stt), None, None, stream)
        args_s = args[:9] + (p(blob), stream)
        res[f"f{prec}_step_host"] = bench(lambda: env.lib.sit_step_host(*args))
        res[f"f{prec}_step_host_state"] = bench(lambda: env.lib.sit_step_host(*args_s))
        a_d = torch.from_numpy(a_h).to(dev)
        z_d = torch.zeros(1, dtype=torch.uint8, device=dev)
        o = [torch.zeros(10, dtype=env.dtype, device=dev), torch.zeros(1, dtype=env.dtype, device=dev),
             torch.zeros(1, dtype=torch.uint8, device=dev), torch.zeros(1, dtype=torch.int32, device=dev)]
        dargs = (env.handle, a_d.data_ptr(), z_d.data_ptr(), z_d.data_ptr(), *[t.data_ptr() for t in o], None, stream)

        def dev_step():
            env.lib.sit_step(*dargs)
            hip.hipStreamSynchronize(stream)
        res[f"f{prec}_sit_step_device"] = bench(dev_step)
        res[f"f{prec}_kernel"] = env.lib.sit_step_kernel(env.handle).decode()
    from helpers import golden
    from ref_assets import args as ref_args
    from ref_assets import fixture_assets, polygon_obstacle
    from sac_maritime_ast_amd.compat import MultiShipRLEnv
    d = golden("env_nominal")
    for rec in (False, True):
        e = MultiShipRLEnv(fixture_assets(d), polygon_obstacle(), False, 30, ref_args(), device=dev,
                           wpt_capacity=d["routes"].shape[1], record=rec)
        e.reset()
        e.init_step()
        it = iter(range(10 ** 6))
        acts = [(float(a), float(b)) for a, b in zip(d["action_n"][:600], d["action_e"][:600])]
        sacs, inits = [bool(x) for x in d["sac_update"][:600]], [bool(x) for x in d["init"][:600]]

        def cstep():
            i = next(it) % 600
            e.step(acts[i], sacs[i], inits[i])
        res[f"compat_f64_record_{rec}"] = bench(cstep)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
