"""Diagnostic: action-row angles on non-sampling rows (float32 handle)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from sac_maritime_ast_amd import VecMultiShipRLEnv, make_scenario  # noqa: E402

for prec in (32, 64):
    env = VecMultiShipRLEnv(scenario=make_scenario(2048, cap=48), precision=prec, device="cuda:0")
    env.reset()
    env.init_step()
    out = env.rollout(300, seed=11)
    a = out["action"].cpu().numpy()
    sac = a[..., 3] > 0.5
    bad = ~np.isnan(a[..., 2]) & ~sac
    print(prec, "rows", a.shape, "sac", sac.sum(), "non-sac", (~sac).sum(), "non-nan non-sac", bad.sum())
    if bad.any():
        idx = np.argwhere(bad)[:10]
        for t, e in idx:
            print("  t", t, "e", e, "row", a[t, e], "status", out["status"][t, e].item(), "done", out["done"][t, e].item())
