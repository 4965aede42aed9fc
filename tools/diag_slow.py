"""Which envs make a step-kernel block slow?  (diagnostic; SIT_DIAG_PHASES build)

    SIT_LIBRARY=build_diag/libsit_phases.so python tools/diag_slow.py
Runs the bench workload to steady state, times every wave of one launch and prints the
state of the envs in the slowest blocks next to that of median blocks."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from sac_maritime_ast_amd import VecMultiShipRLEnv, make_scenario, _lib  # noqa: E402
from oracle import sit_oracle as so  # noqa: E402  (diagnostic geometry only)

n_env, chunk = 32768, 200
lib = ctypes.CDLL(_lib.LIB_PATH)
sc = make_scenario(n_env, cap=48)
env = VecMultiShipRLEnv(scenario=sc, precision=32, device="cuda:0")
env.reset()
env.init_step()
for _ in range(200):
    env.rollout(chunk, seed=25450)
st0 = {k: v.cpu().numpy().copy() for k, v in env.get_state().items()}
out = env.rollout(chunk, seed=25450)
torch.cuda.synchronize()
nw = 2 * n_env // 64
wb = (ctypes.c_ulonglong * (4 * nw))()
assert lib.sit_diag_read_waves(wb, nw) == 0
w = np.array(wb[:], dtype=np.uint64).reshape(nw, 4)
dur = ((w[:, 1] - w[:, 0]).astype(np.float64) * 10e-3).reshape(-1, 2).max(1)
order = np.argsort(dur)
act = out["action"].cpu().numpy()
done = out["done"].cpu().numpy()
status = out["status"].cpu().numpy().astype(np.int64) & 0xffffffff
ns = out["next_state"].cpu().numpy()


def show(b):
    e = np.arange(b * 64, (b + 1) * 64)
    ev = (act[:, e, 3] > 0.5).sum()
    dn = done[:, e].sum()
    # per lane distance to the shore along the launch (test and obstacle ship)
    dt = so.distance_to_polygons(sc.polys, ns[:, e, 0].astype(np.float64).ravel(), ns[:, e, 1].astype(np.float64).ravel())
    do = so.distance_to_polygons(sc.polys, ns[:, e, 6].astype(np.float64).ravel(), ns[:, e, 7].astype(np.float64).ravel())
    near_t = (dt < 60).reshape(chunk, 64).any(1).sum()
    near_o = (do < 60).reshape(chunk, 64).any(1).sum()
    out_t = ((ns[:, e, 0] < -1500) | (ns[:, e, 0] > 11500) | (ns[:, e, 1] < -1500) | (ns[:, e, 1] > 11500)).any(1).sum()
    out_o = ((ns[:, e, 6] < -1500) | (ns[:, e, 6] > 11500) | (ns[:, e, 7] < -1500) | (ns[:, e, 7] > 11500)).any(1).sum()
    stop_o = st0["stop"][1, e].sum()
    print(f"block {b:4d} {dur[b]:7.1f} us | events {ev:4d} dones {dn:3d} | steps with a lane <60 m from shore "
          f"test {near_t:3d} obs {near_o:3d} | off-grid steps test {out_t:3d} obs {out_o:3d} | obs stopped at start {stop_o}"
          f" | status bits {np.bitwise_or.reduce(status[:, e].ravel()):#x}")


print("slowest blocks:")
for b in order[::-1][:10]:
    show(b)
print("median blocks:")
for b in order[len(order) // 2 - 5: len(order) // 2 + 5]:
    show(b)
