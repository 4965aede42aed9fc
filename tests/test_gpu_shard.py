"""GPU path of the multi-rank replay-transition gather (sac_maritime_ast_amd/shard.py) on cuda:0.

The gloo tests (tests/test_distributed.py) cover the collective logic on CPU tensors; this drives
``AsyncTransitionGather``'s device branch — the collective stream, the count copy into pinned host
memory behind an event, the stream-side wait before a slot is reused — through bench.py's rollout
loop (buffers(i) -> launch i writes its sampling-event records -> start(i) -> progress(i - 1)) at
world size 1, where rank 0 is the learner.  This is the consumer path of ``memory.push``
(test_beds/main_ast.py:385-396).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

sit = pytest.importorskip("sac_maritime_ast_amd")
from sac_maritime_ast_amd import VecMultiShipRLEnv, make_scenario  # noqa: E402
from sac_maritime_ast_amd.shard import AsyncTransitionGather  # noqa: E402

DEV = "cuda:0"


def _sorted(rec):
    """Records per env in step order (one wave writes an env's records in order)."""
    rec = rec.cpu().numpy()
    return rec[np.argsort(rec[:, 23], kind="stable")]


@pytest.mark.parametrize("slots", [2, 3])
def test_async_gather_device_branch_world1(slots):
    n_env, chunk, n_launch = 4096, 400, 9
    cap = max(n_env, n_env * chunk // 192)
    envs = []
    for _ in range(2):
        e = VecMultiShipRLEnv(scenario=make_scenario(n_env, cap=48, seed=3), precision=32, device=DEV)
        e.reset()
        e.init_step()
        envs.append(e)
    env, ref = envs
    ga = AsyncTransitionGather(cap, 24, env.dtype, DEV, world=1, slots=slots)
    assert ga.cuda and ga.stream is not None
    out, ref_out, want, got = {}, {}, [], []
    for i in range(n_launch):
        out["transitions"], out["transition_count"] = ga.buffers(i)
        env.rollout(chunk, seed=11, out=out, transition_capacity=cap)
        ga.start(i)
        ga.progress(i - 1)
        if i >= 1:
            got.append(_sorted(ga.records(i - 1)))      # the previous launch's records, gathered
        r = ref.rollout(chunk, seed=11, out=ref_out, transition_capacity=cap)
        want.append(_sorted(r["transitions"][:int(r["transition_count"].item())]))
    ga.finish()
    got.append(_sorted(ga.records(n_launch - 1)))
    torch.cuda.synchronize()
    total = 0
    for i, (g, w) in enumerate(zip(got, want)):
        assert g.shape == w.shape, f"launch {i}: {g.shape[0]} records gathered, {w.shape[0]} written"
        assert np.array_equal(g, w), f"launch {i}: gathered records differ"
        total += w.shape[0]
    assert total > n_launch * n_env * chunk // 600     # ~1 record per 390 env-steps
    assert ga.gathered == total and ga.dropped() == 0
    assert ga.launches == n_launch


def test_trajectory_gather_device_branch_world1():
    """TrajectoryGather on the GPU (world 1: the learner keeps its own strided rows): the collective
    stream's strided copy behind each launch equals the launch's rows, and the next launch reusing the
    same output buffers does not disturb the gathered copy (the launch stream waits for the copy)."""
    from sac_maritime_ast_amd.shard import TrajectoryGather
    n, k, stride = 2048, 200, 9
    env = VecMultiShipRLEnv(scenario=make_scenario(n, cap=48), precision=32, device="cuda:0")
    env.reset()
    env.init_step()
    g = TrajectoryGather(k, n, stride, env.dtype, "cuda:0", 1)
    out = {}
    for it in range(3):
        env.rollout(k, seed=5, out=out)
        want = {f: out[f][::stride].clone() for f in TrajectoryGather.FIELDS}
        g.start(out)
        env.rollout(k, seed=6, out=out)            # overwrites `out` while the gather's copy is queued
        g.wait()
        for f in TrajectoryGather.FIELDS:
            got = g.gathered(f)[0]
            if got.is_floating_point():
                assert torch.equal(got.view(torch.int32), want[f].view(torch.int32)), (it, f)
            else:
                assert torch.equal(got, want[f]), (it, f)
