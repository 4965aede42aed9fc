"""N > 1 path on CPU (gloo, world size 2): env sharding by global env id plus the gather of the
replay transitions to the learner (sac_maritime_ast_amd.shard: count all-gather, then the valid
records point-to-point to rank 0).  The CPU oracle stands in for the GPU env here; the
GPU runs use the same shard offsets and the same gather over RCCL."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import sit_oracle as so
from sac_maritime_ast_amd.scenario import make_scenario
from sac_maritime_ast_amd.shard import TransitionGather, shard_offset

N_PER_RANK, STEPS, SEED, CAP = 48, 160, 4242, 512


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rollout(n_env, offset):
    sc = make_scenario(n_env, cap=24, seed=SEED, env_offset=offset)
    o = so.OracleEnvs(dict(so.DEFAULT_PARAMS), sc.routes, sc.n_wpt, sc.init, sc.polys)
    o.reset()
    o.init_step()
    return o.rollout(STEPS, seed=SEED, env_id_offset=offset)


def _worker(rank, world, port, result_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        off = shard_offset(rank, N_PER_RANK)
        r = _rollout(N_PER_RANK, off)
        tr = torch.zeros((CAP, 24), dtype=torch.float64)
        k = min(len(r["transitions"]), CAP)
        tr[:k] = torch.from_numpy(r["transitions"][:k])
        cnt = torch.tensor([len(r["transitions"])], dtype=torch.int32)
        g = TransitionGather(CAP, 24, torch.float64, "cpu", world)
        g(tr, cnt)
        ns = torch.from_numpy(r["next_state"])
        all_ns = [torch.empty_like(ns) for _ in range(world)]
        dist.all_gather(all_ns, ns)
        if rank == 0:
            full = _rollout(world * N_PER_RANK, 0)
            got = g.records().numpy()
            want = full["transitions"]
            assert g.dropped() == 0
            key = lambda a: np.lexsort((a[:, 12], a[:, 23]))  # noqa: E731
            got, want = got[key(got)], want[key(want)]
            assert got.shape == want.shape, (got.shape, want.shape)
            np.testing.assert_allclose(got, want, rtol=1e-12, atol=1e-12)
            sharded = torch.cat(all_ns, dim=1).numpy()
            np.testing.assert_allclose(sharded, full["next_state"], rtol=1e-12, atol=1e-9)
            with open(result_path, "w") as f:
                f.write(f"ok {len(got)}")
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_rank_shards_equal_one_big_run(tmp_path):
    path = str(tmp_path / "result.txt")
    mp.spawn(_worker, args=(2, _free_port(), path), nprocs=2, join=True)
    assert open(path).read().startswith("ok")


def _async_worker(rank, world, port, result_path):
    """AsyncTransitionGather: count all-gather per launch, then (one launch later) the valid records
    point-to-point to the learner (rank 0); every record arrives once, none is dropped."""
    from sac_maritime_ast_amd.shard import AsyncTransitionGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = AsyncTransitionGather(16, 24, torch.float64, "cpu", world)
        seen = []
        for i in range(5):
            rec, cnt = g.buffers(i)
            n = 3 + i + rank                       # rank- and launch-dependent record counts
            rec.zero_()
            rec[:n, 0] = float(i)
            rec[:n, 23] = float(rank)
            cnt.fill_(n)
            g.start(i)
            g.progress(i - 1)
            if rank == 0 and i > 0:
                seen.append((i - 1, g.records(i - 1).clone()))
        g.finish()
        if rank == 0:
            seen.append((4, g.records(4).clone()))
            for j, got in seen:
                assert got.shape[0] == sum(3 + j + r for r in range(world))
                assert torch.all(got[:, 0] == j)
                for r in range(world):
                    assert int((got[:, 23] == r).sum()) == 3 + j + r
        assert g.launches == 5 and g.dropped() == 0
        assert g.gathered == sum(3 + j + r for j in range(5) for r in range(world))
        if rank == 0:
            with open(result_path, "w") as f:
                f.write("ok")
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _overflow_worker(rank, world, port, result_path):
    """Records beyond a rank's capacity are counted as dropped, the rest still arrive."""
    from sac_maritime_ast_amd.shard import AsyncTransitionGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = AsyncTransitionGather(8, 24, torch.float64, "cpu", world)
        rec, cnt = g.buffers(0)
        rec[:, 23] = float(rank)
        cnt.fill_(8 + 5 * rank)                    # rank 1 wrote 13 > capacity 8
        g.start(0)
        g.finish()
        assert g.dropped() == 5 and g.gathered == 16
        if rank == 0:
            assert g.records(0).shape[0] == 16
            with open(result_path, "w") as f:
                f.write("ok")
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_transition_gather_counts_overflow(tmp_path):
    path = str(tmp_path / "result_overflow.txt")
    mp.spawn(_overflow_worker, args=(2, _free_port(), path), nprocs=2, join=True)
    assert open(path).read() == "ok"


def test_async_transition_gather_two_ranks(tmp_path):
    path = str(tmp_path / "result_async.txt")
    mp.spawn(_async_worker, args=(2, _free_port(), path), nprocs=2, join=True)
    assert open(path).read() == "ok"


def _traj_worker(rank, world, port, result_path):
    """TrajectoryGather: every stride-th row of each rank's launch rows arrives on the learner in
    rank order (the oracle's sharded rollouts: rank r's rows are global envs [r n, (r + 1) n)), and the
    gathered rows equal the strided rows of one big run."""
    from sac_maritime_ast_amd.shard import TrajectoryGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        off = shard_offset(rank, N_PER_RANK)
        r = _rollout(N_PER_RANK, off)
        out = {"next_state": torch.from_numpy(r["next_state"]), "reward": torch.from_numpy(r["reward"]),
               "done": torch.from_numpy(r["done"].astype(np.uint8)),
               "status": torch.from_numpy(r["status"].astype(np.int32))}
        stride = 7
        g = TrajectoryGather(STEPS, N_PER_RANK, stride, torch.float64, "cpu", world)
        g.start(out)
        g.wait()
        if rank == 0:
            full = _rollout(world * N_PER_RANK, 0)
            ns = g.gathered("next_state")                       # [world, rows, n, 10]
            assert ns.shape == (world, -(-STEPS // stride), N_PER_RANK, 10)
            got = torch.cat(list(ns), dim=1).numpy()            # rank order = global env order
            np.testing.assert_allclose(got, full["next_state"][::stride], rtol=1e-12, atol=1e-9)
            st = torch.cat(list(g.gathered("status")), dim=1).numpy()
            assert np.array_equal(st.astype(np.int64) & 0xFFFFFFFF, full["status"][::stride].astype(np.int64))
            assert g.bytes_moved == sum(t.numel() * t.element_size() for t in g.send.values())
            with open(result_path, "w") as f:
                f.write("ok")
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_trajectory_gather_two_ranks(tmp_path):
    path = str(tmp_path / "result_traj.txt")
    mp.spawn(_traj_worker, args=(2, _free_port(), path), nprocs=2, join=True)
    assert open(path).read() == "ok"


def _subgroup_worker(rank, world, port, result_path):
    """The gathers inside a process subgroup ({1, 2} of a world of 3): ranks, world size and the learner
    count within the group, while torch.distributed's point-to-point ops take GLOBAL peer ranks
    (shard._peer maps them).  Group rank 0 (global rank 1) is the learner and must receive global rank
    2's records and trajectory rows; global rank 0 is not a member and moves nothing."""
    from sac_maritime_ast_amd.shard import TrajectoryGather
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        grp = dist.new_group([1, 2])
        if rank in (1, 2):
            # replay records: 3 + rank valid rows, tagged with the global rank
            tr = torch.zeros((16, 24), dtype=torch.float64)
            n = 3 + rank
            tr[:n, 0] = float(rank)
            tr[:n, 23] = torch.arange(n, dtype=torch.float64)
            g = TransitionGather(16, 24, torch.float64, "cpu", 2, group=grp, dst=0)
            g(tr, torch.tensor([n], dtype=torch.int32))
            # trajectory rows: value = 1000 * global rank + step
            k, n_env, stride = 9, 4, 2
            steps = torch.arange(k, dtype=torch.float64)[:, None]
            out = {"next_state": (1000.0 * rank + steps)[:, :, None].expand(k, n_env, 10).contiguous(),
                   "reward": (1000.0 * rank + steps).expand(k, n_env).contiguous(),
                   "done": torch.zeros((k, n_env), dtype=torch.uint8),
                   "status": torch.full((k, n_env), rank, dtype=torch.int32)}
            tg = TrajectoryGather(k, n_env, stride, torch.float64, "cpu", 2, group=grp, dst=0)
            tg.start(out)
            tg.wait()
            if rank == 1:
                rec = g.records()
                assert rec.shape[0] == (3 + 1) + (3 + 2)
                assert (rec[:4, 0] == 1).all() and (rec[4:, 0] == 2).all()
                rw = tg.gathered("reward")                      # [2, rows, n_env]: group ranks 0, 1
                want = torch.arange(0, k, stride, dtype=torch.float64)[:, None].expand(-1, n_env)
                assert torch.equal(rw[0], 1000.0 + want) and torch.equal(rw[1], 2000.0 + want)
                assert (tg.gathered("status")[1] == 2).all()
                with open(result_path, "w") as f:
                    f.write("ok")
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_gathers_in_a_process_subgroup(tmp_path):
    path = str(tmp_path / "result_group.txt")
    mp.spawn(_subgroup_worker, args=(3, _free_port(), path), nprocs=3, join=True)
    assert open(path).read() == "ok"
