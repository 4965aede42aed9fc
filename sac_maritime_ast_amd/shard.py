"""Multi-GPU sharding of the env population.

Envs are independent units: rank r of W owns global envs [r * n, (r + 1) * n) (its scenario is
built with env_offset = r * n, and the sampler keys its Philox streams by global env id), so
stepping needs no collective.  The only exchange is the replay-transition stream the SAC
learner consumes (test_beds/main_ast.py:385-396): each launch's sampling-event transitions are
appended by the kernel to a fixed-capacity device buffer with a device-side count, and gathered to
the learner (rank 0) over RCCL/xGMI (gloo in the CPU tests):

  1. the per-rank counts are all-gathered (W int32, on the collective's own stream, behind the
     launch's completion event);
  2. once the host has those counts — read after the NEXT launch has been enqueued, so the GPU
     never idles on the host — every rank r > 0 sends exactly its count_r valid records (24 reals
     each) point-to-point to rank 0, which receives each into its own slot.  Nothing but valid
     records crosses xGMI, and only the learner receives them.

Records beyond a rank's buffer capacity are counted (``dropped()``) and never silently lost from
the books: the bench reports the total.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_offset(rank: int, n_env_per_rank: int) -> int:
    return rank * n_env_per_rank


class TransitionGather:
    """Synchronous gather of one chunk's valid records to the learner rank (host-synchronising;
    used by tests and simple loops)."""

    def __init__(self, capacity: int, dim: int, dtype, device, world: int, group=None, dst: int = 0):
        self.capacity, self.dim, self.world, self.group, self.dst = capacity, dim, world, group, dst
        self.rank = dist.get_rank(group) if world > 1 else 0
        self.device = torch.device(device)
        self.recv = [torch.empty((capacity, dim), dtype=dtype, device=device) for _ in range(world)]
        self.counts = torch.zeros(world, dtype=torch.int32, device=device)
        self.host_counts = [0] * world

    def __call__(self, transitions: torch.Tensor, count: torch.Tensor):
        if self.world == 1:
            self.recv[0], self.counts = transitions, count.reshape(1).to(torch.int32)
            self.host_counts = [int(self.counts[0].item())]
            return
        dist.all_gather_into_tensor(self.counts, count.reshape(1).to(torch.int32), group=self.group)
        self.host_counts = [int(c) for c in self.counts.cpu().tolist()]
        ops = _p2p_ops(self.rank, self.dst, self.world, self.host_counts, self.capacity, transitions, self.recv,
                       self.group)
        for w in (dist.batch_isend_irecv(ops) if ops else []):
            w.wait()
        if self.rank == self.dst:
            n = min(self.host_counts[self.rank], self.capacity)
            self.recv[self.rank][:n].copy_(transitions[:n])

    def records(self):
        """Valid records of every rank, concatenated (learner rank only)."""
        return torch.cat([b[:min(c, self.capacity)] for b, c in zip(self.recv, self.host_counts)])

    def dropped(self):
        return sum(max(0, c - self.capacity) for c in self.host_counts)


def _peer(group, r):
    """The global rank of group rank r: torch.distributed's P2POp takes global peer ranks, while
    rank / dst / world here count within `group`."""
    return r if group is None else dist.get_global_rank(group, r)


def _p2p_ops(rank, dst, world, counts, capacity, send, recv, group):
    """Point-to-point ops moving each rank's valid records (counts[r], clamped to the capacity) to
    rank dst.  Sizes are known on every rank, so every send has its matching receive."""
    ops = []
    if rank == dst:
        for r in range(world):
            n = min(counts[r], capacity)
            if r != dst and n > 0:
                ops.append(dist.P2POp(dist.irecv, recv[r][:n], _peer(group, r), group))
    else:
        n = min(counts[rank], capacity)
        if n > 0:
            ops.append(dist.P2POp(dist.isend, send[:n].contiguous(), _peer(group, dst), group))
    return ops


class AsyncTransitionGather:
    """Pipelined gather for the rollout loop (no host wait beside an idle GPU).

    launch i writes into slot i % slots (``buffers(i)``); ``start(i)`` queues the count all-gather
    behind launch i on the collective stream and a copy of the counts to pinned host memory;
    ``progress(i)``, called after launch i + 1 has been enqueued, waits for those counts on the
    host (launch i has finished by then, launch i + 1 keeps the GPU busy) and queues the
    point-to-point transfers of exactly the valid records to the learner.  A slot is reused by
    launch i + slots only after its transfers finished (stream-side wait)."""

    def __init__(self, capacity: int, dim: int, dtype, device, world: int, group=None, slots: int = 2,
                 dst: int = 0):
        self.capacity, self.dim, self.world, self.group, self.dst = capacity, dim, world, group, dst
        self.rank = dist.get_rank(group) if world > 1 else 0
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.slots = slots
        self.send = [torch.zeros((capacity, dim), dtype=dtype, device=device) for _ in range(slots)]
        self.send_count = [torch.zeros(1, dtype=torch.int32, device=device) for _ in range(slots)]
        # receive slots on the learner only
        nrecv = world if self.rank == dst else 0
        self.recv = [[torch.empty((capacity, dim), dtype=dtype, device=device) for _ in range(nrecv)]
                     for _ in range(slots)]
        self.counts = [torch.zeros(world, dtype=torch.int32, device=device) for _ in range(slots)]
        self.host_counts = [torch.zeros(world, dtype=torch.int32, pin_memory=self.cuda) for _ in range(slots)]
        self.counts_ready = [None] * slots
        self.work = [[] for _ in range(slots)]
        self.done_ev = [None] * slots
        self.stream = torch.cuda.Stream(device=self.device) if self.cuda else None
        self.launches = 0
        self.gathered = 0           # valid records moved to (or kept on) the learner
        self.n_dropped = 0          # records beyond a rank's capacity (counted, not written)
        self._started = set()

    def _ctx(self):
        return torch.cuda.stream(self.stream) if self.cuda else _Null()

    def buffers(self, i: int):
        """(records, count) for launch i; waits (stream-side) for the transfers that last used them."""
        k = i % self.slots
        for w in self.work[k]:
            w.wait()
        self.work[k] = []
        if self.cuda and self.done_ev[k] is not None:
            torch.cuda.current_stream(self.device).wait_event(self.done_ev[k])
        return self.send[k], self.send_count[k]

    def start(self, i: int):
        """Queue the count all-gather of launch i (asynchronous)."""
        k = i % self.slots
        if self.cuda:
            self.stream.wait_stream(torch.cuda.current_stream(self.device))
        with self._ctx():
            if self.world > 1:
                dist.all_gather_into_tensor(self.counts[k], self.send_count[k], group=self.group)
            else:
                self.counts[k].copy_(self.send_count[k])
            self.host_counts[k].copy_(self.counts[k], non_blocking=self.cuda)
            if self.cuda:
                ev = torch.cuda.Event()
                ev.record(self.stream)
                self.counts_ready[k] = ev
        self._started.add(i)
        self.launches += 1

    def progress(self, i: int):
        """Queue the record transfers of launch i (waits on the host for its counts only)."""
        if i not in self._started:
            return
        self._started.discard(i)
        k = i % self.slots
        if self.cuda:
            self.counts_ready[k].synchronize()
        counts = [int(c) for c in self.host_counts[k].tolist()]
        self.n_dropped += sum(max(0, c - self.capacity) for c in counts)
        self.gathered += sum(min(c, self.capacity) for c in counts)
        self.last_counts = counts
        with self._ctx():
            ops = _p2p_ops(self.rank, self.dst, self.world, counts, self.capacity, self.send[k], self.recv[k],
                           self.group)
            self.work[k] = dist.batch_isend_irecv(ops) if ops else []
            if self.rank == self.dst and self.world > 1:
                n = min(counts[self.rank], self.capacity)
                self.recv[k][self.rank][:n].copy_(self.send[k][:n])
            if self.cuda:
                ev = torch.cuda.Event()
                ev.record(self.stream)
                self.done_ev[k] = ev

    def finish(self):
        for i in sorted(self._started):
            self.progress(i)
        for k in range(self.slots):
            for w in self.work[k]:
                w.wait()
            self.work[k] = []
        if self.cuda:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)

    def records(self, i: int):
        """Valid records of every rank gathered for launch i (learner rank; after progress(i))."""
        k = i % self.slots
        for w in self.work[k]:
            w.wait()
        self.work[k] = []           # a completed work is waited on once (gloo hangs on a second wait)
        if self.cuda:
            self.stream.synchronize()
        counts = [int(c) for c in self.host_counts[k].tolist()]
        if self.world == 1:
            return self.send[k][:min(counts[0], self.capacity)]
        return torch.cat([b[:min(c, self.capacity)] for b, c in zip(self.recv[k], counts)])

    def dropped(self) -> int:
        return self.n_dropped


class TrajectoryGather:
    """Strided trajectory rows of every rank to the learner rank (the RCCL gather of
    trajectory chunks), for consumers that need whole trajectories on one rank.

    A launch of K steps writes rows [K, n_env, ...] per rank (next_state, reward, done, status); every
    `stride`-th row (rows 0, stride, 2 stride, ...) of each rank is copied into a send buffer on the
    collective stream, behind the launch, and sent point-to-point to the learner, which receives
    rank r's rows into slot r.  Sizes are fixed by (K, stride, n_env), so no count exchange is needed.
    The launch stream waits only for the copy (``start``), not for the transfer; ``wait`` joins the
    transfer.  Why strided: a C3 launch writes 65 B per env-step, 2.1 MB per step per rank; all rows of 7
    ranks into one GPU would need ~7 TB/s, while the transitions the SAC learner consumes are gathered
    whole (AsyncTransitionGather)."""

    FIELDS = ("next_state", "reward", "done", "status")

    def __init__(self, k: int, n_env: int, stride: int, dtype, device, world: int, group=None, dst: int = 0):
        if stride < 1 or k < 1:
            raise ValueError("need k >= 1 and stride >= 1")
        self.k, self.n_env, self.stride, self.world, self.group, self.dst = k, n_env, stride, world, group, dst
        self.rank = dist.get_rank(group) if world > 1 else 0
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.rows = -(-k // stride)
        shapes = {"next_state": ((self.rows, n_env, 10), dtype), "reward": ((self.rows, n_env), dtype),
                  "done": ((self.rows, n_env), torch.uint8), "status": ((self.rows, n_env), torch.int32)}
        self.send = {f: torch.empty(shp, dtype=dt, device=device) for f, (shp, dt) in shapes.items()}
        nrecv = world if self.rank == dst else 0
        self.recv = {f: [torch.empty(shp, dtype=dt, device=device) for _ in range(nrecv)]
                     for f, (shp, dt) in shapes.items()}
        self.stream = torch.cuda.Stream(device=self.device) if self.cuda else None
        self.work = []
        self.bytes_moved = 0     # bytes received by the learner from the other ranks

    def start(self, out: dict):
        """Queue the strided copy of `out`'s rows (behind the launch that wrote them) and their transfer
        to the learner.  The caller's stream waits for the copy only: the next launch may then reuse
        `out` while the rows travel."""
        self.wait()
        cur = torch.cuda.current_stream(self.device) if self.cuda else None
        if self.cuda:
            self.stream.wait_stream(cur)
        ctx = torch.cuda.stream(self.stream) if self.cuda else _Null()
        with ctx:
            for f in self.FIELDS:
                self.send[f].copy_(out[f][::self.stride])
            if self.cuda:
                copied = torch.cuda.Event()
                copied.record(self.stream)
            ops = []
            if self.world > 1:
                if self.rank == self.dst:
                    for r in range(self.world):
                        if r != self.dst:
                            ops += [dist.P2POp(dist.irecv, self.recv[f][r], _peer(self.group, r), self.group)
                                    for f in self.FIELDS]
                else:
                    ops += [dist.P2POp(dist.isend, self.send[f], _peer(self.group, self.dst), self.group)
                            for f in self.FIELDS]
            self.work = dist.batch_isend_irecv(ops) if ops else []
            if self.rank == self.dst:
                for f in self.FIELDS:
                    if self.world > 1:
                        self.recv[f][self.rank].copy_(self.send[f])
                if self.world > 1:
                    self.bytes_moved += (self.world - 1) * sum(t.numel() * t.element_size() for t in self.send.values())
        if self.cuda:
            cur.wait_event(copied)

    def wait(self):
        for w in self.work:
            w.wait()
        self.work = []
        if self.cuda:
            torch.cuda.current_stream(self.device).wait_stream(self.stream)

    def gathered(self, field: str):
        """[world, rows, n_env, ...] of the last started launch (learner rank, after wait())."""
        if self.rank != self.dst:
            raise RuntimeError("only the learner rank holds the gathered rows")
        if self.world == 1:
            return self.send[field].unsqueeze(0)
        return torch.stack(self.recv[field])


class _Null:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False
