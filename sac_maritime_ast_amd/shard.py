"""Multi-GPU sharding of the env population.

Envs are independent units: rank r of W owns global envs [r * n, (r + 1) * n) (its scenario is
built with env_offset = r * n, and the sampler keys its Philox streams by global env id), so
stepping needs no collective.  The only exchange is the replay-transition stream the SAC
learner consumes (test_beds/main_ast.py:385-396): each rollout chunk's sampling-event
transitions are written by the kernel into a fixed-capacity device buffer with a device-side
count, and one all-gather (RCCL over xGMI on MI355X; gloo in CPU tests) moves every rank's
buffer and count to every rank without a host synchronisation.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class TransitionGather:
    def __init__(self, capacity: int, dim: int, dtype, device, world: int, group=None):
        self.capacity, self.dim, self.world, self.group = capacity, dim, world, group
        self.bufs = [torch.empty((capacity, dim), dtype=dtype, device=device) for _ in range(world)]
        self.counts = [torch.empty(1, dtype=torch.int32, device=device) for _ in range(world)]

    def __call__(self, transitions: torch.Tensor, count: torch.Tensor):
        """All-gather one chunk (buffers stay on device; nothing waits on the host)."""
        if self.world == 1:
            self.bufs[0], self.counts[0] = transitions, count
            return
        dist.all_gather(self.counts, count, group=self.group)
        dist.all_gather(self.bufs, transitions, group=self.group)

    def records(self):
        """Valid records of every rank, concatenated (synchronises: learner side only)."""
        out = []
        for b, c in zip(self.bufs, self.counts):
            n = min(int(c.item()), self.capacity)
            out.append(b[:n])
        return torch.cat(out)

    def dropped(self):
        return sum(max(0, int(c.item()) - self.capacity) for c in self.counts)


class AsyncTransitionGather:
    """Double-buffered, asynchronous variant for the rollout loop: launch i writes its records
    into slot i % 2; the all-gather of slot i runs on the collective's own stream while launch
    i + 1 computes (RCCL over xGMI beside the env kernel), and slot i is reused by launch i + 2
    only after its gather finished (a stream-side wait, never a host synchronisation)."""

    def __init__(self, capacity: int, dim: int, dtype, device, world: int, group=None, slots: int = 2):
        self.capacity, self.dim, self.world, self.group = capacity, dim, world, group
        self.send = [torch.zeros((capacity, dim), dtype=dtype, device=device) for _ in range(slots)]
        self.send_count = [torch.zeros(1, dtype=torch.int32, device=device) for _ in range(slots)]
        self.recv = [[torch.empty((capacity, dim), dtype=dtype, device=device) for _ in range(world)]
                     for _ in range(slots)]
        self.recv_count = [[torch.empty(1, dtype=torch.int32, device=device) for _ in range(world)]
                           for _ in range(slots)]
        self.work = [[] for _ in range(slots)]
        self.launches = 0

    def buffers(self, i: int):
        """(records, count) for launch i; waits (stream-side) for the gather that last used them."""
        k = i % len(self.send)
        for w in self.work[k]:
            w.wait()
        self.work[k] = []
        return self.send[k], self.send_count[k]

    def start(self, i: int):
        """Issue the all-gather of launch i's records (asynchronous)."""
        k = i % len(self.send)
        self.work[k] = [dist.all_gather(self.recv_count[k], self.send_count[k], group=self.group, async_op=True),
                        dist.all_gather(self.recv[k], self.send[k], group=self.group, async_op=True)]
        self.launches += 1

    def finish(self):
        for ws in self.work:
            for w in ws:
                w.wait()
        self.work = [[] for _ in self.send]

    def records(self, i: int):
        """Valid records of every rank gathered for launch i (synchronises: learner side only)."""
        k = i % len(self.send)
        for w in self.work[k]:
            w.wait()
        out = []
        for b, c in zip(self.recv[k], self.recv_count[k]):
            out.append(b[:min(int(c.item()), self.capacity)])
        return torch.cat(out)


def shard_offset(rank: int, n_env_per_rank: int) -> int:
    return rank * n_env_per_rank
