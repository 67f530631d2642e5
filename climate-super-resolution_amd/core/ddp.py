"""Data parallelism for the native modules (replaces Lightning DDP, conf/trainer/benchmark.yaml:3-5).

One process per GPU; tiles are independent, so the only exchange is the gradient average once per
optimizer step.  Gradients live in ONE flat fp32 buffer per network (core/flat.py),
so the all-reduce is a handful of large contiguous buckets on RCCL ("nccl" backend = RCCL over
xGMI on MI355X); gloo on CPU for the tests.  No SyncBN: BN statistics stay per rank (the reference
sets sync_batchnorm: False, conf/trainer/default.yaml:31).
"""
from __future__ import annotations

from typing import List

import torch
import torch.distributed as dist


class GradAllReducer:
    """Average a module's flat gradient buffer over the process group in fixed-size buckets."""

    def __init__(self, module, bucket_mb: int = 256, group=None):
        self.flat = module._flat_grad
        self.group = group
        n = self.flat.numel()
        step = max(1, (bucket_mb << 20) // 4)
        self.buckets: List[torch.Tensor] = [self.flat[i:i + step] for i in range(0, n, step)]

    def __call__(self) -> None:
        if not dist.is_initialized() or dist.get_world_size(self.group) == 1:
            return
        ws = dist.get_world_size(self.group)
        avg = dist.get_backend(self.group) == "nccl"
        works = [dist.all_reduce(b, op=dist.ReduceOp.AVG if avg else dist.ReduceOp.SUM, group=self.group, async_op=True)
                 for b in self.buckets]
        for w in works:
            w.wait()
        if not avg:
            self.flat.div_(ws)


class OverlappedGradAllReducer:
    """DDP gradient average overlapped with the backward.

    The native backward calls ``ready(lo)`` when every gradient at flat offsets >= ``lo`` is final
    (generator: after each group of RRDB blocks; discriminator: after its 103 M-parameter fc.0, whose
    gradient is computed first).  ``ready`` launches the all-reduce of the newly final slice
    ``[lo, previous lo)`` with ``async_op=True``: on RCCL the collective runs on the process group's own
    stream, ordered after the work already queued on the caller's stream, so it overlaps the rest of the
    backward.  ``finish()`` reduces what is left (``[0, last lo)``) and makes the caller's stream wait for
    every bucket.  The same ``ready`` / ``finish`` calls are replayed between the hipGraph segments of a
    captured step (bench.py splits the capture at the hook points)."""

    def __init__(self, module, group=None):
        self.flat = module._flat_grad
        self.group = group
        self.hi = self.flat.numel()
        self.works = []
        self.launched = []  # (lo, hi) of every bucket of the current step (tests / diagnostics)

    def _world(self) -> int:
        return dist.get_world_size(self.group) if dist.is_initialized() else 1

    def _reduce(self, lo: int, hi: int) -> None:
        if self.hi == self.flat.numel():  # first bucket of a step
            self.launched = []
        self.launched.append((lo, hi))
        if self._world() == 1 or hi <= lo:
            return
        b = self.flat[lo:hi]
        if dist.get_backend(self.group) == "nccl":
            self.works.append(dist.all_reduce(b, op=dist.ReduceOp.AVG, group=self.group, async_op=True))
        else:  # gloo (CPU tests): synchronous sum, then the average
            dist.all_reduce(b, op=dist.ReduceOp.SUM, group=self.group)
            b.div_(self._world())

    def ready(self, lo: int) -> None:
        lo = max(0, min(int(lo), self.hi))
        if lo < self.hi:
            self._reduce(lo, self.hi)
            self.hi = lo

    def finish(self) -> None:
        if self.hi > 0:
            self._reduce(0, self.hi)
        for w in self.works:
            w.wait()  # the caller's stream waits for the collective (no host sync on RCCL)
        self.works.clear()
        self.hi = self.flat.numel()


def shard_indices(n: int, rank: int, world: int, drop_last: bool = True) -> List[int]:
    """DistributedSampler-equivalent striding (replace_sampler_ddp: True): index i goes to rank i % world."""
    total = (n // world) * world if drop_last else n
    return list(range(rank, total, world))


def rank_seed(seed: int, rank: int) -> int:
    """Per-rank synthetic-data seed (seed 42 + rank)."""
    return seed + rank


def broadcast_module(module, src: int = 0, group=None) -> None:
    """Rank-0 parameters and buffers to every rank (DDP construction / broadcast_buffers semantics)."""
    if not dist.is_initialized():
        return
    flat = getattr(module, "_flat", None)
    if flat is not None:
        dist.broadcast(flat, src, group=group)
    else:
        for p in module.parameters():
            dist.broadcast(p.data, src, group=group)
    for b in module.buffers():
        dist.broadcast(b, src, group=group)
