"""world_size-2 gloo tests of the data-parallel path (CPU): bucketed flat-gradient averaging,
parameter/buffer broadcast, and the per-rank sharding / seeding."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class _FlatNet(torch.nn.Module):
    """Stand-in with the FlatParamsMixin layout (3 params in one flat buffer)."""

    def __init__(self):
        from climsr_amd.core.flat import FlatParamsMixin  # noqa: F401

        super().__init__()
        self.a = torch.nn.Parameter(torch.zeros(5))
        self.b = torch.nn.Parameter(torch.zeros(3, 4))
        self.register_buffer("stat", torch.zeros(2))


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from climsr_amd.core.ddp import GradAllReducer, broadcast_module, shard_indices
        from climsr_amd.core.flat import FlatParamsMixin

        class Net(FlatParamsMixin, _FlatNet):
            def __init__(self):
                _FlatNet.__init__(self)
                self._flatten()

        net = Net()
        net._flat.fill_(float(rank + 1))
        net.stat.fill_(float(rank + 7))
        broadcast_module(net)
        ok_bcast = bool(torch.all(net._flat == 1.0)) and bool(torch.all(net.stat == 7.0))
        g = torch.arange(net._flat_grad.numel(), dtype=torch.float32) * (rank + 1)
        net._flat_grad.copy_(g)
        red = GradAllReducer(net, bucket_mb=0)  # 1-float buckets: exercises many buckets
        red.buckets = [net._flat_grad[i:i + 4] for i in range(0, net._flat_grad.numel(), 4)]
        red()
        want = torch.arange(net._flat_grad.numel(), dtype=torch.float32) * 1.5
        ok_avg = bool(torch.allclose(net._flat_grad, want))
        ok_view = bool(torch.allclose(net.b.grad.reshape(-1) if net.b.grad is not None else want[5:17], want[5:17]))
        q.put((rank, ok_bcast, ok_avg, ok_view, shard_indices(10, rank, world)))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_grad_average_and_broadcast():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_bcast, ok_avg, ok_view, shard in res:
        assert ok_bcast and ok_avg and ok_view
    assert res[0][4] == [0, 2, 4, 6, 8] and res[1][4] == [1, 3, 5, 7, 9]


def test_rank_seeds_differ():
    from climsr_amd.core.ddp import rank_seed

    assert [rank_seed(42, r) for r in range(4)] == [42, 43, 44, 45]


def _ov_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from climsr_amd.core.ddp import OverlappedGradAllReducer

        class M:  # the reducer only needs the flat gradient buffer
            _flat_grad = torch.arange(20, dtype=torch.float32) * (rank + 1)

        red = OverlappedGradAllReducer(M())
        red.ready(14)   # [14, 20) final
        red.ready(14)   # repeated report: no new bucket
        red.ready(5)    # [5, 14)
        red.finish()    # [0, 5)
        buckets = list(red.launched)
        ok = bool(torch.allclose(M._flat_grad, torch.arange(20, dtype=torch.float32) * 1.5))
        red.finish()    # a step with no ready(): one whole-buffer bucket
        q.put((rank, ok, buckets, list(red.launched)))
    finally:
        dist.destroy_process_group()


def test_overlapped_reducer_gloo_world2():
    """Backward-overlapped DDP buckets (core/ddp.OverlappedGradAllReducer): the slices reported ready are
    reduced once each, in report order, and the step's result is the all-rank average."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ov_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    for rank, ok, buckets, second in res:
        assert ok, f"rank {rank}: averaged gradient mismatch"
        assert buckets == [(14, 20), (5, 14), (0, 5)], buckets
        assert second == [(0, 20)], second
