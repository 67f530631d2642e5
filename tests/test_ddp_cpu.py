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


# ------------------------------------------------------------------ the real modules' flat layouts
def _real_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from climsr_amd.core.ddp import GradAllReducer, OverlappedGradAllReducer
        from climsr_amd.models.esrgan import ESRGANGenerator
        from climsr_amd.models.rfb_esrgan import RFBESRGANDiscriminator

        g = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=11, gc=16, scale_factor=4)
        d = RFBESRGANDiscriminator(in_channels=1)
        out = {}
        for name, net in (("G", g), ("D", d)):
            net.grads_as_views()

            def rank_grad(r, n=net._flat_grad.numel()):
                return torch.randn(n, generator=torch.Generator().manual_seed(1000 * r + len(name)))

            want = (rank_grad(0) + rank_grad(1)) / 2
            # (1) reduce-after-backward: 256 MB buckets (D's 430 MB buffer is 2 buckets)
            net._flat_grad.copy_(rank_grad(rank))
            red = GradAllReducer(net)
            nb_buckets = len(red.buckets)
            red()
            ok_bucketed = bool(torch.allclose(net._flat_grad, want, atol=1e-6))
            # (2) overlapped: the slices the native backwards report (G: RRDB blocks 8/5/2, D: fc.0 + fc.2 first)
            net._flat_grad.copy_(rank_grad(rank))
            ov = OverlappedGradAllReducer(net)
            if name == "G":
                net.set_grad_ready_hook(ov.ready)
                los = [net._block_flat_lo(b) for b in net._grad_ready_blocks]
            else:
                los = [net._fc_flat_lo()]
            for lo in los:
                ov.ready(lo)
            ov.finish()
            ok_overlap = bool(torch.allclose(net._flat_grad, want, atol=1e-6))
            # per-parameter .grad views see the averaged values (fc.0 / conv_first)
            p = net.fc[0].weight if name == "D" else net.conv_first.weight
            lo = [off for q_, off, _n in net._flat_index if q_ is p][0]
            ok_view = bool(torch.equal(p.grad.reshape(-1), net._flat_grad[lo:lo + p.numel()]))
            out[name] = (ok_bucketed, ok_overlap, ok_view, nb_buckets, list(ov.launched))
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_real_module_layouts():
    """DDP average on the real FlatParamsMixin layouts of ESRGANGenerator (nb 11, 4.28 M params) and
    RFBESRGANDiscriminator (107.4 M params): bucketed AVG and the backward-overlapped slices both give the
    average of the two ranks' gradient buffers, and every parameter's .grad view sees it."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_real_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, out in res:
        for name, (ok_b, ok_o, ok_v, nbk, launched) in out.items():
            assert ok_b and ok_o and ok_v, (rank, name)
        assert out["D"][3] == 2  # 430 MB fp32 gradient in 256 MB buckets
        g_slices = out["G"][4]
        assert len(g_slices) == 4 and g_slices[-1][0] == 0 and all(a[0] == b[1] for a, b in zip(g_slices, g_slices[1:]))
        d_slices = out["D"][4]
        assert len(d_slices) == 2 and d_slices[0][1] - d_slices[0][0] == 1024 * 100352 + 1024 + 1024 + 1


# ------------------------------------------------------------------ bench.py --gpus N launcher
def test_bench_child_envs():
    import bench

    envs = bench.child_envs(4, 29555, base={"PATH": "/usr/bin"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555" for e in envs)
    assert all(e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" and e["PATH"] == "/usr/bin" for e in envs)


def test_bench_launcher_fans_out(tmp_path):
    """bench.launch starts one child per rank with torchrun's variables and returns 0 when all succeed."""
    import sys

    import bench

    code = ("import os; p = os.path.join(%r, 'rank' + os.environ['RANK']); "
            "open(p, 'w').write(' '.join(os.environ[k] for k in ('LOCAL_RANK', 'WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT')))"
            % str(tmp_path))
    assert bench.launch(3, [sys.executable, "-c", code], timeout=60) == 0
    got = sorted(os.listdir(tmp_path))
    assert got == ["rank0", "rank1", "rank2"]
    ports = set()
    for r in range(3):
        lr, ws, addr, port = open(tmp_path / f"rank{r}").read().split()
        assert (lr, ws, addr) == (str(r), "3", "127.0.0.1")
        ports.add(port)
    assert len(ports) == 1


def test_bench_launcher_propagates_failure():
    import sys

    import bench

    code = "import os, sys, time; r = int(os.environ['RANK']); sys.exit(3) if r == 1 else time.sleep(30)"
    t0 = __import__("time").time()
    assert bench.launch(2, [sys.executable, "-c", code], timeout=60) == 3
    assert __import__("time").time() - t0 < 20  # the surviving rank was killed, not waited for


def test_bench_main_without_world_size_launches(monkeypatch):
    """`python bench.py --gpus N` (no WORLD_SIZE in the environment) goes through the launcher with N ranks."""
    import bench

    seen = {}
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    monkeypatch.setattr(bench, "launch", lambda n, cmd, timeout=None: seen.update(n=n, cmd=cmd) or 0)
    assert bench.main(["--gpus", "8", "--steps", "3"]) == 0
    assert seen["n"] == 8 and seen["cmd"][-4:] == ["--gpus", "8", "--steps", "3"]


# ------------------------------------------------------------------ world-2 step == single-process step
def _dp_step_worker(rank, world, port, q):
    """One data-parallel L1-pretrain step (config 4's algorithm, pl_generator_pre_training.py:18-33): each rank
    takes its shard of the batch, its gradient goes through the real ESRGANGenerator flat layout and the
    product's GradAllReducer, then AdamW.  The per-shard arithmetic is the fp64 oracle (the HIP kernels need a
    GPU; their parity is the -m gpu suite) — what this checks is the data-parallel decomposition itself."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from climsr_amd.core.ddp import GradAllReducer, shard_indices
        from climsr_amd.models.esrgan import ESRGANGenerator
        from oracle import climsr_ref as ref
        from tests.helpers import gen_params

        nb, batch, hr = 1, 4, 32
        p_ref = gen_params(nb, torch.float64)
        g = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=nb, gc=16, scale_factor=4)
        g.load_state_dict({k: v.float() for k, v in p_ref.items()})
        g.grads_as_views()
        keys = ref.trainable_keys(p_ref)
        data = ref.synthetic_batch(batch, hr, dtype=torch.float64)

        def grads_on(idx):
            p = {k: v.clone().requires_grad_(k in keys) for k, v in p_ref.items()}
            sr = ref.generator_forward(p, data["lr"][idx], data["elevation"][idx], data["mask"][idx], nb)
            return ref._grads(ref.l1_loss(sr, data["hr"][idx]), p, keys)

        shard = shard_indices(batch, rank, world)
        local = grads_on(shard)
        for name, prm in g.named_parameters():
            prm.grad.copy_(local[name])
        GradAllReducer(g)()
        avg = {name: prm.grad.double().clone() for name, prm in g.named_parameters()}
        full = grads_on(list(range(batch)))
        num = sum(float((avg[k] - full[k]).norm() ** 2) for k in keys) ** 0.5
        den = sum(float(full[k].norm() ** 2) for k in keys) ** 0.5
        # one optimizer step from the averaged gradient vs the single-process step on the whole batch
        p_dp = {k: v.clone() for k, v in p_ref.items()}
        ref.AdamWState(p_dp, keys, 2e-4, 100).step(p_dp, avg)
        p_sp = {k: v.clone() for k, v in p_ref.items()}
        ref.pretrain_step(p_sp, ref.AdamWState(p_sp, keys, 2e-4, 100), data, nb)
        dp_max = max(float((p_dp[k] - p_sp[k]).abs().max()) for k in keys)
        q.put((rank, shard, num / den, dp_max, float(sum(avg[k].sum() for k in keys))))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_step_equals_concatenated_batch():
    """World-2 DP gradient (each rank's shard, averaged over gloo through the product reducer and the
    generator's flat layout) equals the single-process gradient of the concatenated batch, and one AdamW step
    from it lands on the single-process step's parameters (within fp32 rounding of the flat buffer)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_step_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, s0, rel0, dmax0, sum0), (_, s1, rel1, dmax1, sum1) = res
    assert sorted(s0 + s1) == [0, 1, 2, 3] and not set(s0) & set(s1)
    assert rel0 < 1e-6 and rel1 < 1e-6, (rel0, rel1)
    assert dmax0 < 2e-4 * 1e-3 and dmax1 < 2e-4 * 1e-3, (dmax0, dmax1)  # << lr: same update direction
    assert sum0 == sum1  # both ranks hold the identical averaged gradient


def test_bench_launcher_times_out_hung_rank():
    """A rank that never exits is killed at the launcher's limit (exit 124) instead of hanging the run."""
    import sys
    import time

    import bench

    assert bench.launch.__defaults__[0] == bench.LAUNCH_TIMEOUT_S and bench.LAUNCH_TIMEOUT_S > 0  # on by default
    code = "import time; time.sleep(120)"
    t0 = time.time()
    assert bench.launch(2, [sys.executable, "-c", code], timeout=3) == 124
    assert time.time() - t0 < 30


# ------------------------------------------------------------------ world-2 GAN discriminator pass
def _gan_d_worker(rank, world, port, q):
    """The D pass of one GAN step (pl_gan.py:51-61 loss_d, then AdamW_D) as Lightning DDP runs it: each rank takes
    its shard, D's BatchNorms use the shard's batch statistics (no SyncBN, conf/trainer/default.yaml:31) and the
    relativistic means are over the shard; the per-rank D gradients (fp64 oracle arithmetic; the HIP kernels need a
    GPU) are written into the real RFBESRGANDiscriminator flat gradient buffer and averaged by the product's
    overlapped reducer with the slices D's backward reports (fc first, then the rest)."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from climsr_amd.core.ddp import OverlappedGradAllReducer, shard_indices
        from climsr_amd.models.rfb_esrgan import RFBESRGANDiscriminator
        from oracle import climsr_ref as ref
        from tests.helpers import rfb_d_params

        torch.set_num_threads(2)
        batch, hr = 4, 32
        p0 = rfb_d_params(torch.float64)
        keys = ref.trainable_keys(p0)
        data = ref.synthetic_batch(batch, hr, seed=9, dtype=torch.float64)
        sr_all = torch.tanh(torch.randn((batch, 1, hr, hr), generator=torch.Generator().manual_seed(11), dtype=torch.float64))

        def d_pass(idx):
            p = {k: (v.clone().requires_grad_(k in keys) if v.is_floating_point() else v.clone()) for k, v in p0.items()}
            ld = ref.loss_d(lambda t: ref.rfb_discriminator_forward(p, t, training=True), data["hr"][idx], sr_all[idx])
            grads = ref._grads(ld, p, keys)
            stats = torch.cat([p[pre + ".running_mean"] for pre in ref.rfb_bn_prefixes()]).detach()
            return float(ld), grads, stats

        shard = shard_indices(batch, rank, world)
        loss, local, stats = d_pass(shard)
        d = RFBESRGANDiscriminator(in_channels=1)
        d.grads_as_views()
        for k, prm in d.named_parameters():
            prm.grad.copy_(local[k])
        ov = OverlappedGradAllReducer(d)
        los = d.grad_ready_los()  # the slices the native backward reports, in its order: fc, then conv layer groups
        for lo in los:
            ov.ready(lo)
        ov.finish()
        avg = {k: prm.grad.double().clone() for k, prm in d.named_parameters()}
        # expected: the mean of the two shards' gradients, each with its own BN statistics (computed here in one process)
        shards = [shard_indices(batch, r, world) for r in range(world)]
        per = [d_pass(s) for s in shards]
        want = {k: sum(pp[1][k] for pp in per) / world for k in keys}
        whole = d_pass(list(range(batch)))[1]

        def rel(a, b):
            num = sum(float((a[k] - b[k]).norm() ** 2) for k in keys) ** 0.5
            return num / (sum(float(b[k].norm() ** 2) for k in keys) ** 0.5)

        # each reported slice holds exactly the parameters that are final at that point: fc.*, then features.17 ..
        # (conv 6, its BN, conv 7, its BN), then features.8 .. features.15, then the rest at finish()
        names = {}
        for (prm, off, num), (k, _p) in zip(d._flat_index, d.named_parameters()):
            names[k] = (off, off + num)
        slices = []
        for lo, hi in ov.launched:
            slices.append(sorted(k for k, (a, b) in names.items() if a >= lo and b <= hi))
        q.put((rank, shard, loss, rel(avg, want), rel(want, whole), stats, per[rank][2], list(ov.launched), slices, los))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_gan_discriminator_pass():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gan_d_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=600) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, shard, loss, rel_avg, rel_whole, stats, stats_check, launched, slices, los in res:
        assert rel_avg < 1e-6, (rank, rel_avg)  # product reducer + D flat layout: the average of the per-shard gradients
        assert rel_whole > 1e-3, (rank, rel_whole)  # per-rank BN statistics: not the whole-batch (SyncBN) gradient
        assert torch.equal(stats, stats_check)
        assert len(launched) == 4 and launched[0][1] - launched[0][0] == 1024 * 100352 + 1024 + 1024 + 1
        assert [lo for lo, _hi in launched] == los + [0] and los == sorted(los, reverse=True)
        # contiguous, descending, covering the whole flat buffer
        assert all(launched[i][0] == launched[i + 1][1] for i in range(3))
        assert slices[0] == ["fc.0.bias", "fc.0.weight", "fc.2.bias", "fc.2.weight"]
        assert slices[1] == ["features.17.weight", "features.18.bias", "features.18.weight", "features.20.weight",
                             "features.21.bias", "features.21.weight"]
        assert slices[2][0] == "features.11.weight" and "features.8.weight" in slices[2] and "features.15.weight" in slices[2]
        assert "features.0.weight" in slices[3] and "features.6.weight" in slices[3]
    assert res[0][1] == [0, 2] and res[1][1] == [1, 3]
    assert not torch.allclose(res[0][5], res[1][5])  # each rank's running statistics follow its own shard
    assert res[0][2] != res[1][2]  # and so do the per-rank losses


# ------------------------------------------------------------------ world-2 GAN generator pass
def _gan_g_worker(rank, world, port, q):
    """The G pass of one GAN step (pl_gan.py:28-49 loss_g, then AdamW_G) as Lightning DDP runs it: each rank takes its
    shard, D (frozen, train mode) is called separately on hr and sr with the shard's BatchNorm statistics (no SyncBN,
    conf/trainer/default.yaml:31), the relativistic means are over the shard, and G's gradient flows through D(sr) and
    the pixel loss (the perceptual loss carries none, F7).  The per-rank G gradients (fp64 oracle arithmetic; the HIP
    kernels need a GPU) go into the real ESRGANGenerator flat gradient buffer and are averaged by the product's
    overlapped reducer at the slice the generator's backward reports (after RRDB block 1 of 2), then at finish."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from climsr_amd.core.ddp import OverlappedGradAllReducer, shard_indices
        from climsr_amd.models.esrgan import ESRGANGenerator
        from oracle import climsr_ref as ref
        from tests.helpers import gen_params, rfb_d_params, vgg_params

        torch.set_num_threads(2)
        nb, batch, hr = 2, 4, 32
        g0 = gen_params(nb, torch.float64)
        d0 = rfb_d_params(torch.float64)
        vp = vgg_params(torch.float64)
        keys = ref.trainable_keys(g0)
        data = ref.synthetic_batch(batch, hr, seed=5, dtype=torch.float64)

        def g_pass(idx):
            p = {k: v.clone().requires_grad_(True) for k, v in g0.items()}
            dp = {k: v.clone() for k, v in d0.items()}  # D frozen in the G pass (Lightning toggles requires_grad)
            sr = ref.generator_forward(p, data["lr"][idx], data["elevation"][idx], data["mask"][idx], nb)
            _perc, _adv, _pix, total = ref.loss_g(lambda t: ref.rfb_discriminator_forward(dp, t, training=True), vp,
                                                  data["hr"][idx], sr)
            return float(total), ref._grads(total, p, keys)

        shard = shard_indices(batch, rank, world)
        loss, local = g_pass(shard)
        g = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=nb, gc=16, scale_factor=4)
        g.grads_as_views()
        for k, prm in g.named_parameters():
            prm.grad.copy_(local[k])
        ov = OverlappedGradAllReducer(g)
        g.set_grad_ready_hook(ov.ready)
        for b in g._grad_ready_blocks:  # the slices the native backward reports, in its order
            ov.ready(g._block_flat_lo(b))
        ov.finish()
        avg = {k: prm.grad.double().clone() for k, prm in g.named_parameters()}
        shards = [shard_indices(batch, r, world) for r in range(world)]
        per = [g_pass(s) for s in shards]
        want = {k: sum(pp[1][k] for pp in per) / world for k in keys}
        whole = g_pass(list(range(batch)))[1]

        def rel(a, b):
            num = sum(float((a[k] - b[k]).norm() ** 2) for k in keys) ** 0.5
            return num / (sum(float(b[k].norm() ** 2) for k in keys) ** 0.5)

        q.put((rank, shard, loss, rel(avg, want), rel(want, whole), list(ov.launched)))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_gan_generator_pass():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gan_g_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=600) for _ in procs), key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, shard, loss, rel_avg, rel_whole, launched in res:
        assert rel_avg < 1e-6, (rank, rel_avg)  # product reducer + G flat layout: the average of the per-shard gradients
        # per-rank relativistic means and BN statistics in loss_g: not the gradient of the whole batch
        assert rel_whole > 1e-4, (rank, rel_whole)
        assert len(launched) == 2 and launched[-1][0] == 0 and launched[0][0] == launched[1][1]
    assert res[0][1] == [0, 2] and res[1][1] == [1, 3]
    assert res[0][2] != res[1][2]  # per-rank losses
