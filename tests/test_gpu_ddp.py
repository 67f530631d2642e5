"""The native modules under torch ``DistributedDataParallel`` — the reference's multi-GPU mechanism
(conf/trainer/benchmark.yaml:3-5, ``accelerator: ddp``: Lightning wraps the whole LightningModule in one DDP with
``find_unused_parameters=True`` and calls ``training_step`` inside its forward; conf/trainer/default.yaml:31,42).

World 1 on the one GPU over the ``nccl`` backend (RCCL).  Inside a DDP forward the native G / D hand their parameter
gradients to autograd (core/flat.py ``grads_through_autograd``), so DDP's AccumulateGrad hooks fire and its buckets
reduce them.  Each step (both optimizer passes of pl_gan.py:63-97, Lightning-1.x toggling) is compared with the
unwrapped ``Trainer`` step from the same state: gradients per tensor, the flat-buffer views the fused AdamW needs, and
the parameters after AdamW + OneCycleLR.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist

pytestmark = pytest.mark.gpu
DEV = "cuda"
NB, BATCH, HR = 1, 4, 128
ADAMW = {"_target_": "torch.optim.AdamW", "lr": 1e-4, "weight_decay": 1e-4}
ONE_CYCLE = {"_target_": "torch.optim.lr_scheduler.OneCycleLR", "max_lr": 1e-4, "num_training_steps": 50, "pct_start": 0.05,
             "div_factor": 2, "final_div_factor": 100}


@pytest.fixture(scope="module")
def nccl_world1():
    if dist.is_initialized():
        yield
        return
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1,
                            device_id=torch.device("cuda", 0))
    yield
    dist.destroy_process_group()


def _task():
    from tests.helpers import gen_params, rfb_d_params
    from climsr_amd.task.pl_gan import GANLightningModule

    m = GANLightningModule(
        generator={"_target_": "climsr_amd.models.esrgan.ESRGANGenerator", "in_channels": 3, "out_channels": 1, "nf": 64, "nb": NB,
                   "gc": 16, "scale_factor": 4},
        discriminator={"_target_": "climsr_amd.models.rfb_esrgan.RFBESRGANDiscriminator", "in_channels": 1},
        optimizers={"generator_optimizer": dict(ADAMW), "discriminator_optimizer": dict(ADAMW)},
        schedulers={"generator_scheduler": dict(ONE_CYCLE), "discriminator_scheduler": dict(ONE_CYCLE)})
    m.generator.load_state_dict(gen_params(NB, torch.float32))
    m.discriminator.load_state_dict(rfb_d_params(torch.float32))
    return m.to(DEV)


class _LightningDDPModule(torch.nn.Module):
    """What Lightning 1.x's LightningDistributedModule does: DDP.forward -> training_step."""

    def __init__(self, task):
        super().__init__()
        self.module = task

    def forward(self, batch, batch_idx, optimizer_idx):
        return self.module.training_step(batch, batch_idx, optimizer_idx)


def _rel(a, b):
    return float((a.double() - b.double()).norm() / (b.double().norm() + 1e-30))


def _is_flat_view(net, grads):
    base = grads[0].untyped_storage().data_ptr()
    off = grads[0].storage_offset()
    for (p, _o, n), g in zip(net._flat_index, grads):
        if g is None or g.untyped_storage().data_ptr() != base or g.storage_offset() != off or not g.is_contiguous():
            return False
        off += n
    return True


@pytest.mark.parametrize("set_to_none", [True, False])
def test_gan_steps_under_torch_ddp_equal_unwrapped(nccl_world1, set_to_none):
    from climsr_amd.core.trainer import Trainer
    from oracle import climsr_ref as ref

    plain = _task()
    tr = Trainer(plain)
    wrapped = _task()
    trw = Trainer(wrapped)  # configure_optimizers() on the wrapped task: the same AdamW / OneCycleLR objects Lightning builds
    ddp = torch.nn.parallel.DistributedDataParallel(_LightningDDPModule(wrapped), device_ids=[0], find_unused_parameters=True)
    nets_p = [plain.generator, plain.discriminator]
    nets_w = [wrapped.generator, wrapped.discriminator]
    for step in range(2):
        bt = {k: v.to(DEV) for k, v in ref.synthetic_batch(BATCH, HR, seed=100 + step).items()}
        outs_p = tr.training_batch(bt, step)  # unwrapped: grads written in place into the flat buffers
        for i, opt in enumerate(trw.optimizers):  # Lightning-1.x automatic optimisation around the DDP forward
            trw._toggle(i)
            opt.zero_grad(set_to_none=set_to_none)
            out = ddp(bt, step, i)
            out["loss"].backward()
            net_w, net_p = nets_w[i], nets_p[i]
            grads = [p.grad for p, _o, _n in net_w._flat_index]
            assert all(g is not None for g in grads), f"step {step} opt {i}: DDP left a gradient unset"
            # G (one node per pass): autograd took the native gradient buffer's views as they are (no copy); D (called
            # on real and fake: two nodes) has its two contributions summed by autograd into separate tensors, which
            # the fused AdamW gathers into the flat buffer before its one-launch update
            if i == 0:
                assert _is_flat_view(net_w, grads), f"step {step}: G gradients are not one flat buffer"
            launches = []
            from climsr_amd import ops
            ops.PROFILER = lambda name, flops, fn, tag="", nbytes=0: (launches.append(name), fn())
            try:
                opt.step()
            finally:
                ops.PROFILER = None
            assert launches.count("adamw") == 1, (step, i, launches)
            lw, lp = float(out["loss"]), float(outs_p[i]["loss"])
            assert abs(lw - lp) <= 1e-6 * abs(lp), (step, i, lw, lp)
        for net in nets_w:
            for p in net.parameters():
                p.requires_grad_(True)
        for s in trw.schedulers:
            s["scheduler"].step()
        torch.cuda.synchronize()
        for name, a, b in (("G", nets_w[0], nets_p[0]), ("D", nets_w[1], nets_p[1])):
            # gradients of the last pass of each network: same kernels, same inputs; the D pass sums its two calls
            # (real / fake) in autograd instead of in the kernel epilogue: equal up to fp32 addition order
            ga = {k: p.grad for k, p in a.named_parameters()}
            gb = {k: p.grad for k, p in b.named_parameters()}
            worst = max((_rel(ga[k], gb[k]), k) for k in gb)
            assert worst[0] <= 1e-6, (step, name, worst)
            rel_p = max(_rel(pa, pb) for pa, pb in zip(a.parameters(), b.parameters()))
            u = (a._flat.view(torch.int32).long() - b._flat.view(torch.int32).long()).abs()
            print(f"step {step} {name}: worst grad rel {worst[0]:.2e} ({worst[1]}), param ulp max {int(u.max())}, "
                  f"param rel {rel_p:.2e}", flush=True)
            assert int(u.max()) <= 1, (step, name, int(u.max()))
    # the running statistics of D's BatchNorms (per rank, no SyncBN: conf/trainer/default.yaml:31)
    for (k, va), vb in zip(wrapped.discriminator.named_buffers(), plain.discriminator.buffers()):
        if va.is_floating_point():
            assert torch.allclose(va, vb, rtol=1e-6, atol=1e-7), k
        else:
            assert torch.equal(va, vb), k


def test_ddp_forward_switches_gradient_route(nccl_world1):
    """Outside DDP the generator writes its gradients in place (no AccumulateGrad); inside a DDP forward they go
    through autograd; ``grads_through_autograd`` overrides both ways."""
    from climsr_amd.core.flat import ddp_forward_active
    from climsr_amd.models.esrgan import ESRGANGenerator
    from oracle import climsr_ref as ref
    from tests.helpers import gen_params

    g = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=NB, gc=16, scale_factor=4)
    g.load_state_dict(gen_params(NB, torch.float32))
    g = g.to(DEV)
    bt = {k: v.to(DEV) for k, v in ref.synthetic_batch(2, 64, seed=3).items()}
    assert not ddp_forward_active()

    def grads_of(fn):
        for p in g.parameters():
            p.grad = None
        fn(g, bt).abs().mean().backward()
        torch.cuda.synchronize()
        return torch.cat([p.grad.reshape(-1) for p in g.parameters()]).clone()

    ref_grads = grads_of(lambda net, b: net(b["lr"], b["elevation"], b["mask"]))
    assert g.conv_first.weight.grad.data_ptr() == g._flat_grad.data_ptr()  # in place: the module's own flat buffer
    g.grads_through_autograd = True
    via = grads_of(lambda net, b: net(b["lr"], b["elevation"], b["mask"]))
    assert g.conv_first.weight.grad.data_ptr() != g._flat_grad.data_ptr()  # stolen views of the fresh buffer
    assert torch.equal(via, ref_grads)
    g.grads_through_autograd = None

    class Wrap(torch.nn.Module):
        def __init__(self, net):
            super().__init__()
            self.net = net

        def forward(self, b):
            assert ddp_forward_active()
            return self.net(b["lr"], b["elevation"], b["mask"])

    ddp = torch.nn.parallel.DistributedDataParallel(Wrap(g), device_ids=[0])
    in_ddp = grads_of(lambda net, b: ddp(b))
    assert torch.equal(in_ddp, ref_grads)
    np.testing.assert_equal(ddp_forward_active(), False)
