"""Parity of the step bench.py times (VERDICT r02 "next" #1).

The headline GAN step runs ``GraphedAdamW`` (AdamW + OneCycleLR with every scalar computed on the device by
``adamw_hparams_kernel``) and replays the step as hipGraph segments (``bench.make_runner``).  Every other step-level
test drives the eager path the reference's Lightning loop would: ``Trainer`` + zero-argument ``configure_optimizers()``
-> ``core.optim.AdamW`` stepped by torch's own ``OneCycleLR`` (conf/optimizers/adamw.yaml,
conf/schedulers/one_cycle_schedule.yaml, climsr/core/instantiator.py:48-64, climsr/task/pl_gan.py:63-97).

* ``test_adamw_hparams_kernel_vs_torch_onecycle``: the device schedule's lr, beta1, step size lr / (1 - beta1^t) and
  sqrt(1 - beta2^t) equal what torch's OneCycleLR + AdamW use, in fp32, for every step of two schedules (warm-up ->
  anneal boundary crossed; one run to the final step).
* ``test_timed_step_equals_eager_trainer``: the bench workload built by ``bench.build_train`` (nb 11, B 32, 64 -> 256:
  the headline shape) and replayed by ``bench.make_runner`` (2 eager warm-up steps + 3 graph replays; also with the
  split capture of the overlapped DDP path) lands on the same losses and the same fp32 parameters (bit-equal, or within
  1 ulp per element) and BatchNorm running statistics as 5 eager Trainer steps from the same state and batch.
"""
import math
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("total_steps,pct_start,n_steps", [(60, 0.05, 20), (20, 0.3, 20)])
def test_adamw_hparams_kernel_vs_torch_onecycle(total_steps, pct_start, n_steps):
    from climsr_amd import _lib

    lib = _lib.load()
    lr, div, fdiv, b2, eps, wd = 1e-4, 2.0, 100.0, 0.999, 1e-8, 1e-4
    state = torch.zeros(2, dtype=torch.float64, device=DEV)
    hp = torch.zeros(8, dtype=torch.float32, device=DEV)
    p = torch.nn.Parameter(torch.zeros(4))
    opt = torch.optim.AdamW([p], lr=lr, weight_decay=wd, betas=(0.9, b2), eps=eps)
    sch = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=lr, total_steps=total_steps, pct_start=pct_start, div_factor=div,
                                              final_div_factor=fdiv)
    end0 = pct_start * total_steps - 1
    phases = set()
    for t in range(1, n_steps + 1):
        _lib.check(lib.climsr_adamw_hparams(state.data_ptr(), total_steps, lr, pct_start, div, fdiv, b2, eps, wd, hp.data_ptr(),
                                            _lib.stream_ptr()), "adamw_hparams")
        got = hp.cpu().numpy()
        grp = opt.param_groups[0]
        lr_t, b1_t = grp["lr"], grp["betas"][0]
        # torch's single-tensor AdamW: step_size = lr / (1 - beta1^t), denom = sqrt(v) / sqrt(1 - beta2^t) + eps
        want = np.array([lr_t, b1_t, b2, eps, wd, lr_t / (1 - b1_t ** t), math.sqrt(1 - b2 ** t), 0.0], dtype=np.float32)
        ulp = np.abs(got.view(np.int32).astype(np.int64) - want.view(np.int32).astype(np.int64))
        assert ulp.max() <= 1, (t, got, want, ulp)
        phases.add("warmup" if t - 1 <= end0 else "anneal")
        p.grad = torch.zeros_like(p)
        opt.step()
        sch.step()
    assert phases == {"warmup", "anneal"}
    assert int(state[0].item()) == n_steps and int(state[1].item()) == n_steps
    if n_steps == total_steps:  # ran to the end: the final lr is initial_lr / final_div_factor
        assert abs(float(hp[0]) - lr / div / fdiv) <= 1e-6 * lr


def _ulp_diff(a, b):
    ai = a.contiguous().view(torch.int32).long()
    bi = b.contiguous().view(torch.int32).long()
    return (ai - bi).abs()


def _eager_module(bench, args, total_steps):
    """The same networks and initial state as bench.build_train, driven the Lightning way."""
    from climsr_amd.core.init import init_state, spec_from_shapes
    from climsr_amd.core.trainer import Trainer
    from climsr_amd.models.esrgan import ESRGANGenerator
    from climsr_amd.task.pl_gan import GANLightningModule

    g = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=args.nb, gc=16, scale_factor=4)
    st = init_state(spec_from_shapes({k: tuple(v.shape) for k, v in g.state_dict().items()}))
    g.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    adamw = {"_target_": "torch.optim.AdamW", "lr": 1e-4, "weight_decay": 1e-4}
    one_cycle = {"_target_": "torch.optim.lr_scheduler.OneCycleLR", "max_lr": 1e-4, "num_training_steps": total_steps,
                 "pct_start": 0.05, "div_factor": 2, "final_div_factor": 100}
    m = GANLightningModule(generator=g.to(DEV),
                           discriminator={"_target_": "climsr_amd.models.rfb_esrgan.RFBESRGANDiscriminator", "in_channels": 1},
                           optimizers={"generator_optimizer": dict(adamw), "discriminator_optimizer": dict(adamw)},
                           schedulers={"generator_scheduler": dict(one_cycle), "discriminator_scheduler": dict(one_cycle)})
    d = m.discriminator
    dst = init_state(spec_from_shapes({k: tuple(v.shape) for k, v in d.state_dict().items()},
                                      [n_ for n_, m_ in d.named_modules() if isinstance(m_, torch.nn.BatchNorm2d)]))
    d.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in dst.items()})
    m = m.to(DEV)
    return m, Trainer(m)


@pytest.mark.parametrize("overlap_split", [False, True])
def test_timed_step_equals_eager_trainer(monkeypatch, overlap_split):
    import bench

    if overlap_split:  # the overlapped-DDP structure at N = 1: grad-ready hooks split the captures (no-op reductions)
        monkeypatch.setenv("CLIMSR_DDP_OVERLAP_TEST", "1")
    else:
        monkeypatch.delenv("CLIMSR_DDP_OVERLAP_TEST", raising=False)
    args = bench.parse(["--steps", "3", "--warmup", "0", "--median-steps", "0"])
    dev = torch.device(DEV)
    w = bench.build_train(args, "gan", 1, dev)
    total_steps = max(1000, 2 * (args.warmup + args.steps + args.median_steps) + 10)  # build_train's schedule length
    rn = bench.make_runner(w, 1, dev, use_graph=True)  # 2 eager warm-up steps, then the capture
    assert rn["overlap"] == overlap_split
    if overlap_split:
        assert any(len(subs) > 1 for subs, _n in rn["graphs"]), "the grad-ready hooks did not split a capture"
    for _ in range(3):
        rn["run"]()
    torch.cuda.synchronize()
    timed = [float(v) for v in w["loss_buf"].cpu()]

    m, tr = _eager_module(bench, args, total_steps)
    assert tr.schedulers[0]["scheduler"].total_steps == total_steps
    B, hr = args.batch, 4 * args.lr_size
    gen = torch.Generator(device="cpu").manual_seed(42)  # build_train's batch (rank 0)
    t = torch.rand((B, 1, hr, hr), generator=gen) * 2 - 1
    e = torch.rand((B, 1, hr, hr), generator=gen) * 2 - 1
    msk = (torch.rand((B, 1, hr, hr), generator=gen) < 0.7).float()
    lr = torch.cat([t, e, msk], 1)[:, :, ::4, ::4].contiguous()
    batch = {k: v.to(dev) for k, v in {"lr": lr, "hr": t, "elevation": e, "mask": msk}.items()}
    for k in ("lr", "hr", "elevation", "mask"):
        assert torch.equal(batch[k], w["batch"][k]), k
    for i in range(5):
        out = tr.training_batch(batch, i)
    torch.cuda.synchronize()
    eager = [float(out[0]["loss"]), float(out[1]["loss"])]
    print("losses timed", timed, "eager", eager, flush=True)
    for a, b in zip(timed, eager):
        assert abs(a - b) <= 1e-6 * abs(b), (timed, eager)

    worst = {}
    for name, net_t, net_e in (("G", w["g"], m.generator), ("D", w["d"], m.discriminator)):
        u = _ulp_diff(net_t._flat, net_e._flat)
        worst[name] = (int(u.max()), int((u > 0).sum()))
        bt, be = dict(net_t.named_buffers()), dict(net_e.named_buffers())
        for k in be:
            if be[k].is_floating_point():
                ub = _ulp_diff(bt[k].float(), be[k].float())
                assert int(ub.max()) <= 1, (name, k, int(ub.max()))
            else:
                assert torch.equal(bt[k], be[k]), (name, k)
    print("parameter ulp differences (max, count):", worst, flush=True)
    assert all(v[0] <= 1 for v in worst.values()), worst
