"""GPU parity for the BASELINE configs not covered elsewhere.

* config 1 (BASELINE.json configs[0]): the RRDB generator of conf/generator/esrgan.yaml (nb 11) pixel-loss-only,
  32 -> 128, batch 2, driven the way Lightning drives it: ``SuperResolutionLightningModule.training_step``
  (reference climsr/task/pl_generator_pre_training.py:18-33) through the built-in Trainer with the zero-argument
  ``configure_optimizers()`` built from conf/optimizers/adamw.yaml + conf/schedulers/one_cycle_schedule.yaml
  (task.py:173-226).  The reference runs this config on the CPU; this product is GPU-only (no CPU fallback, by
  design), so config 1 runs here on the GPU against tests/golden/config1_steps.json (the reference's own module in
  float64, tests/golden/make_config1_golden.py) and the fp64 oracle's three steps.
* config 5: whole-grid inference, LR 720x360 -> HR 2880x1440 (reference climsr/inference/inference.py:48,62-70,168:
  a plain fp32 forward of the whole grid) for the ESRGAN generator (nb 11) and RCAN 10x20 (conf/inference.yaml's
  default), against the oracle's forward evaluated in fp32 with torch ops on the GPU (test-only checker).  The
  product computes in bf16 with fp32 accumulation (config 5 names fp16: same width, declared in DESIGN.md).
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import climsr_ref as ref
from tests.helpers import gemm_conv, gen_params, psnr, scalar_cap, update_envelope

pytestmark = pytest.mark.gpu
DEV = "cuda"

ADAMW_YAML = {"_target_": "torch.optim.AdamW", "lr": 1e-4, "weight_decay": 1e-4}
POOL_BELOW = 256  # gradients of fewer elements (the biases) are compared pooled (helpers.pool_small)
ONE_CYCLE_YAML = {"_target_": "torch.optim.lr_scheduler.OneCycleLR", "max_lr": 1e-4, "num_training_steps": -1, "epochs": 1,
                  "pct_start": 0.05, "div_factor": 2, "final_div_factor": 100}


def test_config1_trainer_steps_vs_golden(golden_dir, monkeypatch):
    from climsr_amd.core.trainer import Trainer
    from climsr_amd.task.pl_generator_pre_training import SuperResolutionLightningModule

    want = json.load(open(os.path.join(golden_dir, "config1_steps.json")))
    nb, b, hr = want["nb"], want["batch"], want["hr_size"]
    m = SuperResolutionLightningModule(
        generator={"_target_": "climsr_amd.models.esrgan.ESRGANGenerator", "in_channels": 3, "out_channels": 1, "nf": 64,
                   "nb": nb, "gc": 16, "scale_factor": 4},
        optimizers={"generator_optimizer": dict(ADAMW_YAML)},
        schedulers={"generator_scheduler": dict(ONE_CYCLE_YAML)})
    p64 = gen_params(nb, torch.float64)
    m.generator.load_state_dict({k: v.float() for k, v in p64.items()})
    m = m.to(DEV)
    before = {k: v.detach().double().cpu().clone() for k, v in m.generator.named_parameters()}
    # Lightning's Trainer(limit_train_batches=10, max_epochs=1): num_training_steps -> 10 (task.py:61-83)
    tr = Trainer(m, limit_train_batches=want["total_steps"], max_epochs=1)
    assert tr.schedulers[0]["scheduler"].total_steps == want["total_steps"]
    batches = [{k: v.to(DEV) for k, v in ref.synthetic_batch(b, hr, seed=s).items()} for s in want["seeds"]]
    losses, lrs, states, grads = [], [], [], []
    for i, bt in enumerate(batches):
        lrs.append(tr.optimizers[0].param_groups[0]["lr"])
        states.append({k: v.detach().double().cpu().clone() for k, v in m.generator.named_parameters()})
        out = tr.training_batch(bt, i)
        losses.append(float(out[0]))
        grads.append({k: v.grad.double().cpu().clone() for k, v in m.generator.named_parameters()})
    torch.cuda.synchronize()
    states.append({k: v.detach().double().cpu().clone() for k, v in m.generator.named_parameters()})
    print("config-1 losses", losses, "want", want["loss"])
    for i, (got, w) in enumerate(zip(losses, want["loss"])):
        scalar_cap(f"config-1 step {i} L1 loss vs reference fixture", got, w)
    assert np.allclose(lrs, want["lr"], rtol=1e-9), (lrs, want["lr"])
    assert "train/loss" in m.logged
    lr = 1e-4
    sums, norms = {}, {}
    for k, p in m.generator.named_parameters():
        n = p.numel()
        pa = p.detach().double().cpu()
        sums[k] = abs(float(pa.sum() - before[k].sum()) - (want["params_after"][k][0] - float(before[k].sum()))) / n / lr
        norms[k] = abs(float(pa.norm()) - want["params_after"][k][1]) / n ** 0.5 / lr
    ws, wn = max(sums.items(), key=lambda kv: kv[1]), max(norms.items(), key=lambda kv: kv[1])
    print("config-1 worst per-tensor |dsum|/n/lr", ws, "|dnorm|/sqrt(n)/lr", wn)
    assert ws[1] <= 0.25, ws
    assert wn[1] <= 0.25, wn
    # Each step, split into the two things the product computes (CPU oracle, test-only):
    # (a) the gradient at the native parameters of that step vs the fp64 oracle's gradient at the same parameters, per
    #     tensor within 2x the deviation of the oracle's own reduced-precision runs at that point -- torch autocast fp16
    #     with the loss scaled as precision=16's GradScaler scales it (init scale 2^16), and autocast bf16, each over
    #     the whole batch and as two half-batch passes (their spread is the statistic's own noise level); the biases
    #     (16-64 elements, each a sum over 2 x 32 x 32 or more pixels of mostly cancelling terms) are compared pooled;
    # (b) the fused AdamW + OneCycleLR update given those native gradients vs the same update in fp64.
    # (Comparing whole 3-step update vectors instead mixes the two: Adam's first steps move every element by ~lr *
    # sign(grad), so the few near-zero gradient elements of a 64-element bias flip at random between runs.)
    torch.set_num_threads(min(16, os.cpu_count() or 1))
    keys = list(before.keys())

    def oracle_grads(state, bt, dev, dtype, autocast=None, scale=1.0, halves=False):
        """Gradient of the L1 loss at `state`; halves: the two batch halves' contributions computed separately and
        summed (the same math in another accumulation order: a second, equally valid reduced-precision sample)."""
        q = {k: v.to(dev, dtype).requires_grad_(True) for k, v in state.items()}
        b_ = {k: v.to(dev, dtype) for k, v in bt.items()}
        parts = [slice(0, b // 2), slice(b // 2, b)] if halves else [slice(0, b)]
        out = {k: 0.0 for k in keys}
        for sl in parts:
            with torch.autocast("cuda", dtype=autocast or torch.float16, enabled=autocast is not None):
                sr = ref.generator_forward(q, b_["lr"][sl], b_["elevation"][sl], b_["mask"][sl], nb)
            loss = ref.l1_loss(sr.to(dtype), b_["hr"][sl]) * ((sl.stop - sl.start) / b)
            gs = torch.autograd.grad(loss * scale, [q[k] for k in keys])
            for k, g in zip(keys, gs):
                out[k] = out[k] + g.double().cpu() / scale
        assert all(torch.isfinite(g).all() for g in out.values()), "loss scale overflowed"
        return out

    opt64 = ref.AdamWState({k: v.clone() for k, v in before.items()}, keys, lr=lr, total_steps=want["total_steps"])
    for i, s in enumerate(want["seeds"]):
        bt64 = ref.synthetic_batch(b, hr, seed=s, dtype=torch.float64)
        g64 = oracle_grads(states[i], bt64, "cpu", torch.float64)
        with monkeypatch.context() as mp:
            mp.setattr(ref, "_conv", gemm_conv)  # rocBLAS GEMMs on the GPU (no MIOpen per-shape compiles)
            torch.backends.cuda.matmul.allow_tf32 = False
            amps = [oracle_grads(states[i], bt64, DEV, torch.float32, dt, scale=sc, halves=hv)
                    for dt, sc in ((torch.float16, 2.0 ** 16), (torch.bfloat16, 1.0)) for hv in (False, True)]
        bad, worst, rows = update_envelope(grads[i], g64, amps, pool_below=POOL_BELOW)
        rels = sorted(r for r, _ra in rows.values())
        ratios = sorted(r / ra for r, ra in rows.values())
        print(f"config-1 step {i} gradient rel L2 vs fp64 over {len(rows)} tensors: worst {worst}, median "
              f"{rels[len(rels) // 2]:.3e}; native / envelope median {ratios[len(ratios) // 2]:.2f} max {ratios[-1]:.2f}", flush=True)
        assert not bad, f"step {i}: {len(bad)} gradients outside 2x the autocast deviation: {bad[:8]}"
        q = {k: v.clone() for k, v in states[i].items()}
        opt64.step(q, grads[i])
        opt64.sched()
        upd = {k: (states[i + 1][k] - states[i][k], q[k] - states[i][k]) for k in keys}
        worst_u = max((float((a - e).norm() / (e.norm() + 1e-30)), k) for k, (a, e) in upd.items())
        print(f"config-1 step {i} AdamW update rel L2 vs fp64 (native gradients): {worst_u}", flush=True)
        assert worst_u[0] <= 1e-3, worst_u


def _grid(h, w, seed=42):
    g = torch.Generator().manual_seed(seed)
    t = torch.rand((1, 1, 4 * h, 4 * w), generator=g) * 2 - 1
    e = torch.rand((1, 1, 4 * h, 4 * w), generator=g) * 2 - 1
    m = (torch.rand((1, 1, 4 * h, 4 * w), generator=g) < 0.7).float()
    lr = torch.cat([t, e, m], 1)[:, :, ::4, ::4].contiguous()
    return lr.to(DEV), e.to(DEV), m.to(DEV)


def _stats(got, want):
    got, want = got.double(), want.double()
    gc, wc = got - got.mean(), want - want.mean()
    return psnr(got, want), float((gc * wc).sum() / (gc.norm() * wc.norm())), float((got - want).norm() / want.norm())


def _compare(got, want, amps_fn, what, min_psnr=50.0):
    """Native vs the fp32 oracle: PSNR >= min_psnr dB and centred correlation >= 0.999, OR inside the envelope of the
    reference's own reduced-precision inference (config 5 runs the reference in fp16: the oracle under torch
    autocast fp16 / bf16 on the same grid) -- relative L2 <= 2x the worse autocast run's and correlation no worse
    than 1 - 2 (1 - its correlation)."""
    assert got.shape == want.shape, (got.shape, want.shape)
    assert torch.isfinite(got).all(), what
    p, corr, rel = _stats(got, want)
    print(f"{what}: PSNR {p:.2f} dB, corr {corr:.6f}, rel L2 {rel:.2e}", flush=True)
    if p >= min_psnr and corr >= 0.999:
        return
    amp = [_stats(a, want) for a in amps_fn()]  # only needed when the absolute bar is missed
    rel_amp, corr_amp = max(a[2] for a in amp), min(a[1] for a in amp)
    print(f"{what}: autocast fp16/bf16: " + ", ".join(f"PSNR {a[0]:.2f} dB corr {a[1]:.6f} rel {a[2]:.2e}" for a in amp), flush=True)
    ok_amp = rel <= 2.0 * rel_amp and corr >= 1.0 - 2.0 * (1.0 - corr_amp)
    assert ok_amp, f"{what}: PSNR {p:.2f} dB, centred correlation {corr:.6f}, rel L2 {rel:.2e} (autocast {amp})"


def _autocast_runs(fn):
    outs = []
    for dt in (torch.float16, torch.bfloat16):
        with torch.no_grad(), torch.autocast("cuda", dtype=dt):
            outs.append(fn().float())
    return outs


@pytest.fixture
def fp32_torch():
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False


def test_config5_esrgan_whole_grid_vs_oracle_fp32(fp32_torch):
    from climsr_amd.models.esrgan import ESRGANGenerator

    nb, h, w = 11, 360, 720
    p32 = gen_params(nb, torch.float32)
    net = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=nb, gc=16, scale_factor=4)
    net.load_state_dict(p32)
    net = net.to(DEV).eval()
    lr, e, m = _grid(h, w)
    with torch.no_grad():
        sr = net(lr, e, m)
        again = net(lr, e, m)
        torch.cuda.synchronize()
        print("native done", flush=True)
        assert torch.equal(sr, again), float((sr - again).abs().max())  # deterministic (fixed-order reductions)
        pd = {k: v.to(DEV) for k, v in p32.items()}
        want = ref.generator_forward(pd, lr, e, m, nb)
    assert sr.shape == (1, 1, 4 * h, 4 * w)
    _compare(sr, want, lambda: _autocast_runs(lambda: ref.generator_forward(pd, lr, e, m, nb)),
             "config-5 ESRGAN nb11 720x360 -> 2880x1440")


def test_config5_rcan_whole_grid_vs_oracle_fp32(fp32_torch):
    from climsr_amd.core.init import init_state, spec_from_shapes
    from climsr_amd.models.rcan import RCAN

    h, w = 360, 720
    net = RCAN(n_resgroups=10, n_resblocks=20, n_feats=64, reduction=16, scaling_factor=4, in_channels=3, out_channels=1)
    st = init_state(spec_from_shapes({k: tuple(v.shape) for k, v in net.state_dict().items()}))
    p32 = {k: torch.from_numpy(np.asarray(v)).float() for k, v in st.items()}
    net.load_state_dict(p32)
    net = net.to(DEV).eval()
    lr, e, m = _grid(h, w, seed=43)
    with torch.no_grad():
        sr = net(lr, e, m)
        again = net(lr, e, m)
        torch.cuda.synchronize()
        print("native done", flush=True)
        # every reduction runs in a fixed order and no launch reads what it writes: bit-identical reruns
        assert torch.equal(sr, again), float((sr - again).abs().max())
        pd = {k: v.to(DEV) for k, v in p32.items()}
        want = ref.rcan_forward(pd, lr, e, m, 10, 20, 4)
    _compare(sr, want, lambda: _autocast_runs(lambda: ref.rcan_forward(pd, lr, e, m, 10, 20, 4)),
             "config-5 RCAN 10x20 720x360 -> 2880x1440")
