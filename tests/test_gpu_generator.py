"""GPU model-level parity of the native ESRGAN generator (forward, backward, one L1-pretrain step)
against the reference-generated golden fixtures and the fp64 CPU oracle.

Tolerances (bf16 storage / bf16 MFMA inputs, fp32 accumulation):
  * generator output: PSNR >= 55 dB and SSIM >= 0.999 vs the fp64 reference output;
  * parameter gradients: relative L2 error per tensor <= 2x that of torch autocast (fp16/bf16) on the
    same weights, cosine >= 0.97 (see test_generator_backward_vs_oracle);
  * AdamW step: mean |delta_native - delta_oracle| <= 5% of lr.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import climsr_ref as ref
from tests.helpers import gen_params, psnr, scalar_cap, ssim

pytestmark = pytest.mark.gpu

DEV = "cuda"


def build_gen(nb, scale=4):
    from climsr_amd.models.esrgan import ESRGANGenerator

    g = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=nb, gc=16, scale_factor=4)
    p = gen_params(nb, torch.float32)
    g.load_state_dict(p)
    return g.to(DEV), gen_params(nb, torch.float64)


@pytest.mark.parametrize("tag,nb,b,hr", [("g_nb1_16to64", 1, 2, 64), ("g_nb1_32to128", 1, 2, 128), ("g_nb11_16to64", 11, 1, 64)])
def test_generator_forward_vs_golden(golden_dir, tag, nb, b, hr):
    g, _ = build_gen(nb)
    bt = ref.synthetic_batch(b, hr)
    with torch.no_grad():
        sr = g(bt["lr"].to(DEV), bt["elevation"].to(DEV), bt["mask"].to(DEV))
    torch.cuda.synchronize()
    want = torch.from_numpy(np.load(os.path.join(golden_dir, tag + ".npz"))["sr"])
    got = sr.double().cpu()
    assert got.shape == want.shape
    p = psnr(got, want)
    s = ssim(got, want)
    assert p >= 55.0, f"PSNR {p:.2f} dB"
    assert s >= 0.999, f"SSIM {s:.5f}"


def test_generator_forward_training_mode_equals_inference_mode():
    g, _ = build_gen(1)
    bt = ref.synthetic_batch(2, 64)
    args = [bt[k].to(DEV) for k in ("lr", "elevation", "mask")]
    with torch.no_grad():
        a = g(*args)
    b_ = g(*args)
    torch.cuda.synchronize()
    assert torch.equal(a, b_.detach()), "keep/no-keep forward paths must be bit-identical"


def _amp_reference_grads(p64, bt, nb, loss_fn, dtype=torch.float16):
    """The reference's own training precision (precision: 16 = native AMP fp16 with GradScaler 2^16,
    conf/experiment/*.yaml) -- and the same autocast at bf16, the build's dtype -- on the same weights:
    torch ops under autocast on the GPU (test only)."""
    keys = list(p64.keys())
    p = {k: v.float().to(DEV).requires_grad_(True) for k, v in p64.items()}
    b = {k: v.to(DEV) for k, v in bt.items()}
    with torch.autocast("cuda", dtype=dtype):
        sr = ref.generator_forward(p, b["lr"], b["elevation"], b["mask"], nb)
    loss = loss_fn(sr.float(), b["hr"])
    grads = torch.autograd.grad(loss * 65536.0, [p[k] for k in keys])
    return {k: (gr.double() / 65536.0).cpu() for k, gr in zip(keys, grads)}


def test_generator_backward_vs_oracle():
    """Parameter gradients vs the fp64 oracle, bounded by the reference's own AMP-fp16 deviation.

    Random-init parameter gradients are heavily cancelling sums over pixels, so activation-mask
    flips from any reduced-precision forward move them by several percent; the native bf16 path
    must stay within 2x the deviation of the same reference run under torch autocast (fp16 as the
    reference trains, or bf16 = the build's dtype, whichever is larger) and keep cosine >= 0.97."""
    nb = 1
    g, p64 = build_gen(nb)
    bt = ref.synthetic_batch(2, 64, seed=3)
    sr = g(bt["lr"].to(DEV), bt["elevation"].to(DEV), bt["mask"].to(DEV))
    from climsr_amd.losses.l1 import l1_loss

    loss = l1_loss(sr, bt["hr"].to(DEV))
    loss.backward()
    torch.cuda.synchronize()
    amp16 = _amp_reference_grads(p64, bt, nb, ref.l1_loss, torch.float16)
    ampbf = _amp_reference_grads(p64, bt, nb, ref.l1_loss, torch.bfloat16)
    keys = list(p64.keys())
    for k in keys:
        p64[k].requires_grad_(True)
    b64 = {k: v.double() for k, v in bt.items()}
    sr_ref = ref.generator_forward(p64, b64["lr"], b64["elevation"], b64["mask"], nb)
    lref = ref.l1_loss(sr_ref, b64["hr"])
    grads = torch.autograd.grad(lref, [p64[k] for k in keys])
    scalar_cap("generator nb-1 B=2 L1 loss vs fp64", float(loss.detach()), float(lref))
    named = dict(g.named_parameters())
    bad = []
    for k, gr in zip(keys, grads):
        got = named[k].grad.double().cpu()
        rel = float((got - gr).norm() / (gr.norm() + 1e-30))
        rel_amp = max(float((amp16[k] - gr).norm() / (gr.norm() + 1e-30)), float((ampbf[k] - gr).norm() / (gr.norm() + 1e-30)))
        cos = float((got * gr).sum() / (got.norm() * gr.norm() + 1e-30))
        if rel > max(2.0 * rel_amp, 2e-2) or cos < 0.97:
            bad.append((k, rel, rel_amp, cos))
    assert not bad, f"gradients outside the AMP-reference envelope: {bad[:6]}"


def test_grad_accumulation_semantics():
    g, _ = build_gen(1)
    bt = ref.synthetic_batch(1, 64, seed=4)
    args = [bt[k].to(DEV) for k in ("lr", "elevation", "mask")]
    from climsr_amd.losses.l1 import l1_loss

    l1_loss(g(*args), bt["hr"].to(DEV)).backward()
    g1 = g._flat_grad.clone()
    l1_loss(g(*args), bt["hr"].to(DEV)).backward()  # accumulates (grads left linked)
    g2 = g._flat_grad.clone()
    assert torch.allclose(g2, 2 * g1, rtol=1e-5, atol=1e-9)
    for p in g.parameters():
        p.grad = None  # zero_grad(set_to_none=True) -> next backward overwrites
    l1_loss(g(*args), bt["hr"].to(DEV)).backward()
    assert torch.equal(g._flat_grad, g1)


def test_pretrain_steps_vs_golden(golden_dir):
    """Three L1-pretrain steps (AdamW + OneCycleLR, total_steps=10) through the native AdamW."""
    want = json.load(open(os.path.join(golden_dir, "pretrain_steps.json")))
    from climsr_amd.core.optim import AdamW
    from climsr_amd.losses.l1 import l1_loss

    g, p64 = build_gen(1)
    before = {k: v.detach().clone().double().cpu() for k, v in g.named_parameters()}
    opt = AdamW(g.parameters(), lr=1e-4, weight_decay=1e-4, owner=g)
    sch = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=1e-4, total_steps=10, pct_start=0.05, div_factor=2,
                                              final_div_factor=100)
    for s in range(3):
        bt = ref.synthetic_batch(2, 64, seed=100 + s)
        opt.zero_grad()
        sr = g(bt["lr"].to(DEV), bt["elevation"].to(DEV), bt["mask"].to(DEV))
        loss = l1_loss(sr, bt["hr"].to(DEV))
        loss.backward()
        scalar_cap(f"pretrain step {s} L1 loss vs reference fixture", float(loss), want["loss"][s])
        opt.step()
        sch.step()
    torch.cuda.synchronize()
    # per tensor: the fixture's [sum, norm] checksums of the updated parameters (reference modules, fp64 torch AdamW)
    lr = 1e-4
    sums, norms = {}, {}
    for k, p in g.named_parameters():
        n = p.numel()
        pa = p.detach().double().cpu()
        sums[k] = abs(float(pa.sum() - before[k].sum()) - (want["params_after"][k][0] - float(before[k].sum()))) / n / lr
        norms[k] = abs(float(pa.norm()) - want["params_after"][k][1]) / n ** 0.5 / lr
    ws, wn = max(sums.items(), key=lambda kv: kv[1]), max(norms.items(), key=lambda kv: kv[1])
    print("pretrain 3 steps worst per-tensor |dsum|/n/lr", ws, "|dnorm|/sqrt(n)/lr", wn)
    assert ws[1] <= 0.25, ws
    assert wn[1] <= 0.25, wn
    # the full update vectors vs the fp64 oracle's three steps from the same state
    p64 = {k: v.clone() for k, v in before.items()}
    opt64 = ref.AdamWState(p64, list(p64.keys()), lr=lr, total_steps=10)
    for s in range(3):
        ref.pretrain_step(p64, opt64, ref.synthetic_batch(2, 64, seed=100 + s, dtype=torch.float64), 1)
    rels = {k: float((p.detach().double().cpu() - before[k] - (p64[k] - before[k])).norm() / ((p64[k] - before[k]).norm() + 1e-30))
            for k, p in g.named_parameters()}
    worst = max(rels.items(), key=lambda kv: kv[1])
    med = float(np.median(list(rels.values())))
    print("pretrain update-vector rel L2: worst", worst, "median", med)
    assert worst[1] <= 0.75 and med <= 0.25, (worst, med)
