"""GPU parity of the native plain discriminator (climsr/models/discriminator.py) against the
reference-generated golden fixture (tests/golden/plain_d.npz) and the fp64 CPU oracle.  bf16 MFMA convs +
fp32 BN statistics: scores within 2 % of their scale, running statistics within 2 %, gradients by cosine and
relative norm against the envelope of the same oracle under bf16 autocast."""
import os

import numpy as np
import pytest
import torch

from oracle import climsr_ref as ref
from tests.helpers import plain_d_params

pytestmark = pytest.mark.gpu
DEV = "cuda"


def build():
    from climsr_amd.models.discriminator import Discriminator

    d = Discriminator(1)
    d.load_state_dict(plain_d_params(torch.float32))
    return d.to(DEV).train()


def test_plain_discriminator_forward_vs_golden(golden_dir):
    want = np.load(os.path.join(golden_dir, "plain_d.npz"))["score_train_128"]
    d = build()
    x = ref.synthetic_batch(2, 128, seed=9)["hr"].to(DEV)
    with torch.no_grad():
        s = d(x)
    torch.cuda.synchronize()
    got = s.double().cpu().numpy()
    scale = float(np.abs(want).max())
    np.testing.assert_allclose(got, want, rtol=0, atol=2e-2 * scale)
    # running statistics vs the oracle's own update (same momentum / unbiased variance)
    p64 = plain_d_params(torch.float64)
    with torch.no_grad():
        ref.plain_discriminator_forward(p64, ref.synthetic_batch(2, 128, seed=9, dtype=torch.float64)["hr"], training=True)
    sd = d.state_dict()
    for pre in ref.plain_bn_prefixes():
        for leaf in ("running_mean", "running_var"):
            np.testing.assert_allclose(sd[f"{pre}.{leaf}"].double().cpu().numpy(), p64[f"{pre}.{leaf}"].numpy(), rtol=2e-2, atol=2e-3)
        assert int(sd[f"{pre}.num_batches_tracked"]) == 1
    # eval mode: running statistics
    d.eval()
    with torch.no_grad():
        se = d(x)
        s64 = ref.plain_discriminator_forward(p64, ref.synthetic_batch(2, 128, seed=9, dtype=torch.float64)["hr"], training=False)
    scale = float(s64.abs().max())
    np.testing.assert_allclose(se.double().cpu().numpy(), s64.numpy(), rtol=0, atol=2e-2 * scale)


def _oracle_grads(p, x, wgt, cast=None):
    keys = ref.trainable_keys(p)
    for k in keys:
        p[k].requires_grad_(True)
    xx = x.clone().requires_grad_(True)
    if cast is None:
        s = ref.plain_discriminator_forward(p, xx, training=True)
    else:
        with torch.autocast("cpu", dtype=cast):
            s = ref.plain_discriminator_forward(p, xx, training=True)
    g = torch.autograd.grad((s.double() * wgt).sum(), [xx] + [p[k] for k in keys])
    return dict(zip(["x"] + keys, [t.double() for t in g]))


def _cmp(a, b):
    return float((a * b).sum() / (a.norm() * b.norm() + 1e-30)), float((a - b).norm() / (b.norm() + 1e-30))


def test_plain_discriminator_backward_vs_oracle():
    """Input and parameter gradients vs the fp64 oracle.  This architecture (LeakyReLU 0.01 feeding BN, ten
    layers, random init) amplifies reduced-precision noise: the SAME oracle under torch bf16 autocast lands at
    cosine 0.95-0.97 / relative error ~0.25 on the early layers.  Bound: no worse than that envelope
    (cosine >= autocast's - 0.01, relative error <= 1.25x autocast's + 0.02)."""
    d = build()
    x = ref.synthetic_batch(2, 128, seed=11)["hr"]
    wgt = torch.tensor([[0.7], [-1.3]], dtype=torch.float64)
    xg = x.to(DEV).requires_grad_(True)
    s = d(xg)
    (s * wgt.float().to(DEV)).sum().backward()
    torch.cuda.synchronize()
    g64 = _oracle_grads(plain_d_params(torch.float64), x.double(), wgt)
    gbf = _oracle_grads(plain_d_params(torch.float32), x.float(), wgt, torch.bfloat16)
    nat = {"x": xg.grad.double().cpu()}
    nat.update({k: v.grad.double().cpu() for k, v in d.named_parameters()})
    bad = []
    for k in g64:
        c_n, r_n = _cmp(nat[k], g64[k])
        c_b, r_b = _cmp(gbf[k], g64[k])
        if c_n < c_b - 0.01 or r_n > 1.25 * r_b + 0.02:
            bad.append((k, c_n, r_n, c_b, r_b))
    assert not bad, bad


def test_plain_discriminator_refuses_other_sizes():
    d = build()
    with pytest.raises(RuntimeError, match="8192"):
        with torch.no_grad():
            d(torch.zeros(2, 1, 64, 64, device=DEV))
