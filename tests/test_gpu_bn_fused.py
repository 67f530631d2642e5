"""BatchNorm backward statistics from the data-gradient epilogue (ClimsrEpilogue.bn_z / bn_part,
climsr_bn_backward_parts): the RFB discriminator's BatchNorm2d + LeakyReLU backward (reference
climsr/models/rfb_esrgan.py:32-50) with sum(d) and sum(d * xhat) accumulated by the kernel that writes d's input
(the next conv's data gradient: the 16x16-tile stride-1 path, EP 10, and the phase-decomposed stride-2 path)
instead of a separate pass over that gradient and z.

Checked against the unfused route on the same inputs (same data gradient bit for bit; dgamma / dbeta / dz up to
the fp32 summation order) and against float64 sums of the same bf16 operands."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _close(got, want, rel, what):
    got, want = got.double().cpu(), want.double().cpu()
    err = float((got - want).abs().max())
    scale = float(want.abs().max()) + 1e-30
    assert err <= rel * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


# (conv in, conv out, stride, dz size): the data gradient of conv `cin -> cout` writes dL/da of the previous layer
# (cin channels), which is a BatchNorm + LeakyReLU layer.  The discriminator's: features.5/6 (128 -> 256 s1 at
# 64^2), features.8/9 (256 -> 512 s1), features.3/4/7/10 (stride 2, 128 / 256 / 512 channels); 64 -> 64 s2 for the
# 2 x 4 dgrad_s2 form; ragged sizes for partial tiles; the last two: >= 64 partial rows.
@pytest.mark.parametrize("cin,cout,stride,h,w", [(128, 256, 1, 32, 32), (256, 512, 1, 16, 16), (128, 256, 1, 20, 36),
                                                 (128, 128, 2, 16, 16), (256, 256, 2, 8, 8), (512, 512, 2, 8, 8),
                                                 (64, 64, 2, 16, 16), (128, 128, 2, 11, 13), (128, 256, 1, 96, 96),
                                                 (256, 256, 2, 64, 48)])
def test_dgrad_bn_backward_partials(cin, cout, stride, h, w):
    from climsr_amd import ops
    from climsr_amd.ops import ConvPlan

    n = 2
    g = torch.Generator(device=DEV).manual_seed(cin + cout + h)
    plan = ConvPlan(cin, cout, 3, stride, 1, "t")
    plan.bind((torch.randn(cout, cin, 3, 3, generator=g, device=DEV) * 0.05).contiguous(), None, need_t=True)
    plan.pack()
    hin, win = h * stride, w * stride  # the previous layer's (this conv's input) size
    dz = (torch.randn((n, h, w, cout), generator=g, device=DEV)).to(torch.bfloat16)
    z = (torch.randn((n, hin, win, cin), generator=g, device=DEV)).to(torch.bfloat16)
    mean = torch.randn(cin, generator=g, device=DEV) * 0.1
    rstd = torch.rand(cin, generator=g, device=DEV) + 0.5
    gamma = torch.rand(cin, generator=g, device=DEV) + 0.5
    beta = torch.rand(cin, generator=g, device=DEV) - 0.5
    npix = n * hin * win
    # keep z off the LeakyReLU kink of BN(z) (|y| ~ 0, where the fp32 affine's sign is a rounding decision)
    y0 = torch.addcmul(beta - mean * (gamma * rstd), z.float().reshape(npix, cin), gamma * rstd).reshape(z.shape)
    z = torch.where(y0.abs() <= 1e-4, (z.float() + 0.05).to(torch.bfloat16), z)
    nparts = plan.dgrad_bn_parts(cout, h, w, cin, n, cin)
    assert nparts > 0, "no fused path for this shape"
    part = torch.full((nparts * 2 * cin,), float("nan"), dtype=torch.float64, device=DEV)
    coef = torch.empty(3 * cin, device=DEV)
    # fused
    g1 = torch.empty((n, hin, win, cin), dtype=torch.bfloat16, device=DEV)
    plan.dgrad(dz, cout, h, w, g1, cin, 0, n, bn_bwd=(part, z, cin, mean, rstd, gamma, beta))
    dz1 = torch.empty_like(g1)
    dgam1, dbet1 = torch.full((cin,), 1.0, device=DEV), torch.full((cin,), -1.0, device=DEV)
    ops.bn_backward_parts(part, nparts, g1, z, npix, cin, mean, rstd, gamma, beta, coef, dgam1, dbet1, True, dz1)
    # unfused
    g2 = torch.empty_like(g1)
    plan.dgrad(dz, cout, h, w, g2, cin, 0, n)
    dz2 = torch.empty_like(g1)
    dgam2, dbet2 = torch.zeros(cin, device=DEV), torch.zeros(cin, device=DEV)
    cache = {}
    ops.bn_backward_z(g2, z, npix, cin, mean, rstd, gamma, beta, ops.bn_workspace(npix, cin, cache, z.device), coef, dgam2, dbet2,
                      False, dz2)
    torch.cuda.synchronize()
    assert not torch.isnan(part).any(), "partials rows left unwritten"
    assert torch.equal(g1, g2), "the data gradient changed"
    # float64 sums of the same bf16 operands (d = g * lrelu'(BN(z)), the sign from the fp32 affine as the kernels do)
    zf = z.float().reshape(npix, cin)
    sc = gamma * rstd
    sh = beta - mean * sc
    y = torch.addcmul(sh, zf, sc)  # fmaf(z, sc, sh) up to rounding: decisions at |y| ~ 0 may differ, excluded below
    keep = y.abs() > 1e-6
    d = g1.double().reshape(npix, cin) * torch.where(y > 0, 1.0, 0.2).double()
    xh = (zf.double() - mean.double()) * rstd.double()
    assert bool(keep.all()), "a z value sits on the LeakyReLU kink; reseed"
    _close(dgam1 - 1.0, (d * xh).sum(0), 1e-5, "dgamma (fused, +=)")
    _close(dbet1 + 1.0, d.sum(0), 1e-5, "dbeta (fused, +=)")
    _close(dgam1 - 1.0, dgam2, 1e-5, "dgamma fused vs unfused")
    _close(dbet1 + 1.0, dbet2, 1e-5, "dbeta fused vs unfused")
    dz64 = gamma.double() * rstd.double() * (d - d.mean(0) - xh * (d * xh).mean(0))
    _close(dz1.reshape(npix, cin), dz64, 2 ** -7, "dz (fused)")
    _close(dz1, dz2, 2 ** -7, "dz fused vs unfused")
