"""GPU parity of the native RCAN against the reference-generated golden outputs
(tests/golden/rcan.npz, climsr/models/rcan.py run in fp64) and of its non-conv kernels:

* nn.PixelShuffle index map: bit-exact vs torch;
* channel attention (pool -> 1x1 -> ReLU -> 1x1 -> sigmoid) and the RCAB residual: rel 1e-5 vs torch fp64;
* whole model: PSNR >= 50 dB and centred correlation >= 0.999 vs the fp64 reference (bf16 activations, fp32
  residual stream; 2x2 and 10x20 residual groups/blocks, x4 and x2 upsamplers).
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from climsr_amd.core.init import init_state, spec_from_shapes
from tests.helpers import psnr

pytestmark = pytest.mark.gpu
DEV = "cuda"
CONFIGS = {"rcan_g2b2_x4": (2, 2, 4, 2, 16), "rcan_g2b2_x2": (2, 2, 2, 1, 24), "rcan_g10b20_x4": (10, 20, 4, 1, 16)}


def batch(b, hr, seed=42, scale=4):
    g = torch.Generator().manual_seed(seed)
    t = torch.rand((b, 1, hr, hr), generator=g) * 2 - 1
    e = torch.rand((b, 1, hr, hr), generator=g) * 2 - 1
    m = (torch.rand((b, 1, hr, hr), generator=g) < 0.7).float()
    lr = torch.cat([t, e, m], 1)[:, :, ::scale, ::scale].contiguous()
    return lr, e, m


@pytest.mark.parametrize("name", list(CONFIGS))
def test_rcan_forward_vs_reference_golden(golden_dir, name):
    from climsr_amd.models.rcan import RCAN

    ng, nb, sf, b, lr_size = CONFIGS[name]
    net = RCAN(n_resgroups=ng, n_resblocks=nb, n_feats=64, reduction=16, scaling_factor=sf, in_channels=3, out_channels=1)
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    st = init_state(spec_from_shapes(shapes))
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()}, strict=True)
    net = net.to(DEV).eval()
    lr, e, m = batch(b, lr_size * sf, scale=sf)
    with torch.no_grad():
        sr = net(lr.to(DEV), e.to(DEV), m.to(DEV))
    torch.cuda.synchronize()
    want = torch.from_numpy(np.load(os.path.join(golden_dir, "rcan.npz"))[name])
    got = sr.double().cpu()
    assert got.shape == want.shape
    p = psnr(got, want)
    gc, wc = got - got.mean(), want - want.mean()
    corr = float((gc * wc).sum() / (gc.norm() * wc.norm()))
    assert p >= 50.0 and corr >= 0.999, f"PSNR {p:.2f} dB, centred correlation {corr:.6f}"


def test_rcan_refuses_training_mode():
    from climsr_amd.models.rcan import RCAN

    net = RCAN(n_resgroups=1, n_resblocks=1).to(DEV).train()
    lr, e, m = batch(1, 32)
    with pytest.raises(NotImplementedError, match="inference-only"):
        net(lr.to(DEV), e.to(DEV), m.to(DEV))


@pytest.mark.parametrize("r,c_out,h,w", [(2, 64, 5, 7), (3, 64, 4, 4), (2, 8, 9, 3)])
def test_pixel_shuffle_bit_exact(r, c_out, h, w):
    from climsr_amd import _lib
    from climsr_amd._lib import check, ptr

    n = 2
    x = torch.randn((n, c_out * r * r, h, w)).to(torch.bfloat16)
    want = F.pixel_shuffle(x, r)  # [n, c_out, h r, w r]
    xd = x.permute(0, 2, 3, 1).contiguous().to(DEV)
    y = torch.empty((n, h * r, w * r, c_out), dtype=torch.bfloat16, device=DEV)
    check(_lib.load().climsr_pixel_shuffle_bf16(ptr(xd), n, h, w, c_out, r, c_out * r * r, ptr(y), c_out, _lib.stream_ptr()), "ps")
    torch.cuda.synchronize()
    assert torch.equal(y.cpu().permute(0, 3, 1, 2), want)


def test_channel_attention_and_rcab_residual():
    from climsr_amd import _lib
    from climsr_amd._lib import check, ptr

    g = torch.Generator().manual_seed(3)
    n, h, w, c, cr = 2, 13, 17, 64, 4
    u = torch.randn((n, h, w, c), generator=g)
    xres = torch.randn((n, h, w, c), generator=g)
    w1 = torch.randn((cr, c), generator=g) * 0.2
    b1 = torch.randn((cr,), generator=g) * 0.1
    w2 = torch.randn((c, cr), generator=g) * 0.2
    b2 = torch.randn((c,), generator=g) * 0.1
    L = _lib.load()
    d = {k: v.to(DEV).contiguous() for k, v in dict(u=u, xres=xres, w1=w1, b1=b1, w2=w2, b2=b2).items()}
    s = torch.empty((n, c), device=DEV)
    ws = torch.empty(L.climsr_channel_attention_workspace(n, c) // 8, dtype=torch.float64, device=DEV)
    xb = torch.empty((n, h, w, c), dtype=torch.bfloat16, device=DEV)
    st = _lib.stream_ptr()
    check(L.climsr_channel_attention(ptr(d["u"]), n, h * w, c, c, ptr(d["w1"]), ptr(d["b1"]), ptr(d["w2"]), ptr(d["b2"]), cr,
                                     ptr(ws), ptr(s), st), "ca")
    xres0 = d["xres"].clone()
    check(L.climsr_ca_scale_add(ptr(d["u"]), 0, c, ptr(s), ptr(d["xres"]), ptr(xb), c, n, h * w, c, st), "scale add")
    torch.cuda.synchronize()
    ud = u.double()
    mean = ud.mean(dim=(1, 2))
    s_ref = torch.sigmoid(torch.relu(mean @ w1.double().T + b1.double()) @ w2.double().T + b2.double())
    assert (s.cpu().double() - s_ref).abs().max() <= 1e-5
    x_ref = ud * s_ref[:, None, None, :] + xres.double()
    assert (d["xres"].cpu().double() - x_ref).abs().max() <= 1e-5 * x_ref.abs().max()
    assert torch.equal(xb.cpu(), d["xres"].cpu().to(torch.bfloat16))
    # the bf16-u form (the RCAB's second conv stores u in bf16): the same update from the bf16-rounded u
    ub = d["u"].to(torch.bfloat16)
    xr2, xb2 = xres0.clone(), torch.empty_like(xb)
    check(L.climsr_ca_scale_add(ptr(ub), 1, c, ptr(s), ptr(xr2), ptr(xb2), c, n, h * w, c, st), "scale add bf16 u")
    torch.cuda.synchronize()
    x_ref2 = ub.double().cpu() * s.cpu().double()[:, None, None, :] + xres.double()
    assert (xr2.cpu().double() - x_ref2).abs().max() <= 1e-5 * x_ref2.abs().max()
    assert torch.equal(xb2.cpu(), xr2.cpu().to(torch.bfloat16))


@pytest.mark.parametrize("n,tpi,c,cr", [(2, 1035, 64, 4), (1, 7, 64, 4), (3, 300, 96, 6), (1, 50, 1024, 16)])
def test_channel_attention_parts_vs_float64(n, tpi, c, cr):
    """climsr_channel_attention_parts (tile sums folded into fp64 slices -> mean -> 1x1-ReLU-1x1-sigmoid, CALayer
    rcan.py:50-69) from per-tile channel sums as the RCAB conv2 epilogue writes them, vs float64; ragged tile counts,
    wide c."""
    from climsr_amd import _lib
    from climsr_amd._lib import check, ptr

    g = torch.Generator().manual_seed(tpi + c)
    part = torch.randn((n, tpi, c), generator=g) * 30.0
    hw = tpi * 256
    w1 = torch.randn((cr, c), generator=g) * 0.2
    b1 = torch.randn((cr,), generator=g) * 0.1
    w2 = torch.randn((c, cr), generator=g) * 0.2
    b2 = torch.randn((c,), generator=g) * 0.1
    L = _lib.load()
    d = {k: v.to(DEV).contiguous() for k, v in dict(part=part, w1=w1, b1=b1, w2=w2, b2=b2).items()}
    s = torch.empty((n, c), device=DEV)
    ws = torch.empty(L.climsr_channel_attention_workspace(n, c) // 8, dtype=torch.float64, device=DEV)
    check(L.climsr_channel_attention_parts(ptr(d["part"]), n, tpi, hw, c, ptr(d["w1"]), ptr(d["b1"]), ptr(d["w2"]), ptr(d["b2"]), cr,
                                           ptr(ws), ptr(s), _lib.stream_ptr()), "ca parts")
    torch.cuda.synchronize()
    mean = part.double().sum(1) / hw
    s_ref = torch.sigmoid(torch.relu(mean @ w1.double().T + b1.double()) @ w2.double().T + b2.double())
    assert (s.cpu().double() - s_ref).abs().max() <= 1e-5
