"""GPU op-level parity: the HIP implicit-GEMM conv (fwd / dgrad / wgrad) through the C ABI vs a
plain PyTorch fp64 reference of the same op on the same bf16-rounded operands.  The only
difference left is fp32 MFMA accumulation order, so the bound is tight (rel 1e-5 of the scale
plus one bf16 ulp where the output is stored in bf16)."""

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from climsr_amd.ops import (ACT_LRELU, ACT_NONE, ACT_RELU, OUT_BF16, OUT_F32, OUT_F32_ADD, ConvPlan, Workspace, act_grad)

DEV = "cuda"


def bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


def to_nhwc(x, cs=None, co=0, dtype=torch.bfloat16):
    n, c, h, w = x.shape
    cs = cs or ((c + 7) // 8 * 8)
    buf = torch.zeros((n, h, w, cs), dtype=dtype, device=DEV)
    buf[..., co:co + c] = x.permute(0, 2, 3, 1).to(dtype)
    return buf


def from_nhwc(buf, c, co=0):
    return buf[..., co:co + c].permute(0, 3, 1, 2).float()


def make_plan(cin, cout, ks, stride=1, pad=None, seed=0, bias=True):
    g = torch.Generator().manual_seed(seed)
    w = (torch.rand((cout, cin, ks, ks), generator=g) * 2 - 1) / (cin * ks * ks) ** 0.5
    b = (torch.rand((cout,), generator=g) * 2 - 1) * 0.1 if bias else None
    p = ConvPlan(cin, cout, ks, stride, pad, "t")
    w_d = w.to(DEV).contiguous()
    b_d = b.to(DEV) if b is not None else None
    p.bind(w_d, b_d)
    p.pack()
    return p, w, b


def check_close(got, want, tol=1e-5, what=""):
    scale = want.abs().max().item() + 1e-12
    err = (got.double() - want.double()).abs().max().item()
    assert err <= tol * scale + 1e-7, f"{what}: max err {err:.3e} vs scale {scale:.3e}"


CASES = [
    # cin, cout, ks, stride, up, n, h, w
    (64, 16, 3, 1, 1, 2, 20, 24),    # RDB conv1
    (80, 16, 3, 1, 1, 2, 16, 16),    # RDB conv2 (cin not a multiple of 32)
    (112, 16, 3, 1, 1, 1, 17, 33),   # RDB conv4, ragged tiles
    (128, 64, 3, 1, 1, 2, 16, 16),   # RDB conv5
    (3, 64, 3, 1, 1, 2, 16, 16),     # conv_first (cin padded to 8)
    (64, 64, 3, 1, 2, 2, 8, 12),     # upconv (nearest x2 on load)
    (64, 1, 3, 1, 1, 2, 16, 16),     # conv_last (cout 1)
    (3, 64, 9, 1, 1, 1, 20, 20),     # srcnn conv1
    (64, 32, 1, 1, 1, 2, 16, 16),    # srcnn conv2
    (32, 1, 5, 1, 1, 2, 16, 16),     # srcnn conv3
    (64, 1, 3, 1, 1, 2, 37, 70),     # conv_last on the MFMA co1 kernel: ragged rows, two column blocks
    (32, 1, 5, 1, 1, 1, 33, 130),    # srcnn conv3, three column blocks
    (24, 1, 5, 1, 1, 1, 20, 20),     # co1 with a partial 32-channel block
    (64, 1, 9, 1, 1, 1, 21, 67),     # 9x9 single output (the srcnn.conv1 data-gradient shape)
    (64, 128, 3, 2, 1, 2, 32, 32),   # D stride-2
    (256, 512, 3, 1, 1, 1, 8, 8),    # D / VGG wide
]


@pytest.mark.parametrize("cin,cout,ks,stride,up,n,h,w", CASES)
def test_conv_fwd_matches_torch(cin, cout, ks, stride, up, n, h, w):
    p, wt, b = make_plan(cin, cout, ks, stride)
    g = torch.Generator().manual_seed(1)
    x = torch.rand((n, cin, h, w), generator=g) * 2 - 1
    xb = bf(x)
    xin = to_nhwc(xb)
    oh, ow = p.out_hw(h, w, up)
    cs_out = (cout + 7) // 8 * 8
    y = torch.zeros((n, oh, ow, cs_out), dtype=torch.float32, device=DEV)
    p.fwd(xin, xin.shape[-1], 0, h, w, y, cs_out, 0, n, up=up, out_mode=OUT_F32)
    torch.cuda.synchronize()
    xr = xb.double()
    if up == 2:
        xr = F.interpolate(xr, scale_factor=2, mode="nearest")
    want = F.conv2d(xr, bf(wt).double(), b.double(), stride=stride, padding=ks // 2)
    check_close(from_nhwc(y, cout).cpu(), want, what=f"fwd {cin}->{cout} k{ks} s{stride} up{up}")


# LDS-DMA form of the 3x3 / 32-channel-chunk conv (conv_fwd_dma_kernel: 32 x 16 tiles, 8 waves, two DMA chunk
# buffers) under each epilogue it takes: activation forward (EP 3), RDB conv5 residual (EP 1), fp32 pull-x data
# gradient with an fp32 residual (EP 2), generic fp32 out with bias (EP 0), plain bf16 (EP 8); ragged rows / columns
DMA_CASES = [
    (64, 128, 2, 64, 64, "act"),
    (128, 64, 2, 96, 40, "conv5"),
    (128, 64, 1, 100, 33, "pullx"),
    (256, 256, 1, 32, 32, "plain"),
    (64, 128, 1, 64, 48, "bf16"),
    # the one-chunk HR shapes (64 -> 64 packed in one 64-channel chunk; upconv's nearest x2 upsample on load)
    (64, 64, 2, 64, 40, "act"),
    (64, 64, 1, 48, 24, "act", 2),
    (64, 64, 1, 64, 32, "bf16"),
]


@pytest.mark.parametrize("case", DMA_CASES)
def test_conv_fwd_lds_dma_matches_torch(case):
    cin, cout, n, h, w, mode = case[:6]
    up = case[6] if len(case) > 6 else 1
    import climsr_amd.ops as ops
    p, wt, b = make_plan(cin, cout, 3, seed=11, bias=mode in ("act", "conv5", "plain"))
    g = torch.Generator().manual_seed(12)
    x = torch.rand((n, cin, h, w), generator=g) * 2 - 1
    xin = to_nhwc(bf(x))
    oh, ow = h * up, w * up
    r = torch.rand((n, cout, oh, ow), generator=g) * 2 - 1
    f32 = mode in ("pullx", "plain")
    y = torch.zeros((n, oh, ow, cout), dtype=torch.float32 if f32 else torch.bfloat16, device=DEV)
    kw = dict(out_mode=OUT_F32 if f32 else OUT_BF16)
    if mode == "act":
        kw["act"] = ACT_RELU
    elif mode == "conv5":
        kw.update(res1=xin, res1_cs=cin, res1_co=0, alpha1=0.2)
    elif mode == "pullx":
        kw.update(use_bias=False, res1=to_nhwc(r, dtype=torch.float32), res1_cs=cout, res1_co=0)
    names = []
    ops.PROFILER = lambda name, flops, fn, tag="", nbytes=0: (names.append(name), fn())
    try:
        p.fwd(xin, cin, 0, h, w, y, cout, 0, n, up=up, **kw)
    finally:
        ops.PROFILER = None
    torch.cuda.synchronize()
    # RDB conv5 / pull-x (EP 1 / 2) and the one-chunk 64 -> 64 shapes stay on the two-workgroups-per-CU / conv_pw
    # kernels (measured faster in the GAN step); the same cases then check those
    dma = not (mode in ("conv5", "pullx") or (cin == 64 and cout == 64))
    assert names and names[-1].startswith("conv_fwd_dma_kernel") == dma, names
    xr = bf(x).double()
    if up == 2:
        xr = F.interpolate(xr, scale_factor=2, mode="nearest")
    want = F.conv2d(xr, bf(wt).double(), None if b is None else b.double(), padding=1)
    if mode == "act":
        want = F.relu(want)
    elif mode == "conv5":
        want = want * 0.2 + bf(x)[:, :cout].double()
    elif mode == "pullx":
        want = want + r.double()
    got = from_nhwc(y, cout).cpu().double()
    if f32:
        check_close(got, want, what=f"dma {mode}")
    else:  # bf16 store: one rounding of the fp32 result
        scale = want.abs().max().item()
        err = ((got - want).abs() - want.abs() * 2.0 ** -8).max().item()
        assert err <= 1e-5 * scale, f"dma {mode}: bf16 err {err:.3e} vs scale {scale:.3e}"


def test_conv_fwd_epilogue_slices_and_residuals():
    """Dense-buffer slices (read [0,80), write at channel 80) + lrelu, and the RRDB double residual."""
    n, h, w = 2, 16, 16
    p, wt, b = make_plan(80, 16, 3)
    g = torch.Generator().manual_seed(2)
    dense = torch.rand((n, h, w, 128), generator=g) * 2 - 1
    dense_d = dense.to(torch.bfloat16).to(DEV)
    before = dense_d.clone()
    p.fwd(dense_d, 128, 0, h, w, dense_d, 128, 80, n, act=ACT_LRELU)
    torch.cuda.synchronize()
    xr = bf(dense[..., :80]).permute(0, 3, 1, 2).double()
    want = F.leaky_relu(F.conv2d(xr, bf(wt).double(), b.double(), padding=1), 0.2)
    got = dense_d[..., 80:96].permute(0, 3, 1, 2).float().cpu()
    check_close(got, want, tol=1e-2, what="slice write")  # bf16 store
    assert torch.equal(dense_d[..., :80], before[..., :80]) and torch.equal(dense_d[..., 96:], before[..., 96:])
    # conv5-style: v = (acc+b)*0.2 + r1; v = v*0.2 + r2
    p5, w5, b5 = make_plan(128, 64, 3, seed=3)
    r2 = (torch.rand((n, h, w, 64), generator=g) * 2 - 1).to(torch.bfloat16).to(DEV)
    out = torch.zeros((n, h, w, 64), dtype=torch.float32, device=DEV)
    p5.fwd(dense_d, 128, 0, h, w, out, 64, 0, n, res1=dense_d, alpha1=0.2, res1_cs=128, res1_co=0, res2=r2, alpha2=0.2,
           res2_cs=64, res2_co=0, out_mode=OUT_F32)
    torch.cuda.synchronize()
    d = dense_d.float().cpu().permute(0, 3, 1, 2).double()
    x5 = F.conv2d(d, bf(w5).double(), b5.double(), padding=1)
    want = (x5 * 0.2 + d[:, :64]) * 0.2 + r2.float().cpu().permute(0, 3, 1, 2).double()
    check_close(from_nhwc(out, 64).cpu(), want, what="double residual")


@pytest.mark.gpu
@pytest.mark.parametrize("cin,ks,act,h,w", [(64, 3, 3, 20, 37), (32, 5, 4, 33, 18), (64, 3, 0, 16, 16)])
def test_dgrad_single_output_stencil(cin, ks, act, h, w):
    """climsr_dgrad_single_output (conv_last / srcnn.conv3 data gradients, esrgan.py:99, srcnn.py:17) vs autograd of
    F.conv2d with the same fp32 weights, the activation derivative taken from a bf16 activation; bf16 output
    (tolerance: bf16 rounding of the result, rel 1e-2)."""
    from climsr_amd.ops import ACT_LRELU_BWD, ACT_NONE, ACT_RELU_BWD

    n = 2
    p, wt, _b = make_plan(cin, 1, ks)
    g = torch.Generator().manual_seed(7)
    dz = bf(torch.rand((n, 1, h, w), generator=g) * 2 - 1)
    dz8 = to_nhwc(dz, cs=8)
    a = bf(torch.rand((n, cin, h, w), generator=g) * 2 - 1)
    ab = to_nhwc(a)
    out = torch.zeros((n, h, w, cin), dtype=torch.bfloat16, device=DEV)
    act_code = {0: ACT_NONE, 3: ACT_LRELU_BWD, 4: ACT_RELU_BWD}[act]
    p.dgrad(dz8, 8, h, w, out, cin, 0, n, act=act_code, res1=ab if act else None, res1_cs=cin, res1_co=0)
    torch.cuda.synchronize()
    x = torch.zeros((n, cin, h, w), dtype=torch.float64, requires_grad=True)
    y = F.conv2d(x, wt.double().cpu(), None, padding=ks // 2)
    (gref,) = torch.autograd.grad(y, x, dz.double())
    if act == 3:
        gref = torch.where(a.double() > 0, gref, gref * 0.2)
    elif act == 4:
        gref = torch.where(a.double() > 0, gref, torch.zeros_like(gref))
    got = from_nhwc(out, cin).cpu().double()
    err = (got - gref).abs().max().item()
    assert err <= 1e-2 * gref.abs().max().item() + 1e-6, f"single-output dgrad max err {err}"


@pytest.mark.parametrize("cin,cout,ks,up,down,h,w", [(64, 16, 3, 1, False, 16, 16), (128, 64, 3, 1, False, 16, 16),
                                                     (80, 16, 3, 1, False, 16, 16), (64, 64, 3, 2, True, 16, 16),
                                                     (32, 1, 5, 1, False, 16, 16), (3, 64, 9, 1, False, 16, 16),
                                                     (64, 32, 1, 1, False, 16, 16), (64, 1, 3, 1, False, 16, 16),
                                                     (32, 1, 5, 1, False, 64, 48), (64, 32, 1, 1, False, 64, 64),
                                                     (3, 64, 9, 1, False, 40, 56), (64, 16, 3, 1, False, 33, 40),
                                                     (64, 64, 3, 2, True, 24, 40)])
def test_conv_dgrad_matches_autograd(cin, cout, ks, up, down, h, w):
    n = 2
    p, wt, b = make_plan(cin, cout, ks)
    g = torch.Generator().manual_seed(4)
    oh, ow = h * up, w * up
    dz = bf(torch.rand((n, cout, oh, ow), generator=g) * 2 - 1)
    dzb = to_nhwc(dz)
    gx = torch.full((n, h, w, p.cin), 0.5, dtype=torch.float32, device=DEV)
    p.dgrad(dzb, dzb.shape[-1], oh, ow, gx, p.cin, 0, n, accumulate=True, down2=down)
    torch.cuda.synchronize()
    x = torch.zeros((n, cin, h, w), dtype=torch.float64, requires_grad=True)
    xin = F.interpolate(x, scale_factor=2, mode="nearest") if up == 2 else x
    y = F.conv2d(xin, bf(wt).double(), None, padding=ks // 2)
    (gref,) = torch.autograd.grad(y, x, dz.double())
    check_close(from_nhwc(gx, cin).cpu() - 0.5, gref, tol=2e-5, what="dgrad")


@pytest.mark.parametrize("cin,cout,ks,stride,up", [(64, 16, 3, 1, 1), (128, 64, 3, 1, 1), (112, 16, 3, 1, 1), (8, 64, 3, 1, 1),
                                                   (3, 64, 3, 1, 1), (1, 64, 3, 1, 1), (3, 64, 5, 1, 1),
                                                   (64, 64, 3, 1, 2), (32, 1, 5, 1, 1), (3, 64, 9, 1, 1), (64, 32, 1, 1, 1),
                                                   (64, 128, 3, 2, 1), (64, 1, 3, 1, 1)])
def test_conv_wgrad_matches_autograd(cin, cout, ks, stride, up):
    n, h, w = 2, 24, 20
    p, wt, b = make_plan(cin, cout, ks, stride)
    g = torch.Generator().manual_seed(5)
    x = bf(torch.rand((n, cin, h, w), generator=g) * 2 - 1)
    oh, ow = p.out_hw(h, w, up)
    dz = bf(torch.rand((n, cout, oh, ow), generator=g) * 2 - 1)
    xb, dzb = to_nhwc(x), to_nhwc(dz)
    p.gw = torch.zeros_like(p.weight)
    p.gb = torch.zeros_like(p.bias)
    p.wgrad(xb, xb.shape[-1], 0, h, w, dzb, dzb.shape[-1], n, Workspace(), accumulate=False, up=up)
    torch.cuda.synchronize()
    wr = bf(wt).double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    xin = F.interpolate(x.double(), scale_factor=2, mode="nearest") if up == 2 else x.double()
    y = F.conv2d(xin, wr, br, stride=stride, padding=ks // 2)
    gw, gb = torch.autograd.grad(y, (wr, br), dz.double())
    check_close(p.gw.cpu(), gw, tol=2e-5, what="wgrad")
    check_close(p.gb.cpu(), gb, tol=2e-5, what="bgrad")


@pytest.mark.parametrize("cin,cout,n,h,w", [(64, 64, 3, 37, 45), (128, 64, 2, 9, 33), (64, 128, 1, 64, 64)])
def test_conv_wgrad64_stride2_ragged(cin, cout, n, h, w):
    """Stride-2 64-block weight gradient (conv_wgrad64_glds_s2_kernel) on odd / ragged sizes: partial 4 x 16 output
    tiles, footprints past the bottom / right edge (zero-filled by the LDS-DMA), one image, two 64-row co blocks."""
    p, wt, b = make_plan(cin, cout, 3, 2)
    g = torch.Generator().manual_seed(7)
    x = bf(torch.rand((n, cin, h, w), generator=g) * 2 - 1)
    oh, ow = p.out_hw(h, w, 1)
    dz = bf(torch.rand((n, cout, oh, ow), generator=g) * 2 - 1)
    xb, dzb = to_nhwc(x), to_nhwc(dz)
    p.gw = torch.zeros_like(p.weight)
    p.gb = torch.zeros_like(p.bias)
    p.wgrad(xb, xb.shape[-1], 0, h, w, dzb, dzb.shape[-1], n, Workspace(), accumulate=False)
    torch.cuda.synchronize()
    wr = bf(wt).double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    y = F.conv2d(x.double(), wr, br, stride=2, padding=1)
    gw, gb = torch.autograd.grad(y, (wr, br), dz.double())
    check_close(p.gw.cpu(), gw, tol=2e-5, what="wgrad s2")
    check_close(p.gb.cpu(), gb, tol=2e-5, what="bgrad s2")


@pytest.mark.parametrize("cin,ks,n,h,w", [(64, 3, 3, 70, 150), (32, 5, 2, 45, 131), (16, 3, 1, 9, 64), (48, 5, 2, 33, 65)])
def test_conv_wgrad_single_output_channel(cin, ks, n, h, w):
    """conv_last / srcnn.conv3 weight gradient on the Toeplitz-fragment MFMA kernel: several 64-column strips,
    ragged last strip, segments that end mid-image."""
    p, wt, b = make_plan(cin, 1, ks)
    g = torch.Generator().manual_seed(9)
    x = bf(torch.rand((n, cin, h, w), generator=g) * 2 - 1)
    dz = bf(torch.rand((n, 1, h, w), generator=g) * 2 - 1)
    xb, dzb = to_nhwc(x), to_nhwc(dz)
    p.gw = torch.zeros_like(p.weight)
    p.gb = torch.zeros_like(p.bias)
    p.wgrad(xb, xb.shape[-1], 0, h, w, dzb, dzb.shape[-1], n, Workspace(), accumulate=False)
    torch.cuda.synchronize()
    wr = bf(wt).double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    y = F.conv2d(x.double(), wr, br, padding=ks // 2)
    gw, gb = torch.autograd.grad(y, (wr, br), dz.double())
    check_close(p.gw.cpu(), gw, tol=2e-5, what="wgrad co1")
    check_close(p.gb.cpu(), gb, tol=2e-5, what="bgrad co1")


@pytest.mark.parametrize("cout,n,h,w", [(32, 3, 70, 150), (64, 2, 33, 47), (16, 1, 9, 13)])
def test_conv_wgrad_1x1_single_pass(cout, n, h, w):
    """srcnn.conv2-shaped 1x1 weight gradient (64 inputs) on the single-pass pixel-range kernel, ragged chunks."""
    p, wt, b = make_plan(64, cout, 1)
    g = torch.Generator().manual_seed(10)
    x = bf(torch.rand((n, 64, h, w), generator=g) * 2 - 1)
    dz = bf(torch.rand((n, cout, h, w), generator=g) * 2 - 1)
    xb, dzb = to_nhwc(x), to_nhwc(dz)
    p.gw = torch.zeros_like(p.weight)
    p.gb = torch.zeros_like(p.bias)
    p.wgrad(xb, xb.shape[-1], 0, h, w, dzb, dzb.shape[-1], n, Workspace(), accumulate=False)
    torch.cuda.synchronize()
    wr = bf(wt).double().requires_grad_(True)
    br = b.double().requires_grad_(True)
    y = F.conv2d(x.double(), wr, br)
    gw, gb = torch.autograd.grad(y, (wr, br), dz.double())
    check_close(p.gw.cpu(), gw, tol=2e-5, what="wgrad 1x1")
    check_close(p.gb.cpu(), gb, tol=2e-5, what="bgrad 1x1")


def test_act_grad():
    n, h, w = 2, 8, 8
    g = torch.Generator().manual_seed(6)
    gr = torch.randn((n, h, w, 128), generator=g)
    y = (torch.randn((n, h, w, 128), generator=g)).to(torch.bfloat16)
    dz = torch.zeros((n, h, w, 16), dtype=torch.bfloat16, device=DEV)
    act_grad(n * h * w, 16, gr.to(DEV), 128, 96, y.to(DEV), 128, 96, ACT_LRELU, dz, 16, scale=0.5)
    want = gr[..., 96:112] * 0.5 * torch.where(y[..., 96:112].float() > 0, 1.0, 0.2)
    assert torch.allclose(dz.float().cpu(), bf(want), rtol=0, atol=0)


@pytest.mark.parametrize("cin,cout,h", [(64, 128, 32), (1, 64, 16), (256, 256, 16), (512, 512, 8)])
def test_conv_dgrad_stride2_matches_autograd(cin, cout, h):
    """Data gradient of the discriminator's stride-2 convs (rfb_esrgan.py:30-50) via zero insertion."""
    n, w = 2, h
    p, wt, b = make_plan(cin, cout, 3, stride=2)
    g = torch.Generator().manual_seed(7)
    oh, ow = h // 2, w // 2
    dz = bf(torch.rand((n, cout, oh, ow), generator=g) * 2 - 1)
    dzb = to_nhwc(dz)
    gx = torch.zeros((n, h, w, p.cin), dtype=torch.float32, device=DEV)
    p.dgrad(dzb, dzb.shape[-1], oh, ow, gx, p.cin, 0, n)
    torch.cuda.synchronize()
    x = torch.zeros((n, cin, h, w), dtype=torch.float64, requires_grad=True)
    y = F.conv2d(x, bf(wt).double(), None, stride=2, padding=1)
    (gref,) = torch.autograd.grad(y, x, dz.double())
    check_close(from_nhwc(gx, cin).cpu(), gref, tol=2e-5, what="dgrad s2")


@pytest.mark.parametrize("cin,cout,ks,h,w", [(3, 64, 9, 40, 36), (1, 64, 3, 20, 20), (3, 64, 9, 70, 67)])
def test_conv_dgrad_single_output_channel(cin, cout, ks, h, w):
    """dgrad restricted to input channel 0 (srcnn.conv1 w.r.t. conv_last's output): single-output MFMA kernel."""
    n = 2
    p, wt, b = make_plan(cin, cout, ks)
    g = torch.Generator().manual_seed(8)
    dz = bf(torch.rand((n, cout, h, w), generator=g) * 2 - 1)
    dzb = to_nhwc(dz)
    gx = torch.zeros((n, h, w, p.cin), dtype=torch.float32, device=DEV)
    p.dgrad(dzb, dzb.shape[-1], h, w, gx, p.cin, 0, n, cout_t=1)
    torch.cuda.synchronize()
    x = torch.zeros((n, cin, h, w), dtype=torch.float64, requires_grad=True)
    y = F.conv2d(x, bf(wt).double(), None, padding=ks // 2)
    (gref,) = torch.autograd.grad(y, x, dz.double())
    check_close(gx[..., :1].permute(0, 3, 1, 2).cpu(), gref[:, :1], tol=2e-5, what="dgrad co1")


def test_rdb_pull_backward_matches_torch():
    """Pull-form RDB data gradient (esrgan.py:17-38): each group's gradient as ONE conv over the
    side-by-side conv output gradients dZ = [dZ1|dZ2|dZ3|dZ4|dZ5], with the LeakyReLU backward read
    from the stored activations (epilogue act 3), fp32 residuals with a scale, and the aux output.
    Each step is checked against fp64 torch fed with the bf16 operands the kernel actually read."""
    from climsr_amd.ops import ACT_LRELU_BWD, PullPacker, PullPlan

    nf, gc, n, h, w = 64, 16, 2, 16, 20
    dc = nf + 4 * gc
    gen = torch.Generator().manual_seed(5)
    ws = [((torch.rand((gc if k < 5 else nf, nf + (k - 1) * gc, 3, 3), generator=gen) * 2 - 1) / ((nf + (k - 1) * gc) * 9) ** 0.5)
          for k in range(1, 6)]
    wd = [t.to(DEV).contiguous() for t in ws]
    pulls = []
    for j in range(5):
        segs = [(wd[k - 1], gc if k < 5 else nf, nf + (k - 1) * gc) for k in range(j + 1, 6)]
        pulls.append(PullPlan(segs, nf if j == 0 else gc, 0 if j == 0 else nf + (j - 1) * gc, 3, f"pull{j}"))
    PullPacker(pulls, torch.device(DEV)).run()
    dense = bf(torch.rand((n, dc, h, w), generator=gen) * 2 - 1)  # x, x1..x4 (signs drive the lrelu mask)
    dense_d = to_nhwc(dense)
    dz = torch.zeros((n, h, w, dc), dtype=torch.bfloat16, device=DEV)
    dz[..., 4 * gc:] = (torch.rand((n, h, w, nf), generator=gen) * 2 - 1).to(torch.bfloat16).to(DEV)  # dZ5
    g_out = (torch.rand((n, h, w, nf), generator=gen) * 2 - 1).to(DEV)
    g_skip = (torch.rand((n, h, w, nf), generator=gen) * 2 - 1).to(DEV)
    for j in (4, 3, 2, 1):
        pulls[j].fwd(dz, dc, j * gc, h, w, dz, dc, (j - 1) * gc, n, act=ACT_LRELU_BWD, use_bias=False, res1=dense_d, res1_cs=dc,
                     res1_co=nf + (j - 1) * gc)
    g_in = torch.empty((n, h, w, nf), dtype=torch.float32, device=DEV)
    aux = torch.zeros((n, h, w, dc), dtype=torch.bfloat16, device=DEV)
    pulls[0].fwd(dz, dc, 0, h, w, g_in, nf, 0, n, use_bias=False, out_mode=OUT_F32, res1=g_out, res1_cs=nf, res1_co=0, beta1=0.2,
                 res2=g_skip, res2_cs=nf, res2_co=0, aux=aux, aux_cs=dc, aux_co=4 * gc, aux_scale=0.04)
    torch.cuda.synchronize()
    dzc = from_nhwc(dz, dc).double().cpu()  # channels: dZ1..dZ4 (gc each), dZ5 (nf)

    def dz_of(k):
        return dzc[:, (k - 1) * gc:k * gc] if k < 5 else dzc[:, 4 * gc:]

    def pull_ref(j):
        lo = 0 if j == 0 else nf + (j - 1) * gc
        width = nf if j == 0 else gc
        tot = 0
        for k in range(j + 1, 6):
            wk = bf(ws[k - 1]).double()
            tot = tot + torch.nn.grad.conv2d_input((n, wk.shape[1], h, w), wk, dz_of(k), padding=1)[:, lo:lo + width]
        return tot

    for j in (4, 3, 2, 1):
        xj = dense[:, nf + (j - 1) * gc:nf + j * gc].double()
        want = pull_ref(j) * torch.where(xj > 0, 1.0, 0.2)
        got = dz_of(j)
        scale = want.abs().max().item()
        assert (got - want).abs().max().item() <= 8e-3 * scale, f"dZ{j}"  # bf16 store: <= 1 ulp (2^-8) of the value
    want = pull_ref(0) + 0.2 * from_nhwc(g_out, nf).double().cpu() + from_nhwc(g_skip, nf).double().cpu()
    check_close(from_nhwc(g_in, nf).cpu(), want, 1e-5, "G_in")
    check_close(from_nhwc(aux, nf, 4 * gc).cpu(), 0.04 * want, 8e-3, "aux")


@pytest.mark.parametrize("n,h,w", [(2, 16, 32), (2, 37, 48), (3, 5, 16), (32, 64, 64), (2, 9, 40), (1, 13, 113), (2, 11, 200),
                                   (1, 24, 720)])
def test_rdb_chain_matches_per_conv(n, h, w):
    """The fused RDB chain (csrc/rdb_chain.hip: conv1..conv4 forward and pull4..pull1 backward in one
    row-streaming launch, strips with recomputed row halos) against the same math run conv by conv (n16 kernel),
    including the bench shape (32 x 64 x 64: 256 strips of 8 rows), strips taller than the image, widths that are no
    multiple of 16 and images wider than the 64-column window (48-column strips with 8-column halos: the reference's
    113 -> 452 Europe tiles, climate_dataset.py:53, and config 5's 720-wide grid, inference.py:70).
    Both are bf16 MFMA with fp32 accumulation; outputs agree to bf16 rounding (1 ulp of the value), the
    chain's level inputs being the same bf16 values the per-conv path reads back from HBM."""
    from climsr_amd.ops import ACT_LRELU_BWD, BatchedPacker, PullPacker, PullPlan, RdbChain

    nf, gc = 64, 16
    dc = nf + 4 * gc
    gen = torch.Generator().manual_seed(9)
    plans = []
    for k in range(1, 6):
        cin, cout = nf + (k - 1) * gc, (gc if k < 5 else nf)
        p = ConvPlan(cin, cout, 3, 1, None, f"conv{k}")
        wt = ((torch.rand((cout, cin, 3, 3), generator=gen) * 2 - 1) / (cin * 9) ** 0.5).to(DEV).contiguous()
        b = ((torch.rand((cout,), generator=gen) * 2 - 1) * 0.1).to(DEV)
        p.bind(wt, b, need_t=False)
        plans.append(p)
    chain = RdbChain(plans, "t")
    pulls = []
    for j in range(5):
        segs = [(plans[k - 1].weight, gc if k < 5 else nf, nf + (k - 1) * gc) for k in range(j + 1, 6)]
        pulls.append(PullPlan(segs, nf if j == 0 else gc, 0 if j == 0 else nf + (j - 1) * gc, 3, f"pull{j}"))
    BatchedPacker(plans, torch.device(DEV), chain.pack_descs()).run()
    PullPacker(pulls, torch.device(DEV), chain.pull_descs()).run()
    x = (torch.rand((n, h, w, dc), generator=gen) * 2 - 1).to(torch.bfloat16).to(DEV)
    ref = x.clone()
    for k in range(1, 5):
        plans[k - 1].fwd(ref, dc, 0, h, w, ref, dc, nf + (k - 1) * gc, n, act=ACT_LRELU)
    got = x.clone()
    chain.forward(got, dc, n, h, w)
    dz0 = torch.zeros((n, h, w, dc), dtype=torch.bfloat16, device=DEV)
    dz0[..., 4 * gc:] = (torch.rand((n, h, w, nf), generator=gen) * 2 - 1).to(torch.bfloat16).to(DEV)
    dref = dz0.clone()
    for j in (4, 3, 2, 1):
        pulls[j].fwd(dref, dc, j * gc, h, w, dref, dc, (j - 1) * gc, n, act=ACT_LRELU_BWD, use_bias=False, res1=ref, res1_cs=dc,
                     res1_co=nf + (j - 1) * gc)
    dgot = dz0.clone()
    chain.pull(dgot, ref, dc, n, h, w)
    torch.cuda.synchronize()
    for name, a_, b_ in [(f"x{k + 1}", got[..., nf + k * gc:nf + (k + 1) * gc], ref[..., nf + k * gc:nf + (k + 1) * gc]) for k in range(4)] + \
            [(f"dZ{k + 1}", dgot[..., k * gc:(k + 1) * gc], dref[..., k * gc:(k + 1) * gc]) for k in range(4)]:
        a64, b64 = a_.double(), b_.double()
        exc = (a64 - b64).abs() - 2 ** -7 * b64.abs()
        err = exc.max().item()
        bad = (exc > 1e-3 * b64.abs().max().item()).nonzero()
        assert err <= 1e-3 * b64.abs().max().item(), (f"{name}: excess error {err}, {len(bad)} bad, first (n,y,x,c): "
                                                      f"{bad[:6].tolist()}, rows {sorted(set(bad[:, 1].tolist()))[:12]}, "
                                                      f"cols {sorted(set(bad[:, 2].tolist()))[:12]}")
    assert torch.equal(got[..., :nf], x[..., :nf]) and torch.equal(dgot[..., 4 * gc:], dz0[..., 4 * gc:])



@pytest.mark.parametrize("cout,ks,act,h,w", [(64, 3, 1, 40, 36), (64, 3, 0, 256, 256), (32, 5, 2, 20, 23)])
def test_conv_single_input_channel_forward(cout, ks, act, h, w):
    """1 -> C forward stencil (climsr_conv_single_input: the RFB discriminator's features.0, rfb_esrgan.py:28) vs fp64
    torch on the same bf16 operands, with bias / leaky relu / relu variants."""
    n = 2
    p, wt, b = make_plan(1, cout, ks, bias=act != 1)
    g = torch.Generator().manual_seed(9)
    x = bf(torch.rand((n, 1, h, w), generator=g) * 2 - 1)
    xb = to_nhwc(x)
    y = torch.empty((n, h, w, cout), dtype=torch.bfloat16, device=DEV)
    acts = {0: ACT_NONE, 1: ACT_LRELU, 2: ACT_RELU}
    p.fwd(xb, xb.shape[-1], 0, h, w, y, cout, 0, n, act=acts[act])
    torch.cuda.synchronize()
    want = F.conv2d(x.double(), wt.double(), None if b is None else b.double(), padding=ks // 2)
    want = F.leaky_relu(want, 0.2) if act == 1 else (F.relu(want) if act == 2 else want)
    got = from_nhwc(y, cout).cpu().double()
    err = (got - want).abs().max().item()
    assert err <= 2 ** -8 * want.abs().max().item() + 1e-6, f"single-input fwd: max err {err:.3e}"


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,h,w,act", [(64, 64, 32, 48, 0), (64, 128, 34, 20, 3), (96, 64, 16, 16, 4), (40, 64, 18, 22, 3),
                                              (128, 128, 64, 64, 0)])
def test_conv_dgrad_stride2_bf16(cin, cout, h, w, act):
    """Data gradient of the discriminator's 3x3 stride-2 convs (rfb_esrgan.py:30-48) as the D backward runs it: bf16
    output, optionally with the previous LeakyReLU/ReLU derivative from its bf16 activation (conv_dgrad_s2_kernel when
    the channels are multiples of 32 -- ragged 17-row / 10-column dz tiles included -- else the zero-inserted generic
    conv) vs autograd of F.conv2d in float64 on the same bf16 weights.  Tolerance: bf16 rounding of the result."""
    from climsr_amd.ops import ACT_LRELU_BWD, ACT_NONE, ACT_RELU_BWD

    n = 2
    p, wt, _b = make_plan(cin, cout, 3, stride=2, bias=False)
    oh, ow = (h + 1) // 2, (w + 1) // 2
    g = torch.Generator().manual_seed(11)
    dz = bf(torch.rand((n, cout, oh, ow), generator=g) * 2 - 1)
    a = bf(torch.rand((n, cin, h, w), generator=g) * 2 - 1)
    out = torch.zeros((n, h, w, p.cin), dtype=torch.bfloat16, device=DEV)
    act_code = {0: ACT_NONE, 3: ACT_LRELU_BWD, 4: ACT_RELU_BWD}[act]
    p.dgrad(to_nhwc(dz), p.cin_t, oh, ow, out, p.cin, 0, n, act=act_code, res1=to_nhwc(a) if act else None, res1_cs=p.cin,
            res1_co=0)
    torch.cuda.synchronize()
    x = torch.zeros((n, cin, h, w), dtype=torch.float64, requires_grad=True)
    y = F.conv2d(x, bf(wt).double(), None, stride=2, padding=1)
    (gref,) = torch.autograd.grad(y, x, dz.double())
    if act == 3:
        gref = torch.where(a.double() > 0, gref, gref * 0.2)
    elif act == 4:
        gref = torch.where(a.double() > 0, gref, torch.zeros_like(gref))
    got = from_nhwc(out, cin).cpu().double()
    err = (got - gref).abs().max().item()
    assert err <= 8e-3 * gref.abs().max().item() + 1e-6, f"stride-2 dgrad max err {err} (scale {gref.abs().max().item()})"


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,h,w,n", [(64, 64, 64, 48, 2), (64, 128, 34, 20, 2), (128, 64, 16, 16, 2), (96, 64, 40, 66, 2),
                                             (32, 64, 128, 130, 13), (64, 64, 128, 130, 13)])
def test_conv_fwd_stride2_plain_bf16(cin, cout, h, w, n):
    """The discriminator's stride-2 convs as its forward runs them (rfb_esrgan.py:30-48): no bias, no activation,
    bf16 out for the BatchNorm (conv_fwd_s2_dma_kernel: LDS-DMA, three chunk buffers; ragged 17-row / 10- and 33-column
    output tiles included) vs F.conv2d in float64 on the same bf16 operands.  Tolerance: bf16 rounding.  The n = 13
    cases have 260 items (just above one per CU), so a workgroup's last item has nothing requested behind its last
    chunks (2 and 4 chunks of 16 channels): the DMA wait there must drain every outstanding piece."""
    p, wt, _b = make_plan(cin, cout, 3, stride=2, bias=False)
    g = torch.Generator().manual_seed(12)
    x = bf(torch.rand((n, cin, h, w), generator=g) * 2 - 1)
    oh, ow = (h + 1) // 2, (w + 1) // 2
    y = torch.zeros((n, oh, ow, cout), dtype=torch.bfloat16, device=DEV)
    p.fwd(to_nhwc(x), p.cin, 0, h, w, y, cout, 0, n, use_bias=False)
    torch.cuda.synchronize()
    want = F.conv2d(x.double(), bf(wt).double(), None, stride=2, padding=1)
    got = from_nhwc(y, cout).cpu().double()
    err = (got - want).abs().max().item()
    assert err <= 8e-3 * want.abs().max().item() + 1e-6, f"stride-2 fwd max err {err}"


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,stride,h,w", [(64, 128, 1, 32, 48), (128, 128, 2, 34, 40), (64, 64, 2, 64, 64), (64, 64, 1, 32, 32),
                                                 (64, 128, 1, 128, 128), (128, 512, 2, 256, 160)])
def test_conv_bn_partials_match_bn_forward(cin, cout, stride, h, w):
    """BatchNorm statistics from the conv epilogue (ClimsrEpilogue.bn_part -> climsr_bn_forward_parts; the discriminator's
    train-mode conv + BatchNorm2d + LeakyReLU, rfb_esrgan.py:30-50) vs climsr_bn_forward's own pass over the same z:
    batch mean / rstd / running stats within fp32 summation-order noise, the activation within one bf16 ulp.  A conv
    whose kernel cannot emit partials (64 -> 64 stride 1: conv_pw) reports 0 rows.  The last two: 128 and 80 partial rows."""
    from climsr_amd import ops

    n = 2
    p, _wt, _b = make_plan(cin, cout, 3, stride=stride, bias=False)
    g = torch.Generator().manual_seed(21)
    x = to_nhwc(bf(torch.rand((n, cin, h, w), generator=g) * 2 - 1))
    oh, ow = p.out_hw(h, w)
    nparts = p.bn_parts(p.cin, h, w, n, cout)
    if cin == 64 and cout == 64 and stride == 1:
        assert nparts == 0
        return
    assert nparts == n * ((oh + 15) // 16) * ((ow + 15) // 16)
    part = torch.full((nparts * 2 * cout,), float("nan"), dtype=torch.float64, device=DEV)
    z = torch.empty((n, oh, ow, cout), dtype=torch.bfloat16, device=DEV)
    z2 = torch.empty_like(z)
    p.fwd(x, p.cin, 0, h, w, z, cout, 0, n, use_bias=False, bn_part=part)
    p.fwd(x, p.cin, 0, h, w, z2, cout, 0, n, use_bias=False)
    gamma = torch.rand(cout, generator=g).to(DEV) + 0.5
    beta = (torch.rand(cout, generator=g) - 0.5).to(DEV)
    npix = n * oh * ow
    outs = []
    for fused in (True, False):
        mean, rstd = torch.empty(cout, device=DEV), torch.empty(cout, device=DEV)
        rm, rv = torch.zeros(cout, device=DEV), torch.ones(cout, device=DEV)
        a = torch.empty_like(z)
        if fused:
            ops.bn_forward_parts(part, nparts, z, npix, cout, gamma, beta, mean, rstd, a, rm, rv)
        else:
            ops.bn_forward(z, npix, cout, gamma, beta, mean, rstd, a, ops.bn_workspace(npix, cout, {}, torch.device(DEV)), rm, rv)
        outs.append((mean, rstd, rm, rv, a))
    torch.cuda.synchronize()
    assert torch.equal(z, z2), "bn_part must not change the conv output"
    assert not torch.isnan(part).any(), "every partial row written"
    for got, want, what in zip(outs[0][:4], outs[1][:4], ("mean", "rstd", "running_mean", "running_var")):
        err = (got.double() - want.double()).abs().max().item()
        assert err <= 1e-5 * (want.abs().max().item() + 1e-3), f"{what}: {err}"
    da = (outs[0][4].float() - outs[1][4].float()).abs()
    assert da.max().item() <= 1e-2 * outs[1][4].float().abs().max().item(), f"activation max diff {da.max().item()}"


WR_CASES = [
    # n, h, w, up, epilogue
    (2, 16, 32, 1, "lrelu"),       # HRconv-like, tile-aligned
    (1, 13, 37, 1, "relu"),        # ragged rows / columns (VGG conv1_2 / RCAB conv1)
    (2, 9, 20, 2, "lrelu"),        # upconv: nearest x2 on load, 18 x 40 output
    (1, 45, 90, 1, "bias"),        # RCAB conv2 (bias, no activation), several persistent rounds
    (1, 12, 24, 1, "res"),         # residual epilogue (v * alpha + beta * r)
    (2, 10, 34, 1, "lrelu_bwd"),   # activation backward from the stored activation (HRconv data gradient)
    (1, 7, 16, 1, "relu_bwd"),
]


@pytest.mark.parametrize("n,h,w,up,mode", WR_CASES)
def test_conv_wr_matches_fp64(n, h, w, up, mode):
    """The 64 -> 64 3x3 conv with the weights in registers (csrc/conv_wr.hip: A fragments in AGPRs read by asm MFMAs,
    wave-private LDS-DMA footprints, no barriers) vs fp64 torch on the same bf16 operands, for each epilogue it takes,
    ragged tiles and the nearest x2 upsample on load."""
    from climsr_amd import ops

    p, wt, b = make_plan(64, 64, 3, seed=11, bias=mode not in ("lrelu_bwd", "relu_bwd"))
    g = torch.Generator().manual_seed(12)
    x = bf(torch.rand((n, 64, h, w), generator=g) * 2 - 1)
    oh, ow = h * up, w * up
    xin = to_nhwc(x, cs=72, co=8)  # channel stride / offset != 64: the strided operand path
    y = torch.full((n, oh, ow, 64), 7.0, dtype=torch.bfloat16, device=DEV)
    r = bf(torch.rand((n, 64, oh, ow), generator=g) * 2 - 1)
    kw = {}
    if mode == "lrelu":
        kw = dict(act=ACT_LRELU)
    elif mode == "relu":
        kw = dict(act=ACT_RELU)
    elif mode == "res":
        kw = dict(res1=to_nhwc(r), res1_cs=64, res1_co=0, alpha1=0.2)
    elif mode in ("lrelu_bwd", "relu_bwd"):
        kw = dict(act=3 if mode == "lrelu_bwd" else 4, use_bias=False, res1=to_nhwc(r), res1_cs=64, res1_co=0)
    names = []
    ops.PROFILER = lambda name, flops, fn, tag="", nbytes=0: (names.append(name), fn())
    try:
        p.fwd(xin, 72, 8, h, w, y, 64, 0, n, up=up, **kw)
    finally:
        ops.PROFILER = None
    torch.cuda.synchronize()
    assert names and names[-1].startswith("conv_wr_kernel"), names
    xr = x.double()
    if up == 2:
        xr = F.interpolate(xr, scale_factor=2, mode="nearest")
    want = F.conv2d(xr, bf(wt).double(), None if (b is None or mode.endswith("bwd")) else b.double(), padding=1)
    if mode == "lrelu":
        want = F.leaky_relu(want, 0.2)
    elif mode == "relu":
        want = F.relu(want)
    elif mode == "res":
        want = 0.2 * want + r.double()
    elif mode == "lrelu_bwd":
        want = torch.where(r.double() > 0, want, 0.2 * want)
    elif mode == "relu_bwd":
        want = torch.where(r.double() > 0, want, torch.zeros_like(want))
    got = from_nhwc(y, 64).double().cpu()
    err = float((got - want).abs().max())
    assert err <= 2 ** -7 * float(want.abs().max()) + 1e-6, f"{mode}: err {err:.3e} vs {float(want.abs().max()):.3e}"


@pytest.mark.parametrize("n,h,w,f32", [(2, 13, 37, True), (1, 45, 90, True), (2, 13, 37, False), (1, 30, 70, False),
                                       (1, 9, 37, True), (1, 180, 360, False)])
def test_conv_wr_fp32_out_channel_sums(n, h, w, f32):
    """conv_wr's fp32-output epilogue (RCAN's RCAB conv2, rcan.py:50-69) and the channel sums it emits for the channel
    attention's global pool (climsr_conv2d_fwd_ch_parts rows: per tile, tiles of an image contiguous; with one image
    one row per workgroup -- 9 tiles leave the last workgroup one wave with a tile, 180 x 360 gives a workgroup several
    tiles a wave): the output vs fp64 torch, the sums of each image's rows vs the image's channel sums of that output."""
    from climsr_amd import ops

    p, wt, b = make_plan(64, 64, 3, seed=21)
    g = torch.Generator().manual_seed(22)
    x = bf(torch.rand((n, 64, h, w), generator=g) * 2 - 1)
    y = torch.full((n, h, w, 64), 7.0, dtype=torch.float32 if f32 else torch.bfloat16, device=DEV)
    rows, tpi = p.ch_parts(64, h, w, n, 64)
    tiles = ((w + 15) // 16) * ((h + 3) // 4)
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    assert rows == n * tpi and tpi == (min((tiles + 3) // 4, ncu) if n == 1 else tiles)
    part = torch.full((rows, 64), 7.0, dtype=torch.float32, device=DEV)
    names = []
    ops.PROFILER = lambda name, flops, fn, tag="", nbytes=0: (names.append(name), fn())
    try:
        p.fwd(to_nhwc(x), 64, 0, h, w, y, 64, 0, n, out_mode=OUT_F32 if f32 else OUT_BF16, ch_part=part)
    finally:
        ops.PROFILER = None
    torch.cuda.synchronize()
    assert names and names[-1].startswith("conv_wr_kernel<3," if f32 else "conv_wr_kernel<4,"), names
    want = F.conv2d(x.double(), bf(wt).double(), b.double(), padding=1)
    check_close(from_nhwc(y, 64).cpu(), want, 1e-5 if f32 else 2 ** -8, "out")
    sums = part.double().cpu().reshape(n, tpi, 64).sum(1)
    # the sums are of the fp32 values (before the bf16 rounding of a bf16 output)
    check_close(sums, want.sum((2, 3)), 1e-5, "channel sums")


@pytest.mark.parametrize("n,h,w", [(2, 32, 32), (1, 45, 70), (3, 20, 100), (1, 5, 7), (2, 64, 96), (1, 37, 36)])
def test_srcnn_tail_matches_fp64(n, h, w):
    """The fused SRCNN tail (csrc/srcnn.hip: conv1 9x9 -> ReLU -> conv2 1x1 -> ReLU -> conv3 5x5 in one launch,
    srcnn.py:9-18) vs fp64 torch on the same bf16 input and weights, with the two intermediates rounded to bf16 as the
    kernel keeps them; ragged tiles, images smaller than a tile, odd group counts per wave.  Input channels past the
    three real ones hold garbage (their weights are zero).  Reruns are bit-identical."""
    from climsr_amd import ops

    p1, w1, b1 = make_plan(3, 64, 9, seed=41)
    p2, w2, b2 = make_plan(64, 32, 1, seed=42)
    p3, w3, b3 = make_plan(32, 1, 5, seed=43)
    tail = ops.SrcnnTail([p1, p2, p3])
    tail.pack()
    g = torch.Generator().manual_seed(44)
    x = bf(torch.rand((n, 3, h, w), generator=g) * 2 - 1)
    xin = torch.full((n, h, w, 8), 5.0, dtype=torch.bfloat16, device=DEV)
    xin[..., :3] = x.permute(0, 2, 3, 1).to(DEV).to(torch.bfloat16)
    out = torch.full((n, 1, h, w), 7.0, dtype=torch.float32, device=DEV)
    names = []
    ops.PROFILER = lambda name, flops, fn, tag="", nbytes=0: (names.append(name), fn())
    try:
        tail.fwd(xin, 8, 0, n, h, w, out)
    finally:
        ops.PROFILER = None
    torch.cuda.synchronize()
    assert names == ["srcnn_tail_kernel"], names
    a1 = F.relu(F.conv2d(x.double(), bf(w1).double(), b1.double(), padding=4))
    a2 = F.relu(F.conv2d(a1.to(torch.bfloat16).double(), bf(w2).double(), b2.double()))
    want = F.conv2d(a2.to(torch.bfloat16).double(), bf(w3).double(), b3.double(), padding=2)
    check_close(out.cpu(), want, 4e-3, "srcnn out")
    out2 = torch.empty_like(out)
    tail.fwd(xin, 8, 0, n, h, w, out2)
    torch.cuda.synchronize()
    assert torch.equal(out, out2)


@pytest.mark.parametrize("n,h,w", [(2, 32, 32), (1, 45, 70), (3, 20, 100), (1, 5, 7)])
def test_srcnn_tail_backward_matches_fp64(n, h, w):
    """The fused SRCNN tail backward (csrc/srcnn.hip srcnn_bwd_kernel: recomputes relu(conv1) / relu(conv2), then
    dZ2 = conv3^T(g) * relu', dZ1 = conv2^T(dZ2) * relu', and the conv2 / conv3 weight + bias gradients) vs fp64 torch
    autograd on the same bf16 operands, with the intermediates rounded to bf16 where the kernel keeps them in bf16
    (relu(conv1), relu(conv2), g, dZ2).  Accumulation into existing gradients, ragged tiles, tiny images."""
    from climsr_amd import ops

    p1, w1, b1 = make_plan(3, 64, 9, seed=51)
    p2, w2, b2 = make_plan(64, 32, 1, seed=52)
    p3, w3, b3 = make_plan(32, 1, 5, seed=53)
    for p in (p2, p3):
        p.gw = torch.full(tuple(p.weight.shape), 0.5, device=DEV)
        p.gb = torch.full(tuple(p.bias.shape), 0.25, device=DEV)
    tail = ops.SrcnnTail([p1, p2, p3])
    tail.pack()
    g = torch.Generator().manual_seed(54)
    x = bf(torch.rand((n, 3, h, w), generator=g) * 2 - 1)
    gout = torch.randn((n, 1, h, w), generator=g)
    xin = torch.full((n, h, w, 8), 5.0, dtype=torch.bfloat16, device=DEV)
    xin[..., :3] = x.permute(0, 2, 3, 1).to(DEV).to(torch.bfloat16)
    dz1 = torch.full((n, h, w, 64), 7.0, dtype=torch.bfloat16, device=DEV)
    names = []
    ops.PROFILER = lambda name, flops, fn, tag="", nbytes=0: (names.append(name), fn())
    try:
        tail.bwd(xin, 8, 0, n, h, w, gout.to(DEV).contiguous(), dz1, ops.Workspace(), accumulate=True)
    finally:
        ops.PROFILER = None
    torch.cuda.synchronize()
    assert names == ["srcnn_bwd_kernel"], names
    d = torch.float64
    a1b = F.relu(F.conv2d(x.double(), bf(w1).double(), b1.double(), padding=4)).to(torch.bfloat16).to(d)
    a2b = F.relu(F.conv2d(a1b, bf(w2).double(), b2.double())).to(torch.bfloat16).to(d)
    gb = bf(gout).double()
    a2v = a2b.clone().requires_grad_()
    w3v = bf(w3).double().requires_grad_()
    F.conv2d(a2v, w3v, b3.double(), padding=2).backward(gb)
    dz2b = (a2v.grad * (a2b > 0)).to(torch.bfloat16).to(d)
    a1v = a1b.clone().requires_grad_()
    w2v = bf(w2).double().requires_grad_()
    F.conv2d(a1v, w2v, b2.double()).backward(dz2b)
    dz1_ref = a1v.grad * (a1b > 0)
    got = dz1.permute(0, 3, 1, 2).double().cpu()
    err = float((got - dz1_ref).abs().max())
    assert err <= 2 ** -7 * float(dz1_ref.abs().max()) + 1e-6, f"dZ1: err {err:.3e} vs {float(dz1_ref.abs().max()):.3e}"
    check_close(p2.gw.cpu() - 0.5, w2v.grad, 2e-3, "dW2")
    check_close(p2.gb.cpu() - 0.25, dz2b.sum((0, 2, 3)), 2e-3, "db2")
    check_close(p3.gw.cpu() - 0.5, w3v.grad, 2e-3, "dW3")
    check_close(p3.gb.cpu() - 0.25, gb.sum().reshape(1), 2e-3, "db3")


# RDB conv5 / pull-x (the 128 -> 64 implicit GEMM with the fused epilogues): ragged widths, images narrower than a
# tile, both epilogue forms incl. the optional second residual / aux output, bit-identical reruns.
RDB5_CASES = [
    (4, 64, 64, "conv5", True), (3, 37, 100, "conv5", False), (2, 32, 32, "pullx", True), (1, 9, 130, "pullx", False),
    (5, 64, 64, "pullx", True), (2, 13, 17, "conv5", True),
]


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w,mode,two", RDB5_CASES)
def test_conv5_pullx_matches_fp64(n, h, w, mode, two):
    """esrgan.py:26,38,54 (conv5 + x5 * 0.2 + x, the RRDB out * 0.2 + x) and its pull-x data gradient (fp32 out = conv +
    beta1 * g_out (+ g_skip), bf16 aux = aux_scale * out into the previous dZ5 slot) vs float64 on the same bf16
    operands.  Tolerances: fp32 out 1e-5 of the scale; bf16 out one rounding (2^-8 relative) of the fp32 value."""
    import climsr_amd.ops as ops

    dc, nf = 128, 64
    conv5 = mode == "conv5"
    p, wt, b = make_plan(dc, nf, 3, seed=31, bias=conv5)
    g = torch.Generator().manual_seed(32)
    x = bf(torch.rand((n, dc, h, w), generator=g) * 2 - 1)
    xin = to_nhwc(x)
    r1 = torch.rand((n, nf, h, w), generator=g) * 2 - 1
    r2 = torch.rand((n, nf, h, w), generator=g) * 2 - 1
    if conv5:
        y = torch.full((n, h, w, dc), 7.0, dtype=torch.bfloat16, device=DEV)  # the next RDB's dense buffer, channels 0..63
        r2d = to_nhwc(bf(r2), cs=dc)
        kw = dict(res1=xin, alpha1=0.2, res1_cs=dc, res1_co=0)
        if two:
            kw.update(res2=r2d, alpha2=0.2, res2_cs=dc, res2_co=0)
        ycs = dc
    else:
        y = torch.full((n, h, w, nf), 7.0, dtype=torch.float32, device=DEV)
        aux = torch.full((n, h, w, dc), 3.0, dtype=torch.bfloat16, device=DEV)
        kw = dict(use_bias=False, out_mode=OUT_F32, res1=to_nhwc(r1, dtype=torch.float32), res1_cs=nf, res1_co=0, beta1=0.2,
                  aux=aux, aux_cs=dc, aux_co=64, aux_scale=0.04)
        if two:
            kw.update(res2=to_nhwc(r2, dtype=torch.float32), res2_cs=nf, res2_co=0)
        ycs = nf
    names = []
    ops.PROFILER = lambda name, flops, fn, tag="", nbytes=0: (names.append(name), fn())
    try:
        p.fwd(xin, dc, 0, h, w, y, ycs, 0, n, **kw)
    finally:
        ops.PROFILER = None
    torch.cuda.synchronize()
    assert names and names[-1].startswith("conv_fwd_kernel<"), names
    first = y.clone()
    p.fwd(xin, dc, 0, h, w, y, ycs, 0, n, **kw)
    torch.cuda.synchronize()
    assert torch.equal(first, y), "rerun not bit-identical"
    want = F.conv2d(x.double(), bf(wt).double(), None if b is None else b.double(), padding=1)
    if conv5:
        want = want * 0.2 + x[:, :nf].double()
        if two:
            want = want * 0.2 + bf(r2).double()
        got = from_nhwc(y, nf).cpu().double()
        scale = want.abs().max().item()
        err = ((got - want).abs() - want.abs() * 2.0 ** -8).max().item()
        assert err <= 1e-5 * scale, f"conv5 bf16 err {err:.3e} vs scale {scale:.3e}"
        assert torch.all(y[..., nf:].float() == 7.0), "conv5 wrote outside its 64 channels"
    else:
        want = want + 0.2 * r1.double()
        if two:
            want = want + r2.double()
        got = from_nhwc(y, nf).cpu().double()
        check_close(got, want, what="pullx")
        ga = from_nhwc(aux, nf, 64).cpu().double()
        err = ((ga - 0.04 * want).abs() - (0.04 * want).abs() * 2.0 ** -8).max().item()
        assert err <= 1e-5 * 0.04 * want.abs().max().item(), f"pullx aux err {err:.3e}"
        assert torch.all(aux[..., :64].float() == 3.0), "pull-x aux wrote outside its slot"


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w,keep", [(2, 64, 64, True), (3, 40, 34, True), (2, 64, 96, False), (1, 30, 18, True)])
def test_d_stem_s2_matches_fp64(n, h, w, keep):
    """The RFB discriminator's features.0 (1 -> 64, LeakyReLU 0.2) + features.2 (64 -> 64 / stride 2) in one launch
    (csrc/stem.hip, rfb_esrgan.py:28-31) vs float64 on the same bf16 operands: a0 (kept output) within one bf16 rounding,
    z2 within 8e-3 of its scale (bf16 store), the BatchNorm partial sums per channel vs the fp64 sums of the stored z2
    (fp32 summation noise), bit-identical reruns; without `keep` nothing is written to a0."""
    from climsr_amd import ops

    g = torch.Generator().manual_seed(41)
    x = bf(torch.rand((n, 1, h, w), generator=g) * 2 - 1)
    w0 = ((torch.rand((64, 1, 3, 3), generator=g) * 2 - 1) / 3).to(DEV).contiguous()
    p2, w2, _b = make_plan(64, 64, 3, stride=2, seed=42, bias=False)
    x8 = to_nhwc(x, cs=8)
    oh, ow = (h + 1) // 2, (w + 1) // 2
    a0 = torch.full((n, h, w, 64), 5.0, dtype=torch.bfloat16, device=DEV) if keep else None
    z2 = torch.empty((n, oh, ow, 64), dtype=torch.bfloat16, device=DEV)
    nparts = ops.d_stem_s2_bn_parts(n, h, w)
    part = torch.full((nparts * 2 * 64,), float("nan"), dtype=torch.float64, device=DEV)
    ops.d_stem_s2(x8, 8, w0, p2, a0, z2, part, n, h, w)
    torch.cuda.synchronize()
    z_first, p_first = z2.clone(), part.clone()
    ops.d_stem_s2(x8, 8, w0, p2, a0, z2, part, n, h, w)
    torch.cuda.synchronize()
    assert torch.equal(z_first, z2) and torch.equal(p_first, part), "rerun not bit-identical"
    a_ref = F.leaky_relu(F.conv2d(x.double(), bf(w0.cpu()).double(), padding=1), 0.2)
    if keep:
        got_a = from_nhwc(a0, 64).cpu().double()
        err = ((got_a - a_ref).abs() - a_ref.abs() * 2.0 ** -8).max().item()
        assert err <= 1e-6 * a_ref.abs().max().item(), f"a0 err {err:.3e}"
    z_ref = F.conv2d(bf(a_ref.float()).double(), bf(w2).double(), padding=1, stride=2)
    got_z = from_nhwc(z2, 64).cpu().double()
    err = (got_z - z_ref).abs().max().item()
    assert err <= 8e-3 * z_ref.abs().max().item(), f"z2 err {err:.3e}"
    pp = part.view(nparts, 2, 64).cpu()
    s_ref = got_z.sum(dim=(0, 2, 3))
    q_ref = (got_z ** 2).sum(dim=(0, 2, 3))
    assert torch.allclose(pp[:, 0].sum(0), s_ref, rtol=1e-4, atol=1e-3 * (oh * ow * n) ** 0.5)
    assert torch.allclose(pp[:, 1].sum(0), q_ref, rtol=1e-4, atol=1e-3)


@pytest.mark.gpu
@pytest.mark.parametrize("cin,cout,n,h,w", [(64, 64, 2, 40, 36), (64, 64, 1, 18, 100), (128, 128, 2, 32, 48), (256, 256, 1, 96, 34),
                                            (128, 64, 2, 64, 16), (512, 512, 1, 32, 32)])
def test_conv_relu_maxpool_fused(cin, cout, n, h, w):
    """conv + bias + ReLU + 2x2 max pool in one kernel (the VGG19 block ends, losses/perceptual.py; the register-resident
    64 -> 64 conv's EP 5 or the LDS-DMA conv's EP 11) vs max_pool2d(relu(conv)) in fp64 on the same bf16 operands."""
    from climsr_amd import ops

    p, wt, b = make_plan(cin, cout, 3, seed=21)
    g = torch.Generator().manual_seed(22)
    x = bf(torch.rand((n, cin, h, w), generator=g) * 2 - 1)
    assert p.pool_ok(cin, h, w, n, cout)
    y = torch.full((n, h // 2, w // 2, cout), 7.0, dtype=torch.bfloat16, device=DEV)
    names = []
    ops.PROFILER = lambda name, flops, fn, tag="", nbytes=0: (names.append(name), fn())
    try:
        p.fwd(to_nhwc(x), cin, 0, h, w, y, cout, 0, n, act=ACT_RELU, pool2=True)
    finally:
        ops.PROFILER = None
    torch.cuda.synchronize()
    assert names and ("<5, 2>" in names[-1] or "<11, false>" in names[-1]), names
    want = F.max_pool2d(F.relu(F.conv2d(x.double(), bf(wt).double(), b.double(), padding=1)), 2)
    got = from_nhwc(y, cout).double().cpu()
    err = float((got - want).abs().max())
    assert err <= 2 ** -7 * float(want.abs().max()) + 1e-6, f"err {err:.3e} vs {float(want.abs().max()):.3e}"


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w", [(2, 64, 64), (1, 37, 70), (3, 16, 130)])
def test_vgg_conv1_1_one_channel_matches_fp64(n, h, w):
    """VGG19 conv1_1 + ReLU on torch.cat([x, x, x], 1) (perceptual.py:16,26-31) as one 1-channel conv with the summed
    of the per-channel bf16 weights (csrc/stem.hip climsr_vgg_conv1_1), two fp32 batches in one launch, vs float64 on the
    bf16-rounded images and weights (the 3-channel conv's operands): within one bf16 rounding of the output plus 2^-16 of
    sum |w x| (the w_hi + w_lo split of the summed weight); ragged tiles; bit-identical reruns."""
    from climsr_amd import ops

    g = torch.Generator().manual_seed(51)
    xa = torch.rand((n, 1, h, w), generator=g) * 2 - 1
    xb = torch.rand((n, 1, h, w), generator=g) * 2 - 1
    wt = ((torch.rand((64, 3, 3, 3), generator=g) * 2 - 1) / 4).contiguous()
    b = (torch.rand(64, generator=g) - 0.5) / 4
    y = torch.full((2 * n, h, w, 64), 9.0, dtype=torch.bfloat16, device=DEV)
    args = (xa.to(DEV).contiguous(), xb.to(DEV).contiguous(), n, h, w, wt.to(DEV), b.to(DEV), y)
    ops.vgg_conv1_1(*args)
    torch.cuda.synchronize()
    first = y.clone()
    ops.vgg_conv1_1(*args)
    torch.cuda.synchronize()
    assert torch.equal(first, y), "rerun not bit-identical"
    x = bf(torch.cat([xa, xb], 0)).double()
    x3 = torch.cat([x, x, x], 1)
    want = F.relu(F.conv2d(x3, bf(wt).double(), b.double(), padding=1))
    mag = F.conv2d(x3.abs(), bf(wt).double().abs(), padding=1)
    got = from_nhwc(y, 64).cpu().double()
    err = ((got - want).abs() - want.abs() * 2.0 ** -8 - mag * 2.0 ** -16).max().item()
    assert err <= 1e-6 * want.abs().max().item(), f"conv1_1 err {err:.3e}"
