"""GPU parity at the benchmarked shapes (BASELINE configs 2/3: B=32, LR 64 -> HR 256).

Several kernels dispatch only at bench-sized problems: ``conv_wgrad64_kernel<2>`` (8-wave tap split, >= 2^20 output
pixels: HRconv / upconv2 weight gradients at 256^2, B=32), the 64-way split-K grouped weight gradient of a residual
dense block at B=32, 64^2 (+ its row-sliced reduction), and ``conv_pw`` walking thousands of persistent XCD-ordered
tiles at 256^2, B=32.  Each is compared here with a float64 GEMM on the GPU (unfold + matmul, test-only torch ops)
over the same bf16-rounded operands: the only difference left is the kernels' fp32 accumulation order, bounded by
``REL`` of the result scale.  The last tests run one whole config-2 step (nb 11, B=32, 64->256) and the config-3
GAN passes (nb 1, B=32, 64->256) against the oracle (oracle/climsr_ref.py) evaluated in fp32 with torch ops on the
GPU, within the same envelope as the reference's own AMP training (test_gpu_generator.py)."""
import pytest
import torch
import torch.nn.functional as F

from oracle import climsr_ref as ref
from tests.helpers import gen_params, rfb_d_params, scalar_envelope, vgg_params

pytestmark = pytest.mark.gpu

DEV = "cuda"
REL = 5e-5  # fp32 accumulation over up to 2^21 products (split-K partials summed in a fixed order)


def bf(t):
    return t.to(torch.bfloat16).to(torch.float32)


def nhwc(x, cs=None, co=0):
    n, c, h, w = x.shape
    cs = cs or ((c + 7) // 8 * 8)
    buf = torch.zeros((n, h, w, cs), dtype=torch.bfloat16, device=DEV)
    buf[..., co:co + c] = x.permute(0, 2, 3, 1).to(torch.bfloat16)
    return buf


def wgrad64(x, dz, ks=3, pad=1, chunk=4):
    """dW[co][ci*k*k] = sum_px dz[px][co] * im2col(x)[px][ci*k*k] in float64 on the GPU, chunked over images."""
    out = None
    for i in range(0, x.shape[0], chunk):
        cols = F.unfold(x[i:i + chunk].double(), ks, padding=pad)           # [b, ci*k*k, L]
        d = dz[i:i + chunk].double().flatten(2)                              # [b, co, L]
        part = torch.einsum("bkl,bcl->ck", cols, d)
        out = part if out is None else out + part
    return out


def close(got, want, rel=REL, what=""):
    scale = float(want.abs().max()) + 1e-30
    err = float((got.double() - want.double()).abs().max())
    assert err <= rel * scale, f"{what}: max err {err:.3e} vs scale {scale:.3e} (rel {err / scale:.2e})"


def plan(cin, cout, ks=3, seed=0):
    from climsr_amd.ops import ConvPlan

    g = torch.Generator().manual_seed(seed)
    w = ((torch.rand((cout, cin, ks, ks), generator=g) * 2 - 1) / (cin * ks * ks) ** 0.5).to(DEV)
    b = ((torch.rand((cout,), generator=g) * 2 - 1) * 0.1).to(DEV)
    p = ConvPlan(cin, cout, ks, 1, None, "bench-shape")
    p.bind(w.contiguous(), b)
    p.pack()
    return p


def test_wgrad64_tap_split_upsampled_at_1m_pixels():
    """upconv2's weight gradient at the bench shape: x [32,64,128,128] nearest-x2 on load -> 256^2, 2^21 output
    pixels (>= 2^20 selects conv_wgrad64_kernel<2>)."""
    from climsr_amd import ops

    n, h = 32, 128
    p = plan(64, 64)
    g = torch.Generator(device=DEV).manual_seed(1)
    x = bf(torch.rand((n, 64, h, h), generator=g, device=DEV) * 2 - 1)
    dz = bf(torch.rand((n, 64, 2 * h, 2 * h), generator=g, device=DEV) * 2 - 1)
    p.gw = torch.zeros_like(p.weight)
    p.gb = torch.zeros_like(p.bias)
    names = []
    ops.PROFILER = lambda name, flops, fn, tag="", nbytes=0: (names.append(name), fn())
    try:
        p.wgrad(nhwc(x), 64, 0, h, h, nhwc(dz), 64, n, ops.Workspace(), accumulate=False, up=2)
    finally:
        ops.PROFILER = None
    torch.cuda.synchronize()
    assert "conv_wgrad64_kernel<2, 1>" in names, names
    xu = F.interpolate(x, scale_factor=2, mode="nearest")
    close(p.gw.reshape(64, -1), wgrad64(xu, dz), what="upconv2 wgrad")
    close(p.gb, dz.double().sum((0, 2, 3)), what="upconv2 bias grad")


def test_wgrad64_hrconv_accumulate_at_2m_pixels():
    """HRconv-shaped (64->64 at 256^2, B=32) weight gradient accumulated onto an existing gradient."""
    n, h = 32, 256
    p = plan(64, 64, seed=2)
    g = torch.Generator(device=DEV).manual_seed(2)
    x = bf(torch.rand((n, 64, h, h), generator=g, device=DEV) * 2 - 1)
    dz = bf(torch.rand((n, 64, h, h), generator=g, device=DEV) * 2 - 1)
    p.gw = torch.full_like(p.weight, 3.0)
    p.gb = torch.full_like(p.bias, -1.0)
    from climsr_amd import ops

    p.wgrad(nhwc(x), 64, 0, h, h, nhwc(dz), 64, n, ops.Workspace(), accumulate=True)
    torch.cuda.synchronize()
    close(p.gw.reshape(64, -1) - 3.0, wgrad64(x, dz), rel=1e-4, what="HRconv wgrad (+=)")
    close(p.gb + 1.0, dz.double().sum((0, 2, 3)), rel=1e-4, what="HRconv bias grad (+=)")


def test_rdb_grouped_wgrad_split_k_at_bench_shape():
    """One residual dense block's five weight gradients as the grouped 128 x 1152 GEMM at B=32, 64^2 (the 64-way
    split-K of conv_wgrad64_kernel<1> + wgrad_reduce_rows), vs per-conv float64 GEMMs."""
    from climsr_amd import ops

    n, h, nf, gc = 32, 64, 64, 16
    cins = [nf + k * gc for k in range(5)]
    couts = [gc] * 4 + [nf]
    plans = []
    for k in range(5):
        p = plan(cins[k], couts[k], seed=10 + k)
        p.gw = torch.full_like(p.weight, float("nan"))
        p.gb = torch.full_like(p.bias, float("nan"))
        plans.append(p)
    gw = ops.GroupedWgrad(plans, 128, "rdb")
    g = torch.Generator(device=DEV).manual_seed(3)
    dense = bf(torch.rand((n, 128, h, h), generator=g, device=DEV) * 2 - 1)
    dz = bf(torch.rand((n, 128, h, h), generator=g, device=DEV) * 2 - 1)
    ws = ops.Workspace()
    d_in, dz_in = nhwc(dense), nhwc(dz)
    from climsr_amd import _lib
    import ctypes

    d = _lib.ConvDesc(n, h, h, 128, 128, 0, 1, 3, 1, 1, h, h, 128, 0, 0, 8)
    assert _lib.load().climsr_conv2d_wgrad_splits(ctypes.byref(d)) >= 32  # the split-K path under test
    gw.run(d_in, 128, 0, h, h, dz_in, 128, n, ws, accumulate=False)
    torch.cuda.synchronize()
    off = 0
    for k, p in enumerate(plans):
        want = wgrad64(dense[:, :cins[k]], dz[:, off:off + couts[k]])
        close(p.gw.reshape(couts[k], -1), want, what=f"RDB conv{k + 1} wgrad")
        close(p.gb, dz[:, off:off + couts[k]].double().sum((0, 2, 3)), what=f"RDB conv{k + 1} bias grad")
        off += couts[k]


@pytest.mark.parametrize("cin,cout,h", [(64, 64, 256), (128, 128, 128), (256, 256, 64), (512, 512, 32)])
def test_wgrad64_stride2_discriminator_layers(cin, cout, h):
    """The RFB discriminator's stride-2 convs (features.2/8/14/20, rfb_esrgan.py:29-49) at B=32 of 256^2 tiles: weight
    gradient on conv_wgrad64_glds_s2_kernel (4 x 16 output tiles over a (2*4+1) x (2*16+1) input footprint, LDS-DMA)."""
    from climsr_amd import ops

    n = 32
    p = plan(cin, cout, seed=cin)
    p2 = ops.ConvPlan(cin, cout, 3, 2, 1, "s2")
    p2.bind(p.weight, None)
    p2.pack()
    g = torch.Generator(device=DEV).manual_seed(cin)
    x = bf(torch.rand((n, cin, h, h), generator=g, device=DEV) * 2 - 1)
    dz = bf(torch.rand((n, cout, h // 2, h // 2), generator=g, device=DEV) * 2 - 1)
    p2.gw = torch.zeros_like(p2.weight)
    names = []
    ops.PROFILER = lambda name, flops, fn, tag="", nbytes=0: (names.append(name), fn())
    try:
        p2.wgrad(nhwc(x), cin, 0, h, h, nhwc(dz), cout, n, ops.Workspace(), accumulate=False)
    finally:
        ops.PROFILER = None
    torch.cuda.synchronize()
    assert "conv_wgrad64_glds_s2_kernel" in names, names
    want = None
    for i in range(0, n, 4):
        cols = F.unfold(x[i:i + 4].double(), 3, padding=1, stride=2)
        part = torch.einsum("bkl,bcl->ck", cols, dz[i:i + 4].double().flatten(2))
        want = part if want is None else want + part
    close(p2.gw.reshape(cout, -1), want, what=f"stride-2 wgrad {cin}->{cout} @{h}")


@pytest.mark.parametrize("act", [0, 1])
def test_conv_pw_forward_at_256_b32(act):
    """HRconv forward at 256^2, B=32 (conv_wr: weights in registers, 32768 wave tiles walked by a persistent
    XCD-ordered grid), bias (+ LeakyReLU)."""
    from climsr_amd import ops

    n, h = 32, 256
    p = plan(64, 64, seed=4)
    g = torch.Generator(device=DEV).manual_seed(4)
    x = bf(torch.rand((n, 64, h, h), generator=g, device=DEV) * 2 - 1)
    y = torch.empty((n, h, h, 64), dtype=torch.bfloat16, device=DEV)
    names = []
    ops.PROFILER = lambda name, flops, fn, tag="", nbytes=0: (names.append(name), fn())
    try:
        p.fwd(nhwc(x), 64, 0, h, h, y, 64, 0, n, act=act)
    finally:
        ops.PROFILER = None
    torch.cuda.synchronize()
    assert any(s.startswith("conv_wr_kernel") for s in names), names
    for i in range(0, n, 8):  # float64 reference, 8 images at a time
        want = F.conv2d(x[i:i + 8].double(), bf(p.weight).double(), p.bias.double(), padding=1)
        if act == 1:
            want = F.leaky_relu(want, 0.2)
        got = y[i:i + 8].permute(0, 3, 1, 2).double()
        err = float((got - want).abs().max())
        assert err <= 2 ** -7 * float(want.abs().max()) + 1e-6, f"images {i}..: err {err:.3e}"  # one bf16 ulp of the output


def test_conv_pw_dgrad_down2_at_256_b32():
    """upconv2's data gradient at the bench shape: conv^T of dz [32,64,256,256], summed over 2x2 blocks (backward of
    the nearest x2 feeding it), LeakyReLU' of upconv1's stored activation, bf16 out at 128^2."""
    from climsr_amd import ops

    n, h = 32, 128
    p = plan(64, 64, seed=5)
    g = torch.Generator(device=DEV).manual_seed(5)
    dz = bf(torch.rand((n, 64, 2 * h, 2 * h), generator=g, device=DEV) * 2 - 1)
    act_out = bf(torch.rand((n, 64, h, h), generator=g, device=DEV) * 2 - 1)
    gx = torch.empty((n, h, h, 64), dtype=torch.bfloat16, device=DEV)
    p.dgrad(nhwc(dz), 64, 2 * h, 2 * h, gx, 64, 0, n, down2=True, act=ops.ACT_LRELU_BWD, res1=nhwc(act_out), res1_cs=64)
    torch.cuda.synchronize()
    for i in range(0, n, 8):
        x = torch.zeros((8, 64, h, h), dtype=torch.float64, device=DEV, requires_grad=True)
        y = F.conv2d(F.interpolate(x, scale_factor=2, mode="nearest"), bf(p.weight).double(), None, padding=1)
        (want,) = torch.autograd.grad(y, x, dz[i:i + 8].double())
        want = want * torch.where(act_out[i:i + 8] > 0, 1.0, 0.2).double()
        got = gx[i:i + 8].permute(0, 3, 1, 2).double()
        err = float((got - want).abs().max())
        assert err <= 2 ** -7 * float(want.abs().max()) + 1e-6, f"images {i}..: err {err:.3e}"


# ------------------------------------------------------------------ whole steps at the bench shape
def _gemm_conv(p, name, x, stride=1, padding=None):
    """The oracle's conv (oracle/climsr_ref.py _conv) as unfold + matmul: rocBLAS GEMMs instead of MIOpen, whose
    per-shape kernel compilation on a fresh box takes minutes.  Same math, autocast-able."""
    w = p[name + ".weight"]
    b = p.get(name + ".bias")
    ks = w.shape[-1]
    pad = ks // 2 if padding is None else padding
    n, _c, h, wd = x.shape
    oh, ow = (h + 2 * pad - ks) // stride + 1, (wd + 2 * pad - ks) // stride + 1
    cols = F.unfold(x, ks, padding=pad, stride=stride)
    y = torch.matmul(w.reshape(w.shape[0], -1), cols)
    if b is not None:
        y = y + b.reshape(1, -1, 1).to(y.dtype)
    return y.reshape(n, w.shape[0], oh, ow)


@pytest.fixture
def gemm_oracle(monkeypatch):
    monkeypatch.setattr(ref, "_conv", _gemm_conv)
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False


def _log(*a):
    print("[bench-shape]", *a, flush=True)


def _cos(a, b):
    return float((a * b).sum() / (a.norm() * b.norm() + 1e-30))


def _envelope(native, ref32, amps, what):
    """Per-tensor, against the fp32 reference: relative L2 error <= max(2x the AMP runs' own error, 2e-2), and
    cosine >= min(0.97, 1 - 2 (1 - cos of the worse AMP run)) -- the reference's own fp16 training (and torch's bf16
    autocast) is the yardstick for how far a reduced-precision forward moves a random-init gradient."""
    bad = []
    for k, want in ref32.items():
        got = native[k]
        rel = float((got - want).norm() / (want.norm() + 1e-30))
        rel_amp = max(float((a[k] - want).norm() / (want.norm() + 1e-30)) for a in amps)
        cos = _cos(got, want)
        cos_amp = min(_cos(a[k], want) for a in amps)
        if rel > max(2.0 * rel_amp, 2e-2) or cos < min(0.97, 1.0 - 2.0 * (1.0 - cos_amp)):
            bad.append((k, round(rel, 4), round(rel_amp, 4), round(cos, 4), round(cos_amp, 4)))
    assert not bad, f"{what}: {len(bad)} tensors outside the AMP envelope: {bad[:6]}"


def _oracle_grads(p32, keys, loss_fn, dtype=None):
    p = {k: v.detach().clone().requires_grad_(k in keys) for k, v in p32.items()}
    if dtype is None:
        loss = loss_fn(p)
    else:
        with torch.autocast("cuda", dtype=dtype):
            loss = loss_fn(p)
    grads = torch.autograd.grad(loss.float() * 65536.0, [p[k] for k in keys])
    _log("oracle", dtype, "loss", float(loss))
    return float(loss), {k: (g_.double() / 65536.0) for k, g_ in zip(keys, grads)}


def test_config2_step_b32_nb11_vs_oracle_fp32(gemm_oracle):
    """Config 2's whole L1-pretrain forward + backward at the bench shape (nb 11, B=32, 64->256): the loss and every
    one of the 348 parameter gradients vs the oracle in fp32 on the GPU, in the AMP envelope."""
    from climsr_amd.losses.l1 import l1_loss
    from climsr_amd.models.esrgan import ESRGANGenerator

    nb = 11
    g = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=nb, gc=16, scale_factor=4)
    p32 = gen_params(nb, torch.float32)
    g.load_state_dict(p32)
    g = g.to(DEV)
    bt = {k: v.to(DEV) for k, v in ref.synthetic_batch(32, 256, seed=42).items()}
    loss = l1_loss(g(bt["lr"], bt["elevation"], bt["mask"]), bt["hr"])
    loss.backward()
    torch.cuda.synchronize()
    native = {k: p.grad.double() for k, p in g.named_parameters()}
    _log("native config-2 loss", float(loss))
    pd = {k: v.to(DEV) for k, v in p32.items()}
    keys = list(pd.keys())

    def fn(p):
        return ref.l1_loss(ref.generator_forward(p, bt["lr"], bt["elevation"], bt["mask"], nb).float(), bt["hr"])

    l32, g32 = _oracle_grads(pd, keys, fn)
    l16, g16 = _oracle_grads(pd, keys, fn, torch.float16)
    lbf, gbf = _oracle_grads(pd, keys, fn, torch.bfloat16)
    scalar_envelope("config-2 nb-11 B=32 L1 loss", float(loss), l32, [l16, lbf])
    _envelope(native, g32, [g16, gbf], "config-2 step gradients")


def test_config3_gan_passes_b32_vs_oracle_fp32(gemm_oracle):
    """Config 3's two passes at the bench shape (nb 1, B=32, 64->256; RFB discriminator with train-mode BN over 32
    tiles, VGG19 perceptual): the generator pass's loss_G + G gradients and the discriminator pass's loss_D + D
    gradients vs the oracle in fp32 on the GPU (same weights, no optimizer step in between), in the AMP envelope."""
    from climsr_amd.task.pl_gan import GANLightningModule

    nb = 1
    m = GANLightningModule(
        generator={"_target_": "climsr_amd.models.esrgan.ESRGANGenerator", "in_channels": 3, "out_channels": 1, "nf": 64, "nb": nb,
                   "gc": 16, "scale_factor": 4},
        discriminator={"_target_": "climsr_amd.models.rfb_esrgan.RFBESRGANDiscriminator", "in_channels": 1})
    gp, dp = gen_params(nb, torch.float32), rfb_d_params(torch.float32)
    m.generator.load_state_dict(gp)
    m.discriminator.load_state_dict(dp)
    m = m.to(DEV)
    vp = {k: v.float().to(DEV) for k, v in vgg_params().items()}
    bt = {k: v.to(DEV) for k, v in ref.synthetic_batch(32, 256, seed=42).items()}
    G, D = m.generator, m.discriminator
    # ---- pass 0 (D frozen)
    for p in D.parameters():
        p.requires_grad_(False)
    hr, sr = m.common_step(bt)
    losses_g = m.loss_g(hr, sr)
    lg = losses_g[3]
    lg.backward()
    torch.cuda.synchronize()
    g_native = {k: p.grad.double() for k, p in G.named_parameters()}
    _log("native pass-0 loss_G", float(lg))
    # ---- pass 1 (G frozen, fresh G forward with the same weights)
    for p in D.parameters():
        p.requires_grad_(True)
    for p in G.parameters():
        p.requires_grad_(False)
    with torch.no_grad():
        _hr, sr2 = m.common_step(bt)
    ld = m.loss_d(hr, sr2)
    ld.backward()
    torch.cuda.synchronize()
    d_native = {k: p.grad.double() for k, p in D.named_parameters()}
    _log("native pass-1 loss_D", float(ld))

    gpd = {k: v.to(DEV) for k, v in gp.items()}
    dpd = {k: (v.to(DEV)) for k, v in dp.items()}

    def d_fn(p):
        return lambda t: ref.rfb_discriminator_forward(p, t, training=True, update_stats=False)

    comps = []  # the oracle's (perceptual, adversarial, pixel, loss_G) per precision: fp32, fp16, bf16

    def pass0(p):
        sr_ = ref.generator_forward(p, bt["lr"], bt["elevation"], bt["mask"], nb).float()
        out = ref.loss_g(d_fn(dpd), vp, bt["hr"], sr_)
        comps.append([float(t) for t in out])
        return out[3]

    gkeys = list(gpd.keys())
    _l32, g32 = _oracle_grads(gpd, gkeys, pass0)
    _a, g16 = _oracle_grads(gpd, gkeys, pass0, torch.float16)
    _b, gbf = _oracle_grads(gpd, gkeys, pass0, torch.bfloat16)
    for i, name in enumerate(("perceptual_loss", "adversarial_loss", "pixel_level_loss", "loss_G")):
        scalar_envelope(f"config-3 pass-0 {name}", float(losses_g[i]), comps[0][i], [comps[1][i], comps[2][i]])
    _envelope(g_native, g32, [g16, gbf], "GAN pass-0 generator gradients")

    with torch.no_grad():
        sr_ref = ref.generator_forward(gpd, bt["lr"], bt["elevation"], bt["mask"], nb).float()
    dkeys = ref.trainable_keys(dpd)

    def pass1(p):
        return ref.loss_d(d_fn(p), bt["hr"], sr_ref)

    l32d, d32 = _oracle_grads(dpd, dkeys, pass1)
    l16d, d16 = _oracle_grads(dpd, dkeys, pass1, torch.float16)
    lbfd, dbf = _oracle_grads(dpd, dkeys, pass1, torch.bfloat16)
    scalar_envelope("config-3 pass-1 loss_D", float(ld), l32d, [l16d, lbfd])
    _envelope(d_native, d32, [d16, dbf], "GAN pass-1 discriminator gradients")


def test_config3_gan_pass0_losses_nb11_b32(gemm_oracle):
    """Config 3 at its benched depth (nb 11, B=32, 64->256): the generator pass's four loss scalars (perceptual,
    adversarial, pixel, loss_G; pl_gan.py:28-49) from the native training forward vs the oracle's fp32 forward on the
    GPU, each within 2x the oracle's own autocast fp16 / bf16 spread or SURVEY's 1e-3."""
    from climsr_amd.task.pl_gan import GANLightningModule

    nb = 11
    m = GANLightningModule(
        generator={"_target_": "climsr_amd.models.esrgan.ESRGANGenerator", "in_channels": 3, "out_channels": 1, "nf": 64, "nb": nb,
                   "gc": 16, "scale_factor": 4},
        discriminator={"_target_": "climsr_amd.models.rfb_esrgan.RFBESRGANDiscriminator", "in_channels": 1})
    gp, dp = gen_params(nb, torch.float32), rfb_d_params(torch.float32)
    m.generator.load_state_dict(gp)
    m.discriminator.load_state_dict(dp)
    m = m.to(DEV)
    for p in m.discriminator.parameters():
        p.requires_grad_(False)
    bt = {k: v.to(DEV) for k, v in ref.synthetic_batch(32, 256, seed=42).items()}
    hr, sr = m.common_step(bt)
    native = [float(t) for t in m.loss_g(hr, sr)]
    torch.cuda.synchronize()
    vp = {k: v.float().to(DEV) for k, v in vgg_params().items()}
    gpd, dpd = {k: v.to(DEV) for k, v in gp.items()}, {k: v.to(DEV) for k, v in dp.items()}

    def oracle(dtype):
        with torch.no_grad(), torch.autocast("cuda", dtype=dtype or torch.float16, enabled=dtype is not None):
            sr_ = ref.generator_forward(gpd, bt["lr"], bt["elevation"], bt["mask"], nb).float()
            d = lambda t: ref.rfb_discriminator_forward(dpd, t, training=True, update_stats=False)  # noqa: E731
            return [float(t) for t in ref.loss_g(d, vp, bt["hr"], sr_)]

    o32, o16, obf = oracle(None), oracle(torch.float16), oracle(torch.bfloat16)
    for i, name in enumerate(("perceptual_loss", "adversarial_loss", "pixel_level_loss", "loss_G")):
        scalar_envelope(f"config-3 nb-11 pass-0 {name}", native[i], o32[i], [o16[i], obf[i]])


@pytest.mark.parametrize("c,h", [(64, 128), (128, 128), (256, 32), (512, 16)])
def test_batchnorm_train_at_bench_shapes(c, h):
    """RFB discriminator BatchNorm2d + LeakyReLU(0.2) (rfb_esrgan.py:32-50) at B=32 bench sizes: batch statistics,
    running-stat update, num_batches_tracked, the fused apply and the backward (dgamma, dbeta, dz) vs float64."""
    from climsr_amd import ops

    n = 32
    npix = n * h * h
    g = torch.Generator(device=DEV).manual_seed(c + h)
    z = bf(torch.randn((npix, c), generator=g, device=DEV) * 1.7 + 0.4)  # off-centre: exercises the variance formula
    zb = z.to(torch.bfloat16)
    gamma = torch.rand(c, generator=g, device=DEV) + 0.5
    beta = torch.rand(c, generator=g, device=DEV) - 0.5
    rm, rv = torch.zeros(c, device=DEV), torch.ones(c, device=DEV)
    nbt = torch.zeros((), dtype=torch.int64, device=DEV)
    mean, rstd = torch.empty(c, device=DEV), torch.empty(c, device=DEV)
    y = torch.empty((npix, c), dtype=torch.bfloat16, device=DEV)
    cache = {}
    ops.bn_forward(zb, npix, c, gamma, beta, mean, rstd, y, ops.bn_workspace(npix, c, cache, z.device), rm, rv,
                   num_batches_tracked=nbt)
    torch.cuda.synchronize()
    zd = z.double()
    m64 = zd.mean(0)
    v64 = zd.var(0, unbiased=False)
    close(mean, m64, rel=1e-6, what="mean")
    close(rstd, 1 / torch.sqrt(v64 + 1e-5), rel=1e-5, what="rstd")
    close(rm, 0.1 * m64, rel=1e-5, what="running_mean")
    close(rv, 0.9 + 0.1 * zd.var(0, unbiased=True), rel=1e-5, what="running_var")
    assert int(nbt) == 1
    y64 = F.leaky_relu((zd - m64) / torch.sqrt(v64 + 1e-5) * gamma.double() + beta.double(), 0.2)
    err = float((y.double() - y64).abs().max())
    assert err <= 2 ** -7 * float(y64.abs().max()), f"bn apply err {err:.3e}"
    # backward through lrelu(bn(z)), lrelu' from the stored bf16 activation (as the kernel does)
    da = torch.randn((npix, c), generator=g, device=DEV)
    dz = torch.empty((npix, c), dtype=torch.bfloat16, device=DEV)
    coef = torch.empty(3 * c, device=DEV)
    dgam, dbet = torch.full((c,), 2.0, device=DEV), torch.full((c,), -3.0, device=DEV)
    ops.bn_backward(da, y, zb, npix, c, mean, rstd, gamma, ops.bn_workspace(npix, c, cache, z.device), coef, dgam, dbet, True, dz)
    torch.cuda.synchronize()
    d = da.double() * torch.where(y > 0, 1.0, 0.2).double()
    xh = (zd - mean.double()) * rstd.double()
    close(dgam - 2.0, (d * xh).sum(0), rel=1e-5, what="dgamma (+=)")
    close(dbet + 3.0, d.sum(0), rel=1e-5, what="dbeta (+=)")
    dz64 = gamma.double() * rstd.double() * (d - d.mean(0) - xh * (d * xh).mean(0))
    err = float((dz.double() - dz64).abs().max())
    assert err <= 2 ** -7 * float(dz64.abs().max()), f"bn backward dz err {err:.3e}"
    # the activation-free form (rfb_esrgan.py's D backward): bf16 da, lrelu' recomputed from z -- the same
    # decisions as the stored activation's sign, so the same float64 reference with the bf16-rounded da
    beta = torch.rand(c, generator=g, device=DEV) - 0.5
    ops.bn_forward(zb, npix, c, gamma, beta, mean, rstd, y, ops.bn_workspace(npix, c, cache, z.device))
    dab = da.to(torch.bfloat16)
    dz2 = torch.empty_like(dz)
    dgam2, dbet2 = torch.zeros(c, device=DEV), torch.zeros(c, device=DEV)
    ops.bn_backward_z(dab, zb, npix, c, mean, rstd, gamma, beta, ops.bn_workspace(npix, c, cache, z.device), coef, dgam2, dbet2,
                      False, dz2)
    torch.cuda.synchronize()
    d = dab.double() * torch.where(y > 0, 1.0, 0.2).double()
    xh = (zd - mean.double()) * rstd.double()
    close(dgam2, (d * xh).sum(0), rel=1e-5, what="dgamma (from z)")
    close(dbet2, d.sum(0), rel=1e-5, what="dbeta (from z)")
    dz64 = gamma.double() * rstd.double() * (d - d.mean(0) - xh * (d * xh).mean(0))
    err = float((dz2.double() - dz64).abs().max())
    assert err <= 2 ** -7 * float(dz64.abs().max()), f"bn backward (from z) dz err {err:.3e}"


@pytest.mark.parametrize("n,k,o", [(32, 100352, 1024), (2, 8192, 96), (20, 4096, 256)])
def test_linear_fwd_dgrad_wgrad_vs_float64(n, k, o):
    """fc.0 of the RFB discriminator (rfb_esrgan.py:57: Linear(100352, 1024) + LeakyReLU, B=32) and the plain
    discriminator's padded head: forward (wide / narrow split-K + reduce), data gradient and weight gradient (+=)
    vs float64 matmuls of the same bf16 operands."""
    from climsr_amd import ops

    g = torch.Generator(device=DEV).manual_seed(n + o)
    x = (torch.randn((n, k), generator=g, device=DEV) * 0.5).to(torch.bfloat16)
    w = (torch.randn((o, k), generator=g, device=DEV) / k ** 0.5).to(torch.bfloat16)
    b = torch.randn(o, generator=g, device=DEV) * 0.1
    y = torch.empty((n, o), device=DEV)
    ws = torch.empty((3072 // max(1, o // 64) + 2) * n * o, device=DEV)
    ops.linear_fwd(x, w, b, n, k, o, y, ws, act=ops.ACT_LRELU, slope=0.2)
    torch.cuda.synchronize()
    want = F.leaky_relu(x.double() @ w.double().t() + b.double(), 0.2)
    close(y, want, rel=1e-5, what="linear fwd")
    dy = (torch.randn((n, o), generator=g, device=DEV)).to(torch.bfloat16)
    dx = torch.full((n, k), 1.5, device=DEV)
    ops.linear_dgrad(dy, w, n, k, o, dx, accumulate=True)
    torch.cuda.synchronize()
    close(dx - 1.5, dy.double() @ w.double(), rel=1e-5, what="linear dgrad (+=)")
    n_pad = (n + 31) // 32 * 32
    dy_t = torch.zeros((o, n_pad), dtype=torch.bfloat16, device=DEV)
    dy_t[:, :n] = dy.t()
    x_t = torch.zeros((k, n_pad), dtype=torch.bfloat16, device=DEV)
    x_t[:, :n] = x.t()
    if o % 64 == 0:
        dw = torch.zeros((o, k), device=DEV)
        ops.linear_wgrad(dy_t, x_t, n_pad, k, o, dw, accumulate=False)
        torch.cuda.synchronize()
        close(dw, dy.double().t() @ x.double(), rel=1e-5, what="linear wgrad")


@pytest.mark.parametrize("acc", [False, True])
def test_linear_wgrad2_two_batches_vs_float64(acc):
    """climsr_linear_wgrad2: fc.0's weight gradient over the discriminator's two backward calls of loss_d (real and fake
    batches, pl_gan.py:51-61) in one launch, with and without accumulation, vs float64 at the bench shape."""
    from climsr_amd import ops

    n, k, o = 32, 100352, 1024
    g = torch.Generator(device=DEV).manual_seed(11 + int(acc))
    cols = []
    for _ in range(2):
        dy_t = torch.randn((o, n), generator=g, device=DEV).to(torch.bfloat16)
        x_t = (torch.randn((k, n), generator=g, device=DEV) * 0.5).to(torch.bfloat16)
        cols.append((dy_t, x_t))
    dw = torch.full((o, k), 0.5, device=DEV)
    ops.linear_wgrad2(cols[0][0], cols[0][1], n, cols[1][0], cols[1][1], n, k, o, dw, acc)
    torch.cuda.synchronize()
    want = sum(dy_t.double() @ x_t.double().t() for dy_t, x_t in cols)
    close(dw - 0.5 if acc else dw, want, rel=1e-5, what="linear wgrad2")


@pytest.mark.parametrize("act", [0, 1, 2])
@pytest.mark.parametrize("train", [True, False])
def test_batchnorm_apply_every_activation(act, train):
    """The BatchNorm apply for each activation it is compiled for (bn_apply_kernel<MODE, ACT>: none, LeakyReLU(0.2),
    ReLU) in both modes -- batch statistics (climsr_bn_forward) and running statistics (climsr_bn_inference, eval-mode
    BatchNorm2d) -- vs float64, on a ragged pixel count."""
    from climsr_amd import ops

    npix, c = 4099, 64
    g = torch.Generator(device=DEV).manual_seed(11 + act + 3 * train)
    z = bf(torch.randn((npix, c), generator=g, device=DEV) * 1.3 - 0.2)
    gamma = torch.rand(c, generator=g, device=DEV) + 0.5
    beta = torch.rand(c, generator=g, device=DEV) - 0.5
    y = torch.empty((npix, c), dtype=torch.bfloat16, device=DEV)
    zd = z.double()
    if train:
        mean, rstd = torch.empty(c, device=DEV), torch.empty(c, device=DEV)
        ops.bn_forward(z.to(torch.bfloat16), npix, c, gamma, beta, mean, rstd, y, ops.bn_workspace(npix, c, {}, z.device), act=act)
        m64, r64 = zd.mean(0), 1 / torch.sqrt(zd.var(0, unbiased=False) + 1e-5)
    else:
        rm = torch.randn(c, generator=g, device=DEV) * 0.1
        rv = torch.rand(c, generator=g, device=DEV) + 0.5
        ops.bn_inference(z.to(torch.bfloat16), npix, c, rm, rv, gamma, beta, y, act=act)
        m64, r64 = rm.double(), 1 / torch.sqrt(rv.double() + 1e-5)
    torch.cuda.synchronize()
    x64 = (zd - m64) * r64 * gamma.double() + beta.double()
    y64 = {0: x64, 1: F.leaky_relu(x64, 0.2), 2: F.relu(x64)}[act]
    err = float((y.double() - y64).abs().max())
    assert err <= 2 ** -7 * float(y64.abs().max()), f"act {act}: err {err:.3e}"
