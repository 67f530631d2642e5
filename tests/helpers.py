"""Shared test helpers: deterministic parameter dicts for the oracle, keyed like the reference."""
import numpy as np
import torch

from climsr_amd.core.init import init_state, spec_from_shapes
from oracle import climsr_ref as ref


def gen_params(nb=1, dtype=torch.float64, in_channels=3):
    shapes = ref.generator_shapes(in_channels=in_channels, nb=nb)
    st = init_state(spec_from_shapes(shapes))
    return {k: torch.from_numpy(np.asarray(v)).to(dtype) for k, v in st.items()}


def rfb_d_params(dtype=torch.float64):
    shapes = ref.rfb_discriminator_shapes()
    st = init_state(spec_from_shapes(shapes, ref.rfb_bn_prefixes()))
    return {k: (torch.from_numpy(np.asarray(v)).to(dtype) if np.asarray(v).dtype != np.int64 else torch.from_numpy(np.asarray(v)))
            for k, v in st.items()}


def plain_d_params(dtype=torch.float64):
    shapes = ref.plain_discriminator_shapes()
    st = init_state(spec_from_shapes(shapes, ref.plain_bn_prefixes()))
    return {k: (torch.from_numpy(np.asarray(v)).to(dtype) if np.asarray(v).dtype != np.int64 else torch.from_numpy(np.asarray(v)))
            for k, v in st.items()}


def vgg_params(dtype=torch.float64):
    shapes = ref.vgg19_shapes()
    st = init_state(spec_from_shapes(shapes), gain=float(np.sqrt(6.0)))
    return {k: torch.from_numpy(np.asarray(v)).to(dtype) for k, v in st.items()}


def psnr(a, b, data_range=None):
    a = a.double()
    b = b.double()
    if data_range is None:
        data_range = float(b.max() - b.min())
    mse = float(((a - b) ** 2).mean())
    return float("inf") if mse == 0 else 10 * np.log10(data_range ** 2 / mse)


def ssim(a, b, data_range=None, kernel=11, sigma=1.5):
    """Gaussian-window SSIM (torchmetrics defaults: 11x11, sigma 1.5, k1 .01, k2 .03, valid region)."""
    import torch.nn.functional as F

    a = a.double()
    b = b.double()
    if data_range is None:
        data_range = float(b.max() - b.min())
    x = torch.arange(kernel, dtype=torch.float64) - (kernel - 1) / 2
    g = torch.exp(-(x ** 2) / (2 * sigma ** 2))
    g = g / g.sum()
    w = (g[:, None] * g[None, :])[None, None].repeat(a.shape[1], 1, 1, 1)
    c1 = (0.01 * data_range) ** 2
    c2 = (0.03 * data_range) ** 2

    def f(t):
        return F.conv2d(t, w, groups=a.shape[1])

    mu_a, mu_b = f(a), f(b)
    saa = f(a * a) - mu_a ** 2
    sbb = f(b * b) - mu_b ** 2
    sab = f(a * b) - mu_a * mu_b
    m = ((2 * mu_a * mu_b + c1) * (2 * sab + c2)) / ((mu_a ** 2 + mu_b ** 2 + c1) * (saa + sbb + c2))
    return float(m.mean())


def gemm_conv(p, name, x, stride=1, padding=None):
    """The oracle's conv (oracle/climsr_ref.py _conv) as unfold + matmul: rocBLAS GEMMs instead of MIOpen (whose per-shape
    kernel compilation on a fresh box takes minutes).  Same math, autocast-able.  Test-only (monkeypatched in)."""
    import torch.nn.functional as F

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


def rel_l2(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


def pool_small(tensors, below):
    """The dict with every tensor of fewer than `below` elements replaced by one concatenated entry (key order): a
    16-element bias gradient's relative error is a handful of sign-random terms, pooled it is a statistic."""
    big = {k: v for k, v in tensors.items() if v.numel() >= below}
    small = [v.reshape(-1).double() for k, v in tensors.items() if v.numel() < below]
    if small:
        big[f"<{len(small)} tensors under {below} elements>"] = torch.cat(small)
    return big


def update_envelope(native, ref64, amps, floor=2e-2, pool_below=0):
    """Per tensor: the relative L2 distance of the native update (or gradient) from the fp64 oracle's must stay within
    2x the reduced-precision spread of the same quantity -- the larger of the oracle's own torch-autocast fp16 / bf16
    runs' distances from it (the reference trains with precision 16) and of those two runs' distance from each other
    (two equally valid reduced-precision runs: the noise level of the statistic itself, which for a small tensor is a
    few sign flips of Adam's ~lr*sign(grad) first steps) -- or ``floor``.  pool_below: tensors under that many elements
    are compared as one pooled vector (pool_small).  Returns (offenders, worst, per-tensor table)."""
    if pool_below:
        native, ref64, amps = pool_small(native, pool_below), pool_small(ref64, pool_below), [pool_small(a, pool_below) for a in amps]
    rows = {}
    for k, want in ref64.items():
        rel = rel_l2(native[k], want)
        rel_amp = max(rel_l2(a[k], want) for a in amps)
        for i in range(len(amps)):
            for j in range(i + 1, len(amps)):
                rel_amp = max(rel_amp, rel_l2(amps[i][k], amps[j][k]))
        rows[k] = (rel, rel_amp)
    bad = [(k, round(r, 4), round(ra, 4)) for k, (r, ra) in rows.items() if r > max(2.0 * ra, floor)]
    worst = max(rows.items(), key=lambda kv: kv[1][0] / max(2.0 * kv[1][1], floor))
    return bad, worst, rows


SCALAR_CAP = 1e-3  # loss scalars rel <= 1e-3 (bf16)


def scalar_envelope(what, got, want, amps, cap=SCALAR_CAP):
    """A loss scalar vs the oracle's value on the same inputs: relative deviation <= 2x the reduced-precision spread of
    the same scalar (the oracle's own torch-autocast fp16 / bf16 values' distances from ``want`` and from each other,
    as update_envelope does for tensors), or ``cap`` (SURVEY's 1e-3) where that spread is smaller.  Prints the measured
    deviations; returns (rel, bound)."""
    den = abs(want) + 1e-30
    rel = abs(got - want) / den
    rel_amp = max(abs(a - want) / den for a in amps)
    for i in range(len(amps)):
        for j in range(i + 1, len(amps)):
            rel_amp = max(rel_amp, abs(amps[i] - amps[j]) / den)
    bound = max(2.0 * rel_amp, cap)
    print(f"[loss-scalar] {what}: native {got:.7g} oracle {want:.7g} rel {rel:.3e} autocast {rel_amp:.3e} bound {bound:.3e}",
          flush=True)
    assert rel <= bound, (what, got, want, rel, rel_amp)
    return rel, bound


def scalar_cap(what, got, want, cap=SCALAR_CAP):
    """A loss scalar vs a reference value with no autocast runs beside it: SURVEY 8c's rel <= 1e-3, measured value
    printed."""
    rel = abs(got - want) / (abs(want) + 1e-30)
    print(f"[loss-scalar] {what}: native {got:.7g} reference {want:.7g} rel {rel:.3e} bound {cap:.1e}", flush=True)
    assert rel <= cap, (what, got, want, rel)
    return rel


RCAN_TRAIN = {"rcan_g2b2_x4": (2, 2, 4, 2, 16), "rcan_g1b2_x2": (1, 2, 2, 2, 12), "rcan_g1b1_x3": (1, 1, 3, 1, 10)}


def rcan_train_batch(b, lr_size, sf, seed=7, dtype=torch.float64):
    """The inputs of tests/golden/make_rcan_golden.py's training records: hr [b,1,H,W] in [-1,1), elev, mask, and
    lr = cat[hr, elev, mask] subsampled by sf (the reference RCAN's 3-channel input)."""
    hrs = lr_size * sf
    g = torch.Generator().manual_seed(seed)
    hr = torch.rand((b, 1, hrs, hrs), generator=g, dtype=torch.float64) * 2 - 1
    e = torch.rand((b, 1, hrs, hrs), generator=g, dtype=torch.float64) * 2 - 1
    m = (torch.rand((b, 1, hrs, hrs), generator=g) < 0.7).double()
    lr = torch.cat([hr, e, m], 1)[:, :, ::sf, ::sf].contiguous()
    return {k: v.to(dtype) for k, v in dict(lr=lr, hr=hr, elevation=e, mask=m).items()}


def rcan_params(ng, nb, sf, dtype=torch.float64):
    """The deterministic RCAN weights of the golden records (climsr_amd.core.init keyed by state_dict name)."""
    import numpy as np

    from climsr_amd.core.init import init_state, spec_from_shapes
    from climsr_amd.models.rcan import RCAN

    shapes = {k: tuple(v.shape) for k, v in RCAN(n_resgroups=ng, n_resblocks=nb, scaling_factor=sf).state_dict().items()}
    return {k: torch.from_numpy(np.asarray(v)).to(dtype) for k, v in init_state(spec_from_shapes(shapes)).items()}
