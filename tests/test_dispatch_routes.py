"""Which kernel every hot conv of the product takes, pinned on the CPU.

The dispatcher's dry-run entry points (climsr_conv2d_fwd_kernel / climsr_conv2d_wgrad_kernel: the same C++ dispatch
code, which records the kernel it would launch instead of launching) are asked through the product's own call sites:
ConvPlan.fwd / wgrad and GroupedWgrad.run with the arguments models/esrgan.py, losses/perceptual.py and
models/rfb_esrgan.py pass at the GAN-step shapes (config 3: B=32, 64^2 -> 256^2; VGG on 64 images).  The launch
observer (ops.PROFILER) records the names and runs nothing, so no GPU is needed and the tensors are placeholders.

A dispatch change shows up here as a diff of routes, next to the per-kernel timings it would move
(profiles/r04_v1_gan_kernel_stats.csv names every kernel below except the stride-2 LDS-DMA forward, which replaced
conv_fwd_s2_kernel after that profile: profiles/r04l_s2_dma_ab.jsonl).  The GPU suite checks these same routes
numerically.  Shapes follow /root/reference: climsr/models/esrgan.py:17-102, climsr/losses/perceptual.py:16-36 and
climsr/models/rfb_esrgan.py:28-57.
"""
import pytest
import torch

from climsr_amd import _lib, ops
from climsr_amd.ops import ACT_LRELU, ACT_RELU, OUT_F32, ConvPlan, GroupedWgrad, Workspace

N, H, DC, NF, GC = 32, 64, 128, 64, 16


@pytest.fixture
def routes(monkeypatch):
    try:
        _lib.load()
    except OSError as e:  # the built library is a prerequisite of the whole CPU suite (test_abi)
        pytest.skip(f"libclimsr_hip.so not loadable: {e}")
    names = []
    monkeypatch.setattr(ops, "PROFILER", lambda name, flops, fn, tag="", nbytes=0: names.append(name))
    monkeypatch.setattr(_lib, "stream_ptr", lambda: 0)  # (read before the recorded launches; no device here)
    return names


def bf():
    return torch.empty(8, dtype=torch.bfloat16)


def plan(cin, cout, ks=3, stride=1, bias=True):
    p = ConvPlan(cin, cout, ks, stride, None, "route")
    p.weight = torch.zeros(1)
    p.bias = torch.zeros(cout) if bias else None
    return p


def last(names):
    assert names, "no launch recorded"
    return names[-1]


def test_generator_forward_routes(routes):
    """conv5 (x5 * 0.2 + x, and the RRDB's out * 0.2 + x on its third RDB), trunk_conv (+ fea), upconv1/2 (nearest x2
    on load + LeakyReLU), HRconv, conv_last (64 -> 1) at B=32, 64^2 LR."""
    p5 = plan(DC, NF)
    p5.fwd(bf(), DC, 0, H, H, bf(), DC, 0, N, res1=bf(), alpha1=0.2, res1_cs=DC, res1_co=0)
    assert last(routes) == "conv_fwd_kernel<4, 4, false, 4, 6, 9, 1, 1>"
    p5.fwd(bf(), DC, 0, H, H, bf(), DC, 0, N, res1=bf(), alpha1=0.2, res1_cs=DC, res1_co=0, res2=bf(), alpha2=0.2, res2_cs=DC,
           res2_co=0)
    assert last(routes) == "conv_fwd_kernel<4, 4, false, 4, 6, 9, 1, 1>"
    pt = plan(NF, NF)
    pt.fwd(bf(), DC, 0, H, H, bf(), NF, 0, N, res1=bf(), alpha1=1.0, res1_cs=NF, res1_co=0)
    assert last(routes) == "conv_wr_kernel<1, 0>"
    pu = plan(NF, NF)
    for s in (1, 2):  # upconv1 (64 -> 128), upconv2 (128 -> 256)
        pu.fwd(bf(), NF, 0, s * H, s * H, bf(), NF, 0, N, up=2, act=ACT_LRELU)
        assert last(routes) == "conv_wr_kernel<0, 1>"
    pu.fwd(bf(), NF, 0, 4 * H, 4 * H, bf(), NF, 0, N, act=ACT_LRELU)
    assert last(routes) == "conv_wr_kernel<0, 1>"
    pl = plan(NF, 1)
    pl.fwd(bf(), NF, 0, 4 * H, 4 * H, bf(), 8, 0, N)
    assert last(routes) == "conv_co1m_kernel<3, 2>"


def test_conv_wr_bf16_output_needs_8_channel_alignment(routes):
    """conv_wr's bf16 epilogues store 16 B (8 channels) per lane: an output at channel offset 4 (mod 8) must take
    another kernel, an 8-aligned one conv_wr."""
    pu = plan(NF, NF)
    pu.fwd(bf(), NF, 0, 2 * H, 2 * H, bf(), NF + 8, 8, N, act=ACT_LRELU)
    assert last(routes) == "conv_wr_kernel<0, 1>"
    pu.fwd(bf(), NF, 0, 2 * H, 2 * H, bf(), NF + 8, 4, N, act=ACT_LRELU)
    assert not last(routes).startswith("conv_wr_kernel"), last(routes)


@pytest.mark.parametrize("cin,cout,hw,want", [
    (3, 64, 256, "conv_pw_kernel<8, 2, 4, false, 2, 3, 2>"),     # conv1_1: 4-channel taps
    (64, 64, 256, "conv_wr_kernel<0, 2>"),                         # conv1_2: weights in registers
    (64, 128, 128, "conv_fwd_dma_kernel<3, false>"),            # conv2_1 .. conv4_4: the roofline kernel
    (128, 128, 128, "conv_fwd_dma_kernel<3, false>"),
    (128, 256, 64, "conv_fwd_dma_kernel<3, false>"),
    (256, 256, 64, "conv_fwd_dma_kernel<3, false>"),
    (256, 512, 32, "conv_fwd_dma_kernel<3, false>"),
    (512, 512, 32, "conv_fwd_dma_kernel<3, false>"),
    (512, 512, 16, "conv_fwd_kernel<4, 4, false, 4, 6, 9, 3, 1>"),  # conv5_x at 16^2: 32-row tiles would be half empty
])
def test_vgg19_routes(routes, cin, cout, hw, want):
    """The perceptual loss's VGG19 convs (bias + ReLU, 64 images: hr and sr of B=32)."""
    p = plan(cin, cout)
    p.fwd(bf(), p.cin, 0, hw, hw, bf(), cout, 0, 2 * N, act=ACT_RELU)
    assert last(routes) == want


@pytest.mark.parametrize("cin,cout,hw,want", [
    (64, 64, 256, "conv_wr_kernel<5, 2>"),              # conv1_2 + pool1
    (128, 128, 128, "conv_fwd_dma_kernel<11, false>"),  # conv2_2 + pool2
    (256, 256, 64, "conv_fwd_dma_kernel<11, false>"),   # conv3_4 + pool3
    (512, 512, 32, "conv_fwd_dma_kernel<11, false>"),   # conv4_4 + pool4
])
def test_vgg19_pooled_routes(routes, cin, cout, hw, want):
    """The VGG19 convs followed by ReLU + 2x2 max pool take the fused pooled epilogue (losses/perceptual.py)."""
    p = plan(cin, cout)
    assert p.pool_ok(p.cin, hw, hw, 2 * N, cout)
    p.fwd(bf(), p.cin, 0, hw, hw, bf(), cout, 0, 2 * N, act=ACT_RELU, pool2=True)
    assert last(routes) == want
    assert not p.pool_ok(p.cin, hw + 1, hw + 1, 2 * N, cout)  # odd sizes: no fused pool


@pytest.mark.parametrize("stride,cin,cout,hw,want", [
    (2, 64, 64, 256, "conv_fwd_s2_dma_kernel<true>"),
    (2, 128, 128, 128, "conv_fwd_s2_dma_kernel<true>"),
    (2, 256, 256, 64, "conv_fwd_s2_dma_kernel<true>"),
    (2, 512, 512, 32, "conv_fwd_s2_dma_kernel<true>"),
    (1, 64, 128, 128, "conv_fwd_dma_kernel<9, false>"),
    (1, 128, 256, 64, "conv_fwd_dma_kernel<9, false>"),
    (1, 256, 512, 32, "conv_fwd_dma_kernel<9, false>"),
])
def test_discriminator_bn_conv_routes(routes, stride, cin, cout, hw, want):
    """The RFB discriminator's BatchNorm'd convs: plain bf16 out with the BatchNorm partials from the epilogue."""
    p = plan(cin, cout, 3, stride, bias=False)
    assert p.bn_parts(cin, hw, hw, N, cout) > 0, "BatchNorm partials must come from the conv epilogue"
    p.fwd(bf(), cin, 0, hw, hw, bf(), cout, 0, N, use_bias=False, bn_part=torch.empty(1, dtype=torch.float64))
    assert last(routes) == want


def test_rdb_pullx_route(routes):
    """pull-x (the RDB-input gradient as one 128 -> 64 conv over [dZ1 .. dZ5]: fp32 out, fp32 skip gradients, the
    previous RDB's bf16 dZ5 as aux) takes the row-streaming kernel."""
    px = plan(DC, NF, bias=False)
    f32 = torch.empty(8, dtype=torch.float32)
    px.fwd(bf(), DC, 0, H, H, f32, NF, 0, N, use_bias=False, out_mode=OUT_F32, res1=f32, res1_cs=NF, res1_co=0, beta1=0.2,
           res2=f32, res2_cs=NF, res2_co=0, aux=bf(), aux_cs=DC, aux_co=4 * GC, aux_scale=0.04)
    assert last(routes) == "conv_fwd_kernel<4, 4, true, 4, 6, 9, 2, 1>"


def _wgrad_name(routes):
    kernels = [r for r in routes if "kernel" in r]
    assert kernels, routes
    return kernels[-1]


def test_weight_gradient_routes(routes):
    """The RDB's grouped 128 x 1152 weight-gradient GEMM (conv1..conv5 of one RDB in one launch), the HR 64 -> 64
    convs (HRconv at 256^2), upconv with the nearest x2 on load, and a discriminator stride-2 conv."""
    plans = [plan(NF + GC * (k - 1), GC if k < 5 else NF) for k in range(1, 6)]
    GroupedWgrad(plans, DC, "rdb").run(bf(), DC, 0, H, H, bf(), DC, N, Workspace(), accumulate=False)
    assert _wgrad_name(routes) == "conv_wgrad64_glds_kernel"
    routes.clear()
    p = plan(NF, NF)
    p.wgrad(bf(), NF, 0, 4 * H, 4 * H, bf(), NF, N, Workspace(), accumulate=False)
    assert _wgrad_name(routes) == "conv_wgrad64_kernel<2, 1>"
    routes.clear()
    p.wgrad(bf(), NF, 0, 2 * H, 2 * H, bf(), NF, N, Workspace(), accumulate=False, up=2)
    assert _wgrad_name(routes) == "conv_wgrad64_kernel<2, 1>"
    routes.clear()
    p2 = plan(128, 128, 3, 2, bias=False)
    p2.wgrad(bf(), 128, 0, 128, 128, bf(), 128, N, Workspace(), accumulate=False)
    assert _wgrad_name(routes) == "conv_wgrad64_glds_s2_kernel"
