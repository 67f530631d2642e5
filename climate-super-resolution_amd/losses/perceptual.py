"""Perceptual loss (drop-in for ``climsr.losses.perceptual.PerceptualLoss``, perceptual.py:7-36).

VGG19 ``features[:35]`` (conv1_1 .. conv5_4, the last without ReLU) applied to the 1->3 channel
repeat of both images, L1 between the feature maps, all without gradient (F7: the loss adds to
the value only).  Both images run as ONE batch through native implicit-GEMM convs with fused
bias+ReLU epilogues and MaxPool2d(2,2) kernels; the L1 is a deterministic bf16 reduction.
conv1_1 on the repeat is one 1-channel conv with the summed weight (``climsr_vgg_conv1_1``), read
straight from the two fp32 image batches.

Weights: ``vgg19(pretrained=True)`` (perceptual.py:15) downloads ImageNet weights, impossible
offline; the module is built with the reference's parameter names (``loss_network.{i}.weight``)
so a torchvision VGG19 state_dict loads with ``load_state_dict`` when available.  By default it
is initialised with the deterministic He-uniform initializer (climsr_amd.core.init, gain sqrt(6)).
"""
from typing import List

import numpy as np
import torch
import torch.nn as nn

from .. import ops
from ..core.init import init_state, spec_from_shapes
from ..ops import ACT_NONE, ACT_RELU, ConvPlan, OUT_BF16

VGG19_E = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]


def _vgg19_features_35() -> nn.Sequential:
    layers: List[nn.Module] = []
    cin = 3
    for v in VGG19_E:
        if v == "M":
            layers.append(nn.MaxPool2d(kernel_size=2, stride=2))
        else:
            layers += [nn.Conv2d(cin, v, kernel_size=3, padding=1), nn.ReLU(inplace=True)]
            cin = v
    return nn.Sequential(*layers[:35])


class PerceptualLoss(nn.Module):
    """Assumes input images of shape Nx1xHxW (perceptual.py:8-10)."""

    def __init__(self, deterministic_init: bool = True):
        super().__init__()
        loss_network = _vgg19_features_35().eval()
        if deterministic_init:
            shapes = {k: tuple(v.shape) for k, v in loss_network.state_dict().items()}
            st = init_state(spec_from_shapes({"loss_network." + k: s for k, s in shapes.items()}), gain=float(np.sqrt(6.0)))
            loss_network.load_state_dict({k[len("loss_network."):]: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
        for param in loss_network.parameters():
            param.requires_grad = False
        self.loss_network = loss_network
        self._plans = None
        self._dev = None

    def _build(self, dev):
        plans = []
        mods = list(self.loss_network)
        for i, m in enumerate(mods):
            if isinstance(m, nn.Conv2d):
                relu = i + 1 < len(mods) and isinstance(mods[i + 1], nn.ReLU)
                pool = i + 2 < len(mods) and isinstance(mods[i + 2], nn.MaxPool2d)
                p = ConvPlan(m.in_channels, m.out_channels, 3, 1, 1, f"loss_network.{i}")
                w = m.weight.detach().contiguous().float()
                b = m.bias.detach().contiguous().float()
                p.bind(w, b, need_t=False)
                p.pack()
                plans.append((p, relu, pool))
        self._plans = plans
        self._dev = dev
        c11 = mods[0]
        self._c11_w = c11.weight.detach().contiguous().float()
        self._c11_b = c11.bias.detach().contiguous().float()
        self._version = sum(int(p.weight._version) for p, _r, _q in plans)

    def features(self, x3: torch.Tensor, n: int, h: int, w: int, start: int = 0, cs: int = 8) -> torch.Tensor:
        """x3: NHWC bf16 [n,h,w,cs]: the image in channels 0..2 (start 0), or the output of conv plan start - 1.
        Returns conv5_4 features (bf16)."""
        a = x3
        for p, relu, pool in self._plans[start:]:
            act = ACT_RELU if relu else ACT_NONE
            if pool and p.pool_ok(cs, h, w, n, p.cout, act):  # conv + ReLU + 2x2 max pool in one kernel
                h, w = h // 2, w // 2
                y = torch.empty((n, h, w, p.cout), dtype=torch.bfloat16, device=x3.device)
                p.fwd(a, cs, 0, 2 * h, 2 * w, y, p.cout, 0, n, act=act, out_mode=OUT_BF16, pool2=True)
                a, cs = y, p.cout
                continue
            y = torch.empty((n, h, w, p.cout), dtype=torch.bfloat16, device=x3.device)
            p.fwd(a, cs, 0, h, w, y, p.cout, 0, n, act=act, out_mode=OUT_BF16)
            a, cs = y, p.cout
            if pool:
                h2, w2 = h // 2, w // 2
                yp = torch.empty((n, h2, w2, cs), dtype=torch.bfloat16, device=x3.device)
                ops.maxpool2(a, n, h, w, cs, yp)
                a, h, w = yp, h2, w2
        return a

    @torch.no_grad()
    def forward(self, fake_high_resolution, high_resolution):
        a, b = fake_high_resolution, high_resolution
        if not a.is_cuda:
            raise RuntimeError("climsr_amd.PerceptualLoss runs on the GPU only (no CPU fallback)")
        if self._plans is None or self._dev != a.device:
            self.loss_network.to(a.device)
            self._build(a.device)
        n, _c, h, w = a.shape
        a32, b32 = a.contiguous().float(), b.contiguous().float()
        # conv1_1 + ReLU on torch.cat([x, x, x], dim=1) (perceptual.py:26-31) = one 1-channel conv with the summed
        # weight, straight from the fp32 images (both batches in one launch)
        c11 = self.loss_network[0]
        y1 = torch.empty((2 * n, h, w, 64), dtype=torch.bfloat16, device=a.device)
        ops.vgg_conv1_1(a32, b32, n, h, w, self._c11_w, self._c11_b, y1)
        f = self.features(y1, 2 * n, h, w, start=1, cs=c11.out_channels)
        half = f.numel() // 2
        ws = torch.empty(512, dtype=torch.float64, device=a.device)
        out = torch.empty((), dtype=torch.float32, device=a.device)
        ops.l1_bf16(f.view(-1)[half:], f.view(-1)[:half], half, ws, out)
        return out
