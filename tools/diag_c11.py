"""Diagnostic (round 6): VGG conv1_1 via the 1-channel kernel vs the 3-channel route on the perceptual test's inputs;
signed / absolute differences of the conv1_1 outputs and both perceptual losses.  python tools/diag_c11.py"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import ops  # noqa: E402
from climsr_amd.losses.perceptual import PerceptualLoss  # noqa: E402
from climsr_amd.ops import ACT_RELU, ConvPlan  # noqa: E402

dev = "cuda"
pl = PerceptualLoss().to(dev)
g = torch.Generator().manual_seed(0)
hr = torch.rand(2, 1, 64, 64, generator=g)
sr = torch.rand(2, 1, 64, 64, generator=g)
a, b = sr.to(dev).contiguous(), hr.to(dev).contiguous()
new = float(pl(a, b))
n, h, w = 2, 64, 64
c11 = pl.loss_network[0]
wt, bias = c11.weight.detach().contiguous().float(), c11.bias.detach().contiguous().float()
y_new = torch.empty((2 * n, h, w, 64), dtype=torch.bfloat16, device=dev)
ops.vgg_conv1_1(a, b, n, h, w, wt, bias, y_new)
x3 = torch.empty((2 * n, h, w, 8), dtype=torch.bfloat16, device=dev)
ops.pack_planes8([(a, 0)] * 3, n, h, w, x3[:n])
ops.pack_planes8([(b, 0)] * 3, n, h, w, x3[n:])
p = ConvPlan(3, 64, 3, 1, 1, "c11")
p.bind(wt, bias, need_t=False)
p.pack()
y_old = torch.empty_like(y_new)
p.fwd(x3, 8, 0, h, w, y_old, 64, 0, 2 * n, act=ACT_RELU)
f_old = pl.features(y_old, 2 * n, h, w, start=1, cs=64)
half = f_old.numel() // 2
old = float((f_old.view(-1)[half:].float() - f_old.view(-1)[:half].float()).abs().mean())
x = torch.cat([a, b], 0).to(torch.bfloat16).double()
ref = torch.nn.functional.conv2d(torch.cat([x] * 3, 1), wt.double(), bias.double(), padding=1).relu().permute(0, 2, 3, 1)
d_new, d_old = y_new.double() - ref, y_old.double() - ref
print("loss new", new, "old-route", old)
print("conv1_1 new: mean signed", d_new.mean().item(), "max abs", d_new.abs().max().item(), "mean abs", d_new.abs().mean().item())
print("conv1_1 old: mean signed", d_old.mean().item(), "max abs", d_old.abs().max().item(), "mean abs", d_old.abs().mean().item())
print("x3 ch0 vs bf16(a)", (x3[:n, ..., 0].double() - a.to(torch.bfloat16).double().view(n, h, w)).abs().max().item(),
      "x3 ch3..7 max", x3[..., 3:].abs().max().item())
