"""VGG19 conv1_1 of the perceptual loss at the GAN step's shape (64 images: sr and hr of B=32, 256^2), same process, same
library, hipGraph replay: the 1-channel form (climsr_vgg_conv1_1 straight from the two fp32 batches) against the
3-channel route it replaced (two pack_planes8 passes into 8-channel NHWC + the generic conv on 4-channel taps), and the
whole perceptual forward.  One JSON line.
    python tools/perf_vgg_c11.py <label>"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import _lib, ops  # noqa: E402
from climsr_amd.losses.perceptual import PerceptualLoss  # noqa: E402
from climsr_amd.ops import ACT_RELU, ConvPlan  # noqa: E402
from tools.perf_conv_timing import timeit  # noqa: E402

dev, n, h, w = "cuda", 32, 256, 256
res = {"label": sys.argv[1] if len(sys.argv) > 1 else "", "lib": _lib.LIB_PATH}
g = torch.Generator(device=dev).manual_seed(3)
a = torch.rand((n, 1, h, w), device=dev, generator=g)
b = torch.rand((n, 1, h, w), device=dev, generator=g)
pl = PerceptualLoss().to(dev)
pl(a, b)
c11 = pl.loss_network[0]
wt, bias = c11.weight.detach().contiguous().float(), c11.bias.detach().contiguous().float()
y1 = torch.empty((2 * n, h, w, 64), dtype=torch.bfloat16, device=dev)
p = ConvPlan(3, 64, 3, 1, 1, "conv1_1")
p.bind(wt, bias, need_t=False)
p.pack()
x3 = torch.empty((2 * n, h, w, 8), dtype=torch.bfloat16, device=dev)


def three_channel():
    ops.pack_planes8([(a, 0)] * 3, n, h, w, x3[:n])
    ops.pack_planes8([(b, 0)] * 3, n, h, w, x3[n:])
    p.fwd(x3, 8, 0, h, w, y1, 64, 0, 2 * n, act=ACT_RELU)


for _ in range(2):
    res.setdefault("c11_one_channel_us", []).append(round(timeit(lambda: ops.vgg_conv1_1(a, b, n, h, w, wt, bias, y1), 10), 2))
    res.setdefault("c11_three_channel_us", []).append(round(timeit(three_channel, 10), 2))
    res.setdefault("perceptual_fwd_us", []).append(round(timeit(lambda: pl(a, b), 5), 2))
print(json.dumps(res), flush=True)
