"""The VGG19 block-end convs with the fused ReLU + 2x2 max pool (conv1_2 on conv_wr, conv2_2 / conv3_4 / conv4_4 on the
LDS-DMA conv) at the perceptual loss's shapes (64 images, 256^2 input), under one libclimsr_hip.so (CLIMSR_HIP_LIB
selects an A/B build).  One JSON line.   python tools/perf_vgg_pool.py <label>"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import _lib  # noqa: E402
from climsr_amd.ops import ACT_RELU, ConvPlan  # noqa: E402
from tools.perf_conv_timing import timeit  # noqa: E402

dev, n = "cuda", 64
res = {"label": sys.argv[1] if len(sys.argv) > 1 else "", "lib": _lib.LIB_PATH}
for c, hw in ((64, 256), (128, 128), (256, 64), (512, 32)):
    p = ConvPlan(c, c, 3, 1, None, f"vgg{c}")
    p.bind((torch.randn(c, c, 3, 3, device=dev) * 0.05).contiguous(), torch.zeros(c, device=dev))
    p.pack()
    x = torch.randn(n, hw, hw, c, device=dev).to(torch.bfloat16)
    y = torch.empty(n, hw // 2, hw // 2, c, device=dev, dtype=torch.bfloat16)
    res[f"pool_{c}_{hw}_us"] = round(timeit(lambda: p.fwd(x, c, 0, hw, hw, y, c, 0, n, act=ACT_RELU, pool2=True), 10), 2)
print(json.dumps(res), flush=True)
