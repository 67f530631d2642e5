"""Time the 64-block LDS-DMA weight gradient (conv_wgrad64_glds_kernel + its split-K reduce) at the GAN step's shapes
(B=32) under one libclimsr_hip.so (CLIMSR_HIP_LIB selects an A/B build), hipGraph replay: the grouped RDB GEMM
(128 x 1152, 64^2), the trunk conv (64 -> 64, 64^2), upconv1 (64 -> 64, nearest x2 on load, 128^2) and the RFB
discriminator's stride-1 convs.  One JSON line (us per launch, kernel + reduce).
    CLIMSR_HIP_LIB=... python tools/perf_wgrad64.py <label>"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import _lib, ops  # noqa: E402
from climsr_amd.ops import ConvPlan, Workspace  # noqa: E402
from tools.perf_conv_timing import timeit  # noqa: E402

dev, n = "cuda", 32
res = {"label": sys.argv[1] if len(sys.argv) > 1 else "", "lib": _lib.LIB_PATH}
g = torch.Generator(device=dev).manual_seed(1)


def plan(cin, cout, name):
    p = ConvPlan(cin, cout, 3, 1, 1, name)
    p.bind((torch.randn(cout, cin, 3, 3, device=dev, generator=g) * 0.05).contiguous(), torch.zeros(cout, device=dev), need_t=False)
    p.gw, p.gb = torch.zeros_like(p.weight), torch.zeros_like(p.bias)
    return p


# the grouped RDB GEMM (ops.GroupedWgrad): conv1-5 of one dense block as one 128 x 1152 weight gradient
plans = [plan(64 + 16 * k, 16 if k < 4 else 64, f"rdb.conv{k + 1}") for k in range(5)]
gw = ops.GroupedWgrad(plans, 128, "rdb")
dense = torch.randn((n, 64, 64, 128), device=dev, generator=g).to(torch.bfloat16)
dz = torch.randn((n, 64, 64, 128), device=dev, generator=g).to(torch.bfloat16)
ws = Workspace()
res["rdb_grouped_us"] = round(timeit(lambda: gw.run(dense, 128, 0, 64, 64, dz, 128, n, ws, accumulate=False), 20), 2)
d = _lib.ConvDesc(n, 64, 64, 128, 128, 0, 1, 3, 1, 1, 64, 64, 128, 0, 0, 8)
res["rdb_splits"] = int(_lib.load().climsr_conv2d_wgrad_splits(ctypes.byref(d)))
for cin, cout, h, up, name in [(64, 64, 64, 1, "trunk"), (64, 64, 128, 2, "upconv1"), (64, 128, 128, 1, "d64_128"),
                               (128, 256, 64, 1, "d128_256"), (256, 512, 32, 1, "d256_512"), (512, 512, 16, 1, "d512_512")]:
    p = plan(cin, cout, name)
    hin = h // up
    x = torch.randn((n, hin, hin, cin), device=dev, generator=g).to(torch.bfloat16)
    z = torch.randn((n, h, h, cout), device=dev, generator=g).to(torch.bfloat16)
    wsp = Workspace()
    res[f"{name}_us"] = round(timeit(lambda: p.wgrad(x, cin, 0, hin, hin, z, cout, n, wsp, accumulate=False, up=up), 20), 2)
print(json.dumps(res), flush=True)
