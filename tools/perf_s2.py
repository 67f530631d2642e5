"""Time the discriminator's stride-2 forwards (rfb_esrgan.py:30-48 at the GAN step's shapes, B=32, plain bf16 out with
the BatchNorm partials) and their weight gradients (split-K kernel + its reduce) under one libclimsr_hip.so (CLIMSR_HIP_LIB selects an A/B build).  One JSON line.
    CLIMSR_HIP_LIB=... python tools/perf_s2.py <label>"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import _lib  # noqa: E402
from climsr_amd.ops import ConvPlan, Workspace  # noqa: E402
from tools.perf_conv_timing import timeit  # noqa: E402

dev, n = "cuda", 32
res = {"label": sys.argv[1] if len(sys.argv) > 1 else "", "lib": _lib.LIB_PATH}
tot = wtot = 0.0
wsp = Workspace()
for cin, cout, hw in ((64, 64, 256), (128, 128, 128), (256, 256, 64), (512, 512, 32)):
    p = ConvPlan(cin, cout, 3, 2, 1, f"s2 {cin}")
    p.bind((torch.randn(cout, cin, 3, 3, device=dev) * 0.05).contiguous(), None)
    p.pack()
    x = torch.randn(n, hw, hw, cin, device=dev).to(torch.bfloat16)
    oh = hw // 2
    y = torch.empty(n, oh, oh, cout, device=dev, dtype=torch.bfloat16)
    rows = p.bn_parts(cin, hw, hw, n, cout)
    part = torch.empty((max(rows, 1), 2, cout), dtype=torch.float64, device=dev)
    t = timeit(lambda: p.fwd(x, cin, 0, hw, hw, y, cout, 0, n, bn_part=part if rows else None), 10)
    res[f"s2_{cin}_{hw}_us"] = round(t, 2)
    tot += t
    dz = torch.randn(n, oh, oh, cout, device=dev).to(torch.bfloat16)
    p.gw = torch.zeros_like(p.weight)
    t = timeit(lambda: p.wgrad(x, cin, 0, hw, hw, dz, cout, n, wsp, accumulate=False), 10)
    res[f"wg2_{cin}_{hw}_us"] = round(t, 2)
    wtot += t
res["total_us"] = round(tot, 2)
res["wgrad_total_us"] = round(wtot, 2)
print(json.dumps(res), flush=True)
