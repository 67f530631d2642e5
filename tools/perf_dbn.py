"""Time the RFB discriminator's stride-1 convs with the BatchNorm partials epilogue (conv_fwd_dma_kernel EP 9,
rfb_esrgan.py:32-50) at the GAN step's shapes (B=32, 128^2 / 64^2 / 32^2) under one libclimsr_hip.so
(CLIMSR_HIP_LIB selects an A/B build), hipGraph replay.  One JSON line.
    CLIMSR_HIP_LIB=... python tools/perf_dbn.py <label>"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import _lib  # noqa: E402
from climsr_amd.ops import ConvPlan  # noqa: E402
from tools.perf_conv_timing import timeit  # noqa: E402

dev, n = "cuda", 32
res = {"label": sys.argv[1] if len(sys.argv) > 1 else "", "lib": _lib.LIB_PATH}
g = torch.Generator(device=dev).manual_seed(2)
for cin, cout, h in [(64, 128, 128), (128, 256, 64), (256, 512, 32)]:
    p = ConvPlan(cin, cout, 3, 1, 1, f"d{cin}_{cout}")
    p.bind((torch.randn(cout, cin, 3, 3, device=dev, generator=g) * 0.05).contiguous(), None, need_t=False)
    p.pack()
    x = torch.randn((n, h, h, cin), device=dev, generator=g).to(torch.bfloat16)
    z = torch.empty((n, h, h, cout), dtype=torch.bfloat16, device=dev)
    nparts = p.bn_parts(cin, h, h, n, cout)
    part = torch.empty((nparts * 2 * cout,), dtype=torch.float64, device=dev)
    res[f"bnconv_{cin}_{cout}_{h}_us"] = round(timeit(lambda: p.fwd(x, cin, 0, h, h, z, cout, 0, n, use_bias=False, bn_part=part), 20), 2)
print(json.dumps(res), flush=True)
