"""Time conv_last (64 -> 1, 3x3, esrgan.py:99-100) forward at the GAN step's shape (B=32, 256^2, out channel stride 8:
the SRCNN tail's 4-channel cat buffer) under one libclimsr_hip.so (CLIMSR_HIP_LIB selects an A/B build).  One JSON line.
    CLIMSR_HIP_LIB=... python tools/perf_co1m.py <label>"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import _lib  # noqa: E402
from climsr_amd.ops import ConvPlan  # noqa: E402
from tools.perf_conv_timing import timeit  # noqa: E402

dev, n, hw = "cuda", 32, 256
res = {"label": sys.argv[1] if len(sys.argv) > 1 else "", "lib": _lib.LIB_PATH}
p = ConvPlan(64, 1, 3, 1, None, "conv_last")
p.bind((torch.randn(1, 64, 3, 3, device=dev) * 0.05).contiguous(), torch.zeros(1, device=dev))
p.pack()
x = torch.randn(n, hw, hw, 64, device=dev).to(torch.bfloat16)
y = torch.zeros(n, hw, hw, 8, device=dev, dtype=torch.bfloat16)
res["co1m_fwd_us"] = round(timeit(lambda: p.fwd(x, 64, 0, hw, hw, y, 8, 0, n), 20), 2)
print(json.dumps(res), flush=True)
