"""Time conv_wr_kernel (the register-resident 64 -> 64 3x3 conv, csrc/conv_wr.hip) at its product shapes under one
libclimsr_hip.so (CLIMSR_HIP_LIB selects an A/B build): HRconv / upconv (nearest x2 on load, LeakyReLU, B=32 128^2 ->
256^2, esrgan.py:94-99), a 256^2 ReLU conv (VGG conv1_2 at B=32), and the RCAN RCAB pair on config 5's 360 x 720 LR
grid (rcan.py:50-69: ReLU conv, then the bf16 conv with per-tile channel sums).  One JSON line.
    CLIMSR_HIP_LIB=... python tools/perf_wr.py <label>"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import _lib  # noqa: E402
from climsr_amd.ops import ACT_LRELU, ACT_NONE, ACT_RELU, ConvPlan  # noqa: E402
from tools.perf_conv_timing import timeit  # noqa: E402

dev = "cuda"
res = {"label": sys.argv[1] if len(sys.argv) > 1 else "", "lib": _lib.LIB_PATH}
names = []
p = ConvPlan(64, 64, 3, 1, None, "wr")
p.bind((torch.randn(64, 64, 3, 3, device=dev) * 0.05).contiguous(), torch.randn(64, device=dev) * 0.1)
p.pack()
x = torch.randn(32, 128, 128, 64, device=dev).to(torch.bfloat16)
y = torch.empty(32, 256, 256, 64, device=dev, dtype=torch.bfloat16)
res["hr_up2_lrelu_us"] = round(timeit(lambda: p.fwd(x, 64, 0, 128, 128, y, 64, 0, 32, up=2, act=ACT_LRELU), 10), 2)
x2 = torch.randn(32, 256, 256, 64, device=dev).to(torch.bfloat16)
res["hr_relu_us"] = round(timeit(lambda: p.fwd(x2, 64, 0, 256, 256, y, 64, 0, 32, act=ACT_RELU), 10), 2)
h, w = 360, 720
xr = torch.randn(1, h, w, 64, device=dev).to(torch.bfloat16)
u1 = torch.empty(1, h, w, 64, device=dev, dtype=torch.bfloat16)
u = torch.empty(1, h, w, 64, device=dev, dtype=torch.bfloat16)
rows, _tpi = p.ch_parts(64, h, w, 1, 64)
cp = torch.empty((max(rows, 1), 64), dtype=torch.float32, device=dev)
res["rcan_relu_us"] = round(timeit(lambda: p.fwd(xr, 64, 0, h, w, u1, 64, 0, 1, act=ACT_RELU), 50), 2)
res["rcan_sums_us"] = round(timeit(lambda: p.fwd(u1, 64, 0, h, w, u, 64, 0, 1, act=ACT_NONE, ch_part=cp if rows else None), 50), 2)
print(json.dumps(res), flush=True)
