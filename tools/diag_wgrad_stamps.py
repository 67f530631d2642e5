"""Diagnostic (round 6): per-wave start / end stamps (s_memrealtime, 100 MHz) of conv_wgrad64_glds_kernel
from a timestamping A/B build (CLIMSR_HIP_LIB=ab/lib_wg_stamp.so, which writes them past the split-K slabs), at the
grouped RDB GEMM shape (B=32, 64^2, 128 x 1152).  Prints the launch span, the spread of wave start times and the
wave lifetimes, and the core clock over each wave's life (s_memtime cycles / s_memrealtime time).  Timing only.
    CLIMSR_HIP_LIB=ab/lib_wg_stamp.so python tools/diag_wgrad_stamps.py"""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import _lib  # noqa: E402

dev, n, h = "cuda", 32, 64
lib = _lib.load()
d = _lib.ConvDesc(n, h, h, 128, 128, 0, 1, 3, 1, 1, h, h, 128, 0, 0, 8)
ns = int(lib.climsr_conv2d_wgrad_splits(ctypes.byref(d)))
need = int(lib.climsr_conv2d_wgrad_workspace(ctypes.byref(d), ns))
grid = 4 * ns
part = torch.zeros(need + grid * 8 * 4 + 64, dtype=torch.float32, device=dev)
x = torch.randn((n, h, h, 128), device=dev).to(torch.bfloat16)
dz = torch.randn((n, h, h, 128), device=dev).to(torch.bfloat16)
s = torch.cuda.current_stream().cuda_stream
res = {"splits": ns, "grid": grid, "runs": []}
for rep in range(4):
    _lib.check(lib.climsr_conv2d_wgrad(ctypes.byref(d), x.data_ptr(), dz.data_ptr(), 128, part.data_ptr(), None, ns, s), "wgrad")
    torch.cuda.synchronize()
    st = part[ns * 128 * 1152:ns * 128 * 1152 + grid * 8 * 4].view(torch.int32).view(grid * 8, 4).cpu().to(torch.int64) & 0xFFFFFFFF
    t1 = st[:, 2] | (st[:, 3] << 32)
    t0 = (t1 & ~0xFFFFFFFF) | st[:, 0]  # (the start's high word: the end's; a wrap inside one launch is negligible)
    cyc = st[:, 1].double()  # s_memtime cycles over the wave's life
    base = int(t0.min())
    start = (t0 - base).double() / 100.0  # us (100 MHz)
    end = (t1 - base).double() / 100.0
    life = end - start
    mhz = cyc / life
    q = lambda v, p: round(float(torch.quantile(v, p)), 2)  # noqa: E731
    res["runs"].append({"span_us": round(float(end.max()), 2), "start_us_q": [q(start, p) for p in (0, 0.25, 0.5, 0.75, 1)],
                        "life_us_q": [q(life, p) for p in (0, 0.25, 0.5, 0.75, 1)],
                        "end_us_q": [q(end, p) for p in (0, 0.25, 0.5, 0.75, 1)],
                        "core_mhz_q": [q(mhz, p) for p in (0, 0.5, 1)]})
print(json.dumps(res), flush=True)
