"""Where the time of one rdb5_kernel launch goes (GPU box only; the stamp build tools/diag_build of rdb_conv5.hip with
-DCLIMSR_R5_STAMP, passed as CLIMSR_HIP_LIB): conv5 (mode 1) at the GAN step's shape (B=32, 64^2, 128 -> 64), waves 0 and
4 of every block stamp (s_memrealtime 100 MHz, s_memtime) at kernel entry, after the prologue, and per step before the
DMA wait, after the barrier and after the MFMA groups (with the epilogue / DMA issued between them).  Prints one JSON line of medians over blocks (us)."""
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import _lib  # noqa: E402
from climsr_amd.ops import ConvPlan  # noqa: E402

NST = 48
dev, n, dc = "cuda", 32, 128
p = ConvPlan(128, 64, 3, 1, None, "conv5")
p.bind((torch.randn(64, 128, 3, 3, device=dev) * 0.05).contiguous(), torch.zeros(64, device=dev))
p.pack()
dense = torch.randn(n, 64, 64, dc, device=dev).to(torch.bfloat16)
out = torch.empty(n, 64, 64, dc, device=dev, dtype=torch.bfloat16)
res = {"label": sys.argv[1] if len(sys.argv) > 1 else "", "lib": _lib.LIB_PATH}
lib = _lib.load()
fn = lib.climsr_diag_r5_stamps
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_void_p, ctypes.c_long]
for rep in range(4):
    p.fwd(dense, dc, 0, 64, 64, out, dc, 0, n, res1=dense, res1_cs=dc, alpha1=0.2)
    torch.cuda.synchronize()
nblk = 256
buf = np.zeros((nblk, 2, NST, 2), dtype=np.uint64)
assert fn(buf.ctypes.data, buf.nbytes) == 0
rt = buf[..., 0].astype(np.int64)
ck = buf[..., 1].astype(np.int64)
t0 = rt[:, 0, 0].min()
us = (rt - t0) / 100.0  # 100 MHz -> us
end = us[:, :, NST - 1]
res["kernel_span_us"] = float(end.max())
res["entry_spread_us"] = [float(np.percentile(us[:, 0, 0], q)) for q in (0, 50, 100)]
res["end_spread_us"] = [float(np.percentile(end[:, 0], q)) for q in (0, 50, 100)]
res["prologue_us"] = float(np.median(us[:, 0, 1] - us[:, 0, 0]))
steps = []
s = 0
while 4 + 3 * s < NST - 1 and (rt[:, 0, 4 + 3 * s] > 0).all():
    a, b, c = us[:, :, 2 + 3 * s], us[:, :, 3 + 3 * s], us[:, :, 4 + 3 * s]
    nxt = us[:, :, 2 + 3 * (s + 1)] if (rt[:, 0, 2 + 3 * (s + 1)] > 0).all() and 2 + 3 * (s + 1) < NST - 1 else us[:, :, NST - 1]
    steps.append({"wait_barrier": [round(float(np.median(b[:, w] - a[:, w])), 3) for w in (0, 1)],
                  "groups": [round(float(np.median(c[:, w] - b[:, w])), 3) for w in (0, 1)],
                  "handoff": [round(float(np.median(nxt[:, w] - c[:, w])), 3) for w in (0, 1)]})
    s += 1
res["steps"] = steps
dck = (ck[:, 0, NST - 1] - ck[:, 0, 0]).astype(np.float64)
drt = (rt[:, 0, NST - 1] - rt[:, 0, 0]).astype(np.float64) / 100e6
res["memtime_hz"] = float(np.median(dck / drt))
print(json.dumps(res), flush=True)
