"""Eager launches of the RDB convs (fwd conv1-5 and the pull convs) for rocprofv3 counter passes:
    rocprofv3 --pmc <counters> -d gpurun_out/pmc -- python tools/prof_rdb_convs.py
(graph replays are not instrumented per dispatch, so this stays eager)."""
import sys

sys.path.insert(0, "/root/repo")
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd.ops import ACT_LRELU, ACT_LRELU_BWD, ConvPlan  # noqa: E402

dev, n, dc = "cuda", 32, 128
dense = torch.randn(n, 64, 64, dc, device=dev).to(torch.bfloat16)
dz = torch.randn(n, 64, 64, dc, device=dev).to(torch.bfloat16)
plans = []
for k in range(1, 5):
    cin = 64 + 16 * (k - 1)
    p = ConvPlan(cin, 16, 3, 1, None, f"conv{k}")
    p.bind((torch.randn(16, cin, 3, 3, device=dev) * 0.05).contiguous(), torch.zeros(16, device=dev), need_t=False)
    p.pack()
    plans.append((k, cin, p))
for _ in range(3):
    for k, cin, p in plans:
        p.fwd(dense, dc, 0, 64, 64, dense, dc, cin, n, act=ACT_LRELU)
        # pull-conv shape: dZ suffix in, lrelu backward epilogue (mask from the dense buffer)
        p.fwd(dz, dc, 0, 64, 64, dz, dc, cin, n, act=ACT_LRELU_BWD, use_bias=False, res1=dense, res1_cs=dc, res1_co=cin)
torch.cuda.synchronize()
print("ok")
