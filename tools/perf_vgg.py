"""Generic-conv shapes for counter passes (rocprofv3 --pmc): VGG19 256ch @64^2 and 512ch @32^2 (B 64), RDB conv5
(128 -> 64 @64^2, B 32), each launched 6 times eagerly.  GPU box only."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd.ops import ACT_LRELU, ConvPlan  # noqa: E402

dev = "cuda"


def plan(cin, cout):
    p = ConvPlan(cin, cout, 3, 1, None, f"{cin}->{cout}")
    p.bind((torch.randn(cout, cin, 3, 3, device=dev) * 0.05).contiguous(), torch.zeros(cout, device=dev))
    p.pack()
    return p


for cin, cout, hw, n in ((256, 256, 64, 64), (512, 512, 32, 64), (128, 64, 64, 32)):
    p = plan(cin, cout)
    x = torch.randn(n, hw, hw, cin, device=dev).to(torch.bfloat16)
    y = torch.empty(n, hw, hw, cout, device=dev, dtype=torch.bfloat16)
    for _ in range(6):
        if cout == 64:
            p.fwd(x, cin, 0, hw, hw, y, cout, 0, n, res1=x, res1_cs=cin, alpha1=0.2)
        else:
            p.fwd(x, cin, 0, hw, hw, y, cout, 0, n, act=ACT_LRELU)
    torch.cuda.synchronize()
print("ok")
