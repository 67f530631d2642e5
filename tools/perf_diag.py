"""Time the hot conv shapes under one libclimsr_hip.so (CLIMSR_HIP_LIB selects a diagnostic variant): RDB chain
forward / pull, conv5 (128 -> 64 @64^2 with the x5*0.2+x residual), pull-x (128 -> 64, fp32 out + fp32 residual), and
two VGG layers (B 64).  One JSON line.   CLIMSR_HIP_LIB=... python tools/perf_diag.py <label>"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import _lib  # noqa: E402
from climsr_amd.ops import ACT_LRELU, OUT_F32, BatchedPacker, ConvPlan, RdbChain, Workspace  # noqa: E402
from tools.perf_conv_timing import timeit  # noqa: E402

dev, n, dc = "cuda", 32, 128
res = {"label": sys.argv[1] if len(sys.argv) > 1 else "", "lib": _lib.LIB_PATH}


def plan(cin, cout, ks=3):
    p = ConvPlan(cin, cout, ks, 1, None, f"{cin}->{cout}")
    p.bind((torch.randn(cout, cin, ks, ks, device=dev) * 0.05).contiguous(), torch.zeros(cout, device=dev))
    p.pack()
    return p


dense = torch.randn(n, 64, 64, dc, device=dev).to(torch.bfloat16)
cplans = [plan(64 + 16 * (k - 1), 16 if k < 5 else 64) for k in range(1, 6)]
chain = RdbChain(cplans, "diag")
BatchedPacker(cplans, torch.device(dev), chain.pack_descs()).run()
pd = chain.pull_descs()
arr = (_lib.PullPackDesc * len(pd))(*pd)
tab = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
_lib.check(_lib.load().climsr_pack_pull_weights_batched(tab.data_ptr(), len(pd), 16 * 9 * 128, _lib.stream_ptr()), "pack")
res["chain_fwd_us"] = timeit(lambda: chain.forward(dense, dc, n, 64, 64), 20)
dzb = torch.randn(n, 64, 64, dc, device=dev).to(torch.bfloat16)
res["chain_pull_us"] = timeit(lambda: chain.pull(dzb, dense, dc, n, 64, 64), 20)
p5 = cplans[4]
out = torch.empty(n, 64, 64, dc, device=dev, dtype=torch.bfloat16)
res["conv5_us"] = timeit(lambda: p5.fwd(dense, dc, 0, 64, 64, out, dc, 0, n, res1=dense, res1_cs=dc, alpha1=0.2), 20)
px = plan(128, 64)
g_in = torch.empty(n, 64, 64, 64, device=dev)
g_out = torch.randn(n, 64, 64, 64, device=dev)
res["pullx_us"] = timeit(lambda: px.fwd(dzb, dc, 0, 64, 64, g_in, 64, 0, n, use_bias=False, out_mode=OUT_F32, res1=g_out, res1_cs=64,
                                        res1_co=0), 20)
# weight gradients: the residual dense block's grouped GEMM shape (128 input x 128 output-gradient channels at 64^2)
# and the trunk's 64 -> 64 (both conv_wgrad64_kernel<1, 1>); the wgrad includes its split-K reduce launch
wsp = Workspace()
for cin, cout in ((128, 128), (64, 64)):
    pw = plan(cin, cout)
    pw.gw = torch.zeros_like(pw.weight)
    pw.gb = torch.zeros(cout, device=dev)
    xw = torch.randn(n, 64, 64, cin, device=dev).to(torch.bfloat16)
    dzw = torch.randn(n, 64, 64, cout, device=dev).to(torch.bfloat16)
    res[f"wgrad_{cin}_us"] = timeit(lambda: pw.wgrad(xw, cin, 0, 64, 64, dzw, cout, n, wsp, accumulate=False), 20)
for cin, cout, hw in ((256, 256, 64), (512, 512, 32)):
    p = plan(cin, cout)
    x = torch.randn(64, hw, hw, cin, device=dev).to(torch.bfloat16)
    y = torch.empty(64, hw, hw, cout, device=dev, dtype=torch.bfloat16)
    res[f"vgg_{cin}_{hw}_us"] = timeit(lambda: p.fwd(x, cin, 0, hw, hw, y, cout, 0, 64, act=ACT_LRELU), 10)
print(json.dumps({k: (round(v, 2) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)
