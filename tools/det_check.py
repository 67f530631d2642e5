"""Run-to-run determinism of the hot kernels at the GAN-step shapes under one libclimsr_hip.so (CLIMSR_HIP_LIB selects
an A/B build): each op runs REPS times on the same inputs (with other launches in between, so the LDS / L2 state
differs) and every output is compared bitwise with the first run.  One JSON line: op -> number of differing elements.
    CLIMSR_HIP_LIB=... python tools/det_check.py <label>"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import _lib  # noqa: E402
from climsr_amd.ops import (ACT_LRELU, ACT_RELU, OUT_F32, BatchedPacker, ConvPlan, RdbChain, Workspace)  # noqa: E402

dev, n = "cuda", 32
REPS = 4
res = {"label": sys.argv[1] if len(sys.argv) > 1 else "", "lib": _lib.LIB_PATH}
g = torch.Generator(device="cpu").manual_seed(5)


def rnd(*shape, dtype=torch.bfloat16, scale=1.0):
    return ((torch.rand(shape, generator=g) * 2 - 1) * scale).to(dev).to(dtype)


def plan(cin, cout, ks=3, stride=1, bias=True):
    p = ConvPlan(cin, cout, ks, stride, None, f"{cin}->{cout}")
    p.bind((rnd(cout, cin, ks, ks, dtype=torch.float32, scale=0.05)).contiguous(), rnd(cout, dtype=torch.float32, scale=0.1) if bias else None)
    p.pack()
    return p


noise_x = rnd(n, 128, 128, 64)
noise_p = plan(64, 64)
noise_y = torch.empty_like(noise_x)


def noise():  # a different kernel between reps (other LDS / cache contents)
    noise_p.fwd(noise_x, 64, 0, 128, 128, noise_y, 64, 0, n, act=ACT_LRELU)


def check(name, run, out, fill=True):
    outs = []
    for _ in range(REPS):
        if fill:
            out.fill_(float("nan"))
        run()
        torch.cuda.synchronize()
        outs.append(out.clone())
        noise()
    res[name] = int(sum(int((o.view(torch.int16 if o.dtype == torch.bfloat16 else torch.int32) !=
                             outs[0].view(torch.int16 if o.dtype == torch.bfloat16 else torch.int32)).sum()) for o in outs[1:]))
    res[name + "_nan"] = int(torch.isnan(outs[0].float()).sum())
    if res[name] and out.dim() == 4:  # where: (image, row, column, channel) of up to 12 differing elements, and the run
        for k, o in enumerate(outs[1:], 1):
            vi = (o.view(torch.int16 if o.dtype == torch.bfloat16 else torch.int32) !=
                  outs[0].view(torch.int16 if o.dtype == torch.bfloat16 else torch.int32)).nonzero()
            if len(vi):
                res[name + f"_where{k}"] = vi[:12].tolist()
                res[name + f"_rows{k}"] = sorted(set(int(r) for r in vi[:, 1].tolist()))[:40]
                res[name + f"_chans{k}"] = sorted(set(int(c) for c in vi[:, 3].tolist()))[:64]


dc, h = 128, 64
dense = rnd(n, h, h, dc)
# RDB conv5 (x5 * 0.2 + x, with and without the RRDB residual) and pull-x
p5 = plan(dc, 64)
r2 = rnd(n, h, h, dc)
y5 = torch.empty(n, h, h, dc, dtype=torch.bfloat16, device=dev)
check("conv5", lambda: p5.fwd(dense, dc, 0, h, h, y5, dc, 0, n, res1=dense, alpha1=0.2, res1_cs=dc, res1_co=0), y5)
check("conv5_res2", lambda: p5.fwd(dense, dc, 0, h, h, y5, dc, 0, n, res1=dense, alpha1=0.2, res1_cs=dc, res1_co=0, res2=r2, alpha2=0.2,
                                   res2_cs=dc, res2_co=0), y5)
px = plan(dc, 64, bias=False)
gout = rnd(n, h, h, 64, dtype=torch.float32)
gin = torch.empty(n, h, h, 64, dtype=torch.float32, device=dev)
aux = torch.zeros(n, h, h, dc, dtype=torch.bfloat16, device=dev)
check("pullx", lambda: px.fwd(dense, dc, 0, h, h, gin, 64, 0, n, use_bias=False, out_mode=OUT_F32, res1=gout, res1_cs=64, res1_co=0, beta1=0.2,
                              aux=aux, aux_cs=dc, aux_co=64, aux_scale=0.04), gin)
# RDB chain forward / pull
cplans = [plan(64 + 16 * (k - 1), 16 if k < 5 else 64) for k in range(1, 6)]
chain = RdbChain(cplans, "det")
BatchedPacker(cplans, torch.device(dev), chain.pack_descs()).run()
pd = chain.pull_descs()
arr = (_lib.PullPackDesc * len(pd))(*pd)
tab = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
_lib.check(_lib.load().climsr_pack_pull_weights_batched(tab.data_ptr(), len(pd), 16 * 9 * 128, _lib.stream_ptr()), "pack")
dfw = dense.clone()
check("chain_fwd", lambda: chain.forward(dfw, dc, n, h, h), dfw, fill=False)
dzb = rnd(n, h, h, dc)
dzp = dzb.clone()


def pull():
    dzp.copy_(dzb)
    chain.pull(dzp, dense, dc, n, h, h)


check("chain_pull", pull, dzp, fill=False)
# conv_wr (HR 64 -> 64: upconv with nearest x2 + LeakyReLU, VGG conv1_2 ReLU), conv_last (64 -> 1)
pw = plan(64, 64)
xh = rnd(n, 128, 128, 64)
yh = torch.empty(n, 256, 256, 64, dtype=torch.bfloat16, device=dev)
check("wr_up2", lambda: pw.fwd(xh, 64, 0, 128, 128, yh, 64, 0, n, up=2, act=ACT_LRELU), yh)
x2 = rnd(n, 256, 256, 64)
check("wr_relu", lambda: pw.fwd(x2, 64, 0, 256, 256, yh, 64, 0, n, act=ACT_RELU), yh)
pl = plan(64, 1)
tail = torch.zeros(n, 256, 256, 8, dtype=torch.bfloat16, device=dev)
check("co1m", lambda: pl.fwd(x2, 64, 0, 256, 256, tail, 8, 0, n), tail)
# VGG conv (the LDS-DMA roofline kernel), D stride-2 forward, stride-2 weight gradient
pv = plan(256, 256)
xv = rnd(64, 64, 64, 256)
yv = torch.empty(64, 64, 64, 256, dtype=torch.bfloat16, device=dev)
check("vgg256", lambda: pv.fwd(xv, 256, 0, 64, 64, yv, 256, 0, 64, act=ACT_RELU), yv)
ps = plan(64, 64, 3, 2, bias=False)
xs = rnd(n, 256, 256, 64)
ys = torch.empty(n, 128, 128, 64, dtype=torch.bfloat16, device=dev)
check("s2_fwd", lambda: ps.fwd(xs, 64, 0, 256, 256, ys, 64, 0, n, use_bias=False), ys)
ps2 = plan(128, 128, 3, 2, bias=False)
xs2 = rnd(n, 128, 128, 128)
dzs = rnd(n, 64, 64, 128)
ps2.gw = torch.zeros_like(ps2.weight)
wsp = Workspace()
check("s2_wgrad", lambda: ps2.wgrad(xs2, 128, 0, 128, 128, dzs, 128, n, wsp, accumulate=False), ps2.gw)
print(json.dumps(res), flush=True)
