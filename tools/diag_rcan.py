"""Diagnostic (GPU box): where does the native RCAN's whole-grid error come from?
Native vs the oracle in fp32 and under bf16 autocast for growing depth / grid size, plus one generic conv at the
RCAN shape vs float64 on the same bf16 operands.   python tools/diag_rcan.py"""
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import climsr_amd  # noqa: E402,F401
from climsr_amd.core.init import init_state, spec_from_shapes  # noqa: E402
from climsr_amd.models.rcan import RCAN  # noqa: E402
from oracle import climsr_ref as ref  # noqa: E402

torch.backends.cuda.matmul.allow_tf32 = False
torch.backends.cudnn.allow_tf32 = False
DEV = "cuda"


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


def grid(h, w, seed=43):
    g = torch.Generator().manual_seed(seed)
    t = torch.rand((1, 1, 4 * h, 4 * w), generator=g) * 2 - 1
    e = torch.rand((1, 1, 4 * h, 4 * w), generator=g) * 2 - 1
    m = (torch.rand((1, 1, 4 * h, 4 * w), generator=g) < 0.7).float()
    lr = torch.cat([t, e, m], 1)[:, :, ::4, ::4].contiguous()
    return lr.to(DEV), e.to(DEV), m.to(DEV)


def run(ng, nb, h, w):
    net = RCAN(n_resgroups=ng, n_resblocks=nb, n_feats=64, reduction=16, scaling_factor=4, in_channels=3, out_channels=1)
    st = init_state(spec_from_shapes({k: tuple(v.shape) for k, v in net.state_dict().items()}))
    p32 = {k: torch.from_numpy(np.asarray(v)).float() for k, v in st.items()}
    net.load_state_dict(p32)
    net = net.to(DEV).eval()
    lr, e, m = grid(h, w)
    pd = {k: v.to(DEV) for k, v in p32.items()}
    with torch.no_grad():
        sr = net(lr, e, m).float()
        want = ref.rcan_forward(pd, lr, e, m, ng, nb, 4)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            wbf = ref.rcan_forward(pd, lr, e, m, ng, nb, 4).float()
    err = (sr - want).abs()[0, 0]
    rows = err.mean(1)
    print(f"ng {ng} nb {nb} {h}x{w}: native rel {rel(sr, want):.3e}  bf16-autocast rel {rel(wbf, want):.3e}  "
          f"max err {float(err.max()):.3e} worst row {int(rows.argmax())} ({float(rows.max()):.3e} vs mean {float(rows.mean()):.3e}) "
          f"worst col {int(err.mean(0).argmax())}", flush=True)


def conv_check(h, w):
    from climsr_amd.ops import OUT_F32, ConvPlan

    g = torch.Generator().manual_seed(0)
    wt = ((torch.rand((64, 64, 3, 3), generator=g) * 2 - 1) / 24).to(DEV)
    b = ((torch.rand((64,), generator=g) * 2 - 1) * 0.1).to(DEV)
    p = ConvPlan(64, 64, 3, 1, 1, "diag")
    p.bind(wt.contiguous(), b)
    p.pack()
    x = torch.randn((1, h, w, 64), device=DEV).to(torch.bfloat16)
    y = torch.empty((1, h, w, 64), device=DEV)
    aux = torch.empty((1, h, w, 64), device=DEV, dtype=torch.bfloat16)
    p.fwd(x, 64, 0, h, w, y, 64, 0, 1, out_mode=OUT_F32, aux=aux, aux_cs=64)
    torch.cuda.synchronize()
    want = F.conv2d(x.permute(0, 3, 1, 2).double(), wt.to(torch.bfloat16).double(), b.double(), padding=1).permute(0, 2, 3, 1)
    e = (y.double() - want).abs()
    print(f"conv 64->64 {h}x{w}: max rel {float(e.max() / want.abs().max()):.3e}, worst row {int(e.amax((0, 2, 3)).argmax())}, "
          f"aux vs y {float((aux.double() - y.double()).abs().max()):.3e}", flush=True)


if __name__ == "__main__" and len(sys.argv) == 1:
    conv_check(360, 720)
    conv_check(64, 64)
    for ng, nb, h, w in [(1, 1, 16, 16), (1, 1, 360, 720), (1, 4, 360, 720), (2, 4, 360, 720), (10, 20, 16, 16), (10, 20, 64, 64),
                         (10, 20, 360, 720)]:
        run(ng, nb, h, w)


def locate(ng=10, nb=20, h=360, w=720):
    """Determinism, error map at LR resolution, and the oracle's residual-stream magnitude per group."""
    net = RCAN(n_resgroups=ng, n_resblocks=nb, n_feats=64, reduction=16, scaling_factor=4, in_channels=3, out_channels=1)
    st = init_state(spec_from_shapes({k: tuple(v.shape) for k, v in net.state_dict().items()}))
    p32 = {k: torch.from_numpy(np.asarray(v)).float() for k, v in st.items()}
    net.load_state_dict(p32)
    net = net.to(DEV).eval()
    lr, e, m = grid(h, w)
    pd = {k: v.to(DEV) for k, v in p32.items()}
    with torch.no_grad():
        a = net(lr, e, m).float()
        b = net(lr, e, m).float()
        want = ref.rcan_forward(pd, lr, e, m, ng, nb, 4)
    print("determinism: max |run1 - run2|", float((a - b).abs().max()), flush=True)
    err = F.avg_pool2d((a - want).abs(), 4)[0, 0]
    v, i = err.flatten().topk(8)
    print("top LR-block errors:", [(int(k) // w, int(k) % w, round(float(x), 5)) for x, k in zip(v, i)], "mean", float(err.mean()))
    # oracle residual stream per group
    with torch.no_grad():
        hd = ref._conv(pd, "head.0", lr)
        t = hd
        for gi in range(ng):
            gin = t
            for bi in range(nb):
                pre = f"body.{gi}.body.{bi}.body"
                u = ref._conv(pd, pre + ".2", F.relu(ref._conv(pd, pre + ".0", t)))
                y = u.mean(dim=(2, 3), keepdim=True)
                y = torch.sigmoid(ref._conv(pd, pre + ".3.conv_du.2", F.relu(ref._conv(pd, pre + ".3.conv_du.0", y))))
                t = u * y + t
            t = ref._conv(pd, f"body.{gi}.body.{nb}", t) + gin
            am = t.abs().amax(1)[0]
            k = int(am.flatten().argmax())
            print(f"group {gi}: |t| max {float(am.max()):.3f} at {(k // w, k % w)}, rms {float(t.pow(2).mean().sqrt()):.3f}", flush=True)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "locate":
    locate()
