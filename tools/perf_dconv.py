"""Micro-benchmark (GPU box) of the discriminator / perceptual-loss convs at the GAN bench shapes:
RFB discriminator features (rfb_esrgan.py:28-52, B=32, 256^2 input, no bias, bf16 out for the BN) forward, bf16 data
gradient and weight gradient; VGG19 features[:35] (perceptual.py:15, fake+real = 2B images) forward with bias+ReLU.
    python tools/perf_dconv.py [--batch 32] [--only d|vgg]"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd.ops import ACT_LRELU_BWD, ACT_RELU, ConvPlan, Workspace  # noqa: E402
from tests.perf_conv_timing import timeit  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--reps", type=int, default=10)
ap.add_argument("--only", default="")
args = ap.parse_args()
dev = "cuda"
n = args.batch


def mkplan(cin, cout, stride, bias, name):
    p = ConvPlan(cin, cout, 3, stride, 1, name)
    w = (torch.randn(cout, cin, 3, 3, device=dev) * (2.0 / (9 * cin)) ** 0.5).contiguous()
    p.bind(w, torch.zeros(cout, device=dev) if bias else None, need_t=True)
    p.pack()
    p.gw = torch.zeros_like(w)
    p.gb = None
    return p


tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
ws = Workspace()
if args.only in ("", "d"):
    print("-- RFB discriminator, B=%d --" % n)
    h = 256
    for cin, cout, stride in [(64, 64, 2), (64, 128, 1), (128, 128, 2), (128, 256, 1), (256, 256, 2), (256, 512, 1), (512, 512, 2)]:
        p = mkplan(cin, cout, stride, False, f"{cin}->{cout}s{stride}")
        oh = h // stride
        x = torch.randn(n, h, h, cin, device=dev).to(torch.bfloat16)
        y = torch.empty(n, oh, oh, cout, device=dev, dtype=torch.bfloat16)
        fl = 2 * cin * cout * 9 * n * oh * oh
        t = timeit(lambda: p.fwd(x, cin, 0, h, h, y, cout, 0, n, use_bias=False), args.reps)
        dz = torch.randn(n, oh, oh, cout, device=dev).to(torch.bfloat16)
        g = torch.empty(n, h, h, cin, device=dev, dtype=torch.bfloat16)
        td = timeit(lambda: p.dgrad(dz, cout, oh, oh, g, cin, 0, n), args.reps)
        tw = timeit(lambda: p.wgrad(x, cin, 0, h, h, dz, cout, n, ws, accumulate=False), args.reps)
        if stride == 2 and cin == 64:  # layer 1: the data gradient also applies layer 0's LeakyReLU' (rfb_esrgan.py:29)
            ta = timeit(lambda: p.dgrad(dz, cout, oh, oh, g, cin, 0, n, act=ACT_LRELU_BWD, res1=x, res1_cs=cin, res1_co=0),
                        args.reps)
            print(f"{p.name:14s} @{h:3d}  dgrad + LeakyReLU' {ta:7.1f} us {(dz.numel() + 2 * g.numel()) * 2 / ta / 1e6:5.2f} TB/s")
        tot["fwd"] += t
        tot["dgrad"] += td
        tot["wgrad"] += tw
        io = (x.numel() + y.numel()) * 2
        print(f"{p.name:14s} @{h:3d}  fwd {t:7.1f} us {fl / t / 1e6:6.0f} TF {io / t / 1e6:5.2f} TB/s | dgrad {td:7.1f} us "
              f"{fl / td / 1e6:6.0f} TF | wgrad {tw:7.1f} us {fl / tw / 1e6:6.0f} TF", flush=True)
        h = oh
        del x, y, dz, g
    print(f"D total: fwd {tot['fwd']:.1f} us, dgrad {tot['dgrad']:.1f} us, wgrad {tot['wgrad']:.1f} us", flush=True)
if args.only in ("", "vgg"):
    n2 = 2 * n
    print("-- VGG19 features[:35], %d images --" % n2)
    h, cin, t_all = 256, 64, 0.0
    for cout, pool in [(64, True), (128, False), (128, True), (256, False), (256, False), (256, False), (256, True), (512, False),
                       (512, False), (512, False), (512, True), (512, False), (512, False), (512, False), (512, False)]:
        p = mkplan(cin, cout, 1, True, f"{cin}->{cout}")
        x = torch.randn(n2, h, h, cin, device=dev).to(torch.bfloat16)
        y = torch.empty(n2, h, h, cout, device=dev, dtype=torch.bfloat16)
        fl = 2 * cin * cout * 9 * n2 * h * h
        t = timeit(lambda: p.fwd(x, cin, 0, h, h, y, cout, 0, n2, act=ACT_RELU), args.reps)
        t_all += t
        print(f"{p.name:14s} @{h:3d}  fwd {t:7.1f} us {fl / t / 1e6:6.0f} TF", flush=True)
        cin = cout
        if pool:
            h //= 2
        del x, y
    print(f"VGG total fwd {t_all:.1f} us", flush=True)
