"""Micro-benchmark of the conv kernels on the generator's hot shapes (run on the GPU box):
    python tools/perf_conv.py [--batch 32]
Prints per-op average launch time (HIP events, 20 reps after warm-up) and TFLOP/s."""
import argparse
import sys

sys.path.insert(0, "/root/repo")
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd.ops import ACT_LRELU, OUT_F32, ConvPlan, Workspace  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=32)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--rdb-only", action="store_true")
args = ap.parse_args()
dev = "cuda"
n = args.batch


def timeit(fn, reps):
    """Average GPU time per launch: `reps` launches captured in one hipGraph and replayed (no host overhead)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(gr, stream=side):
            for _ in range(reps):
                fn()
    torch.cuda.synchronize()
    gr.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    gr.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def plan(cin, cout, ks, up=1):
    p = ConvPlan(cin, cout, ks, 1, None, f"{cin}->{cout}k{ks}")
    w = (torch.randn(cout, cin, ks, ks, device=dev) * 0.05).contiguous()
    b = torch.zeros(cout, device=dev)
    p.bind(w, b)
    p.pack()
    p.gw = torch.zeros_like(w)
    p.gb = torch.zeros_like(b)
    return p


rows = []
ws = Workspace()
for (cin, cout, ks, h, up) in [] if args.rdb_only else [(64, 16, 3, 64, 1), (112, 16, 3, 64, 1), (128, 64, 3, 64, 1), (64, 64, 3, 128, 2), (64, 64, 3, 256, 1),
                               (3, 64, 9, 256, 1), (64, 1, 3, 256, 1), (32, 1, 5, 256, 1)]:
    p = plan(cin, cout, ks, up)
    hin = h // up
    dense = torch.randn(n, hin, hin, max(8, (cin + 7) // 8 * 8), device=dev).to(torch.bfloat16)
    cs = dense.shape[-1]
    ocs = (cout + 7) // 8 * 8
    y = torch.zeros(n, h, h, ocs, device=dev, dtype=torch.bfloat16)
    flops = 2 * cin * cout * ks * ks * n * h * h
    t = timeit(lambda: p.fwd(dense, cs, 0, hin, hin, y, ocs, 0, n, up=up, act=ACT_LRELU), args.reps)
    rows.append((f"fwd   {p.name} @{h}", t, flops))
    dz = torch.randn(n, h, h, p.cin_t, device=dev).to(torch.bfloat16)
    g = torch.zeros(n, hin, hin, p.cin, device=dev)
    if up == 1:
        t = timeit(lambda: p.dgrad(dz, p.cin_t, h, h, g, p.cin, 0, n, accumulate=True), args.reps)
    else:
        t = timeit(lambda: p.dgrad(dz, p.cin_t, h, h, g, p.cin, 0, n, accumulate=True, down2=True), args.reps)
    rows.append((f"dgrad {p.name} @{h}", t, flops))
    t = timeit(lambda: p.wgrad(dense, cs, 0, hin, hin, dz, p.cin_t, n, ws, accumulate=False, up=up), args.reps)
    rows.append((f"wgrad {p.name} @{h}", t, flops))
for name, t, f in rows:
    print(f"{name:32s} {t:9.1f} us  {f / t / 1e6:8.1f} TFLOP/s")

# RDB-shaped launches as the generator issues them: 128-channel dense buffer, channel slices
print("-- RDB (dense 128-ch buffer, slices) --")
dc = 128
dense = torch.randn(n, 64, 64, dc, device=dev).to(torch.bfloat16)
for k in range(1, 6):
    cin = 64 + 16 * (k - 1)
    cout = 16 if k < 5 else 64
    p = plan(cin, cout, 3)
    if k < 5:
        t = timeit(lambda: p.fwd(dense, dc, 0, 64, 64, dense, dc, cin, n, act=ACT_LRELU), args.reps)
    else:
        out = torch.empty(n, 64, 64, dc, device=dev, dtype=torch.bfloat16)
        t = timeit(lambda: p.fwd(dense, dc, 0, 64, 64, out, dc, 0, n, res1=dense, res1_cs=dc, alpha1=0.2), args.reps)
    f = 2 * cin * cout * 9 * n * 64 * 64
    print(f"fwd conv{k} {cin}->{cout}".ljust(32), f"{t:9.1f} us  {f / t / 1e6:8.1f} TFLOP/s")

# fused RDB chain (conv1..conv4 / pull4..pull1 in one launch)
from climsr_amd.ops import BatchedPacker, PullPacker, RdbChain  # noqa: E402

cplans = []
for k in range(1, 6):
    cin = 64 + 16 * (k - 1)
    cplans.append(plan(cin, 16 if k < 5 else 64, 3))
chain = RdbChain(cplans, "perf")
BatchedPacker(cplans, torch.device(dev), chain.pack_descs()).run()
PullPacker([], torch.device(dev), chain.pull_descs()).run() if False else None
from climsr_amd import _lib as _l  # noqa: E402
import ctypes as _ct  # noqa: E402

pd = chain.pull_descs()
arr = (_l.PullPackDesc * len(pd))(*pd)
tab = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
_l.check(_l.load().climsr_pack_pull_weights_batched(tab.data_ptr(), len(pd), 16 * 9 * 128, _l.stream_ptr()), "pack")
f = sum(2 * (64 + 16 * k) * 16 * 9 for k in range(4)) * n * 64 * 64
t = timeit(lambda: chain.forward(dense, dc, n, 64, 64), args.reps)
print("chain fwd conv1..4".ljust(32), f"{t:9.1f} us  {f / t / 1e6:8.1f} TFLOP/s")
dzb = torch.randn(n, 64, 64, dc, device=dev).to(torch.bfloat16)
t = timeit(lambda: chain.pull(dzb, dense, dc, n, 64, 64), args.reps)
print("chain pull4..1".ljust(32), f"{t:9.1f} us  {f / t / 1e6:8.1f} TFLOP/s")
