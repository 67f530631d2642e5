"""Microbenchmark (GPU box): fc.0 forward / data gradient of the RFB discriminator at the bench shape (n=32, k=100352,
o=1024), row-major weight against the fragment-order copy (climsr_linear_pack_frag), HIP-event timed medians, plus the
AdamW pass over a flat buffer holding the weight with its bf16 copy written row-major or in fragment order.
    python tools/bench_linear_fc0.py   (one JSON line)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps=30):
    import torch

    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) * 1e3)
    ts.sort()
    return round(ts[len(ts) // 2], 2)


def main():
    import torch

    from climsr_amd import _lib, ops

    n, k, o = 32, 100352, 1024
    dev = "cuda"
    x = (torch.randn((n, k), device=dev) * 0.5).to(torch.bfloat16)
    w32 = torch.randn((o, k), device=dev) / k ** 0.5
    w = w32.to(torch.bfloat16)
    wf = torch.empty(o * k, dtype=torch.bfloat16, device=dev)
    ops.linear_pack_frag(w32, o, k, wf)
    b = torch.zeros(o, device=dev)
    y = torch.empty((n, o), device=dev)
    ws = torch.empty(2000 * n * o, device=dev)
    dy = torch.randn((n, o), device=dev).to(torch.bfloat16)
    dx = torch.empty((n, k), device=dev)
    res = {
        "fwd_us": timed(lambda: ops.linear_fwd(x, w, b, n, k, o, y, ws)),
        "fwd_frag_us": timed(lambda: ops.linear_fwd_frag(x, wf, b, n, k, o, y, ws)),
        "dgrad_us": timed(lambda: ops.linear_dgrad(dy, w, n, k, o, dx)),
        "dgrad_frag_us": timed(lambda: ops.linear_dgrad_frag(dy, wf, n, k, o, dx)),
    }
    lib = _lib.load()
    lo, nf = 4 * 1024 * 1024, o * k + 4 * 1024 * 1024  # D's flat: 4 M conv / BN parameters, then fc.0
    p = torch.randn(nf + 1025, device=dev) * 0.01
    g, m, v = torch.randn_like(p) * 1e-3, torch.zeros_like(p), torch.zeros_like(p)
    hp = torch.tensor([1e-4, 0.9, 0.999, 1e-8, 1e-4, 1e-3, 1.0, 0.0], device=dev)
    mir = torch.empty(o * k, dtype=torch.bfloat16, device=dev)
    s = _lib.stream_ptr()
    P = lambda t: t.data_ptr()  # noqa: E731
    res["adamw_mirror_us"] = timed(lambda: lib.climsr_adamw_step_mirror(p.numel(), P(p), P(g), P(m), P(v), P(hp), lo, o * k, P(mir), s), 10)
    res["adamw_mirror_frag_us"] = timed(lambda: lib.climsr_adamw_step_mirror_frag(p.numel(), P(p), P(g), P(m), P(v), P(hp), lo, o, k,
                                                                                  P(mir), s), 10)
    n_pad = 32
    dy_t = torch.randn((o, n_pad), device=dev).to(torch.bfloat16)
    x_t = torch.randn((k, n_pad), device=dev).to(torch.bfloat16)
    dw = torch.empty((o, k), device=dev)

    def two():
        ops.linear_wgrad(dy_t, x_t, n_pad, k, o, dw, False)
        ops.linear_wgrad(dy_t, x_t, n_pad, k, o, dw, True)

    res["wgrad_two_launches_us"] = timed(two, 10)
    res["wgrad2_us"] = timed(lambda: ops.linear_wgrad2(dy_t, x_t, n_pad, dy_t, x_t, n_pad, k, o, dw, False), 10)
    res["weight_tbs_fwd"] = round(o * k * 2 / res["fwd_us"] / 1e6, 2)
    res["weight_tbs_fwd_frag"] = round(o * k * 2 / res["fwd_frag_us"] / 1e6, 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
