"""Microbenchmark (GPU box): fc.0 forward / dgrad / wgrad of the RFB discriminator at the bench shape
(n=32, k=100352, o=1024), HIP-event timed, each configuration in a fresh child process (env knobs are read per call).
    python tools/bench_linear_fc0.py"""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def one():
    import torch

    from climsr_amd import ops

    n, k, o = 32, 100352, 1024
    dev = "cuda"
    x = (torch.randn((n, k), device=dev) * 0.5).to(torch.bfloat16)
    w = (torch.randn((o, k), device=dev) / k ** 0.5).to(torch.bfloat16)
    b = torch.zeros(o, device=dev)
    y = torch.empty((n, o), device=dev)
    ws = torch.empty(2000 * n * o, device=dev)
    want = (x.float() @ w.float().t())
    res = {}
    for name, fn in [("fwd", lambda: ops.linear_fwd(x, w, b, n, k, o, y, ws))]:
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ts = []
        for _ in range(30):
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
        ts.sort()
        res[name] = ts[len(ts) // 2]
    res["err"] = float((y - want).abs().max() / want.abs().max())
    res["tbs"] = o * k * 2 / res["fwd"] / 1e6
    print(json.dumps(res))


if __name__ == "__main__":
    if len(sys.argv) > 1:
        one()
        sys.exit(0)
    for wg in ["384", "768", "1024", "1536"]:
        for kw in ["1", "2", "4"]:
            for rnd in ["128", "256"]:
                env = dict(os.environ, CLIMSR_LIN_WG=wg, CLIMSR_LIN_KW=kw, CLIMSR_LIN_ROUND=rnd)
                out = subprocess.run([sys.executable, __file__, "one"], env=env, capture_output=True, text=True, timeout=120)
                print(wg, kw, rnd, out.stdout.strip() or out.stderr[-400:], flush=True)
