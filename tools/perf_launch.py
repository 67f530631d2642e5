"""Per-launch floor of back-to-back kernels in one hipGraph (run on the GPU box):
    python tools/perf_launch.py
Times 200 replayed launches of (a) a 1-block torch kernel, (b) an 8 MB fill, (c) a 64 MB fill."""
import torch


def timeit(fn, reps=200):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


t1 = torch.zeros(16, device="cuda")
t8 = torch.zeros(2 << 20, device="cuda")
t64 = torch.zeros(16 << 20, device="cuda")
print(f"tiny add      {timeit(lambda: t1.add_(1)):7.2f} us/launch")
print(f"8 MB fill     {timeit(lambda: t8.fill_(1)):7.2f} us/launch")
print(f"64 MB fill    {timeit(lambda: t64.fill_(1)):7.2f} us/launch")
