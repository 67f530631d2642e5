"""Throughput of the on-device tile pipeline and validation metrics, run on the GPU box:
    python tools/perf_pipeline.py [--tiles 32] [--big 1024]

Kernel times are HIP-event averages over graph-replayed launches on the launch stream.  Algorithmic bytes:
  tile_prepare  per HR pixel: read hr_raw 4 + elev_raw 4; write hr 4 + elevation 4 + mask 4 + lr 12/s^2
                (= 20.75 B at s = 4); tile_minmax reads elev_raw 4 B/px.
  sr_metrics    per HR pixel: read sr, hr, original, mask 16 B (first pass) + 16 B (SSIM pass re-reads).
The CPU baseline is the numpy restatement of the reference's per-sample ClimateDataset work
(oracle/data_ref.py, the same arithmetic the reference's DataLoader workers run), single thread.
"""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import _lib  # noqa: E402
from climsr_amd._lib import TileDesc, check, ptr  # noqa: E402
from climsr_amd.metrics import SRMetrics  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--tiles", type=int, default=32)
ap.add_argument("--big", type=int, default=1024)
ap.add_argument("--hr", type=int, default=128)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--no-cpu", action="store_true")
args = ap.parse_args()
dev = "cuda"
HBM_PEAK = 8.0e12


def graph_time(fn, reps):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(side):
        with torch.cuda.graph(g, stream=side):
            for _ in range(reps):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e-3  # seconds per call


def raw_tiles(n, h, seed=0):
    g = torch.Generator(device=dev).manual_seed(seed)
    hr = torch.rand((n, h, h), device=dev, generator=g) * 40 - 10
    hr = torch.where(torch.rand((n, h, h), device=dev, generator=g) < 0.3, torch.full_like(hr, float("nan")), hr)
    el = torch.rand((n, h, h), device=dev, generator=g) * 2500
    el = torch.where(torch.rand((n, h, h), device=dev, generator=g) < 0.05, torch.full_like(el, -32768.0), el)
    return hr.contiguous(), el.contiguous()


def bench_pipeline(n, h):
    s = 4
    hr_raw, el_raw = raw_tiles(n, h)
    mn = torch.full((n,), -12.5, dtype=torch.float64, device=dev)
    mx = torch.full((n,), 31.0, dtype=torch.float64, device=dev)
    xf = torch.randint(0, 16, (n,), dtype=torch.int32, device=dev)
    lr = torch.empty((n, 3, h // s, h // s), device=dev)
    hr, el, mask = (torch.empty((n, 1, h, h), device=dev) for _ in range(3))
    mm = torch.empty((n, 2), device=dev)
    d = TileDesc(hr_raw=ptr(hr_raw), elev_raw=ptr(el_raw), hr_min=ptr(mn), hr_max=ptr(mx), elev_minmax=ptr(mm), xform=ptr(xf),
                 lr=ptr(lr), hr=ptr(hr), elev=ptr(el), mask=ptr(mask), range_a=-1.0, range_b=1.0, eps=1e-8, nan_sub=0.0,
                 zs_hr_std=1.0, zs_elev_std=1.0, elev_missing=-32768.0, method=0, n=n, h=h, w=h, scale=s, lr_c=3, srcnn=0,
                 use_elev=1, use_mask=1)
    L = _lib.load()

    def minmax():
        check(L.climsr_tile_minmax_f32(ptr(el_raw), n, h * h, -32768.0, 1, ptr(mm), _lib.stream_ptr()), "minmax")

    def prepare():
        check(L.climsr_tile_prepare(ctypes.byref(d), _lib.stream_ptr()), "prepare")

    t_mm = graph_time(minmax, args.reps)
    t_pr = graph_time(prepare, args.reps)
    px = n * h * h
    b_pr = px * (4 + 4 + 4 + 4 + 4 + 12 / (s * s))
    return {"what": "tile_pipeline", "tiles": n, "hr": h, "us_minmax": t_mm * 1e6, "us_prepare": t_pr * 1e6,
            "tiles_per_s": n / (t_mm + t_pr), "prepare_GBps": b_pr / t_pr / 1e9, "prepare_frac": b_pr / t_pr / HBM_PEAK,
            "minmax_GBps": px * 4 / t_mm / 1e9}


def bench_metrics(n, h):
    hr_raw, _ = raw_tiles(n, h, seed=1)
    mask = (~torch.isnan(hr_raw)).float().reshape(n, 1, h, h)
    hr = torch.nan_to_num(hr_raw / 20.0).reshape(n, 1, h, h).contiguous()
    sr = (hr + 0.01 * torch.randn_like(hr)).contiguous()
    orig = hr_raw.reshape(n, 1, h, h).contiguous()
    mn = torch.full((n,), -12.5, dtype=torch.float64, device=dev)
    mx = torch.full((n,), 31.0, dtype=torch.float64, device=dev)
    m = SRMetrics()
    t = graph_time(lambda: m.raw(sr, hr, orig, mask, mn, mx), args.reps)
    px = n * h * h
    return {"what": "sr_metrics", "tiles": n, "hr": h, "us": t * 1e6, "tiles_per_s": n / t, "GBps": 32 * px / t / 1e9,
            "frac": 32 * px / t / HBM_PEAK}


rows = [bench_pipeline(args.tiles, args.hr), bench_pipeline(args.big, args.hr), bench_metrics(args.tiles, args.hr),
        bench_metrics(args.big, args.hr)]
if not args.no_cpu:
    from oracle import data_ref as dr  # CPU baseline (numpy restatement of the reference's per-sample work)

    rs = np.random.RandomState(0)
    n, h = args.tiles, args.hr
    hr_np = (rs.rand(n, h, h).astype(np.float32) * 40 - 10)
    el_np = (rs.rand(n, h, h) * 2500).astype(np.float32)
    t0 = time.perf_counter()
    dr.prepare_batch(hr_np, el_np, np.full(n, -12.5), np.full(n, 31.0), rs.randint(0, 16, n).astype(np.int32))
    t_cpu = time.perf_counter() - t0
    rows.append({"what": "cpu_baseline_tile_pipeline", "tiles": n, "hr": h, "tiles_per_s": n / t_cpu, "cores": 1, "kind": "port"})
    k = 8
    sr = rs.rand(k, 1, h, h).astype(np.float32)
    t0 = time.perf_counter()
    dr.sr_metrics(sr, sr * 0.9, sr * 30, np.ones_like(sr), np.full(k, -12.5), np.full(k, 31.0))
    t_cpu = time.perf_counter() - t0
    rows.append({"what": "cpu_baseline_sr_metrics", "tiles": k, "hr": h, "tiles_per_s": k / t_cpu, "cores": 1, "kind": "port"})
for r in rows:
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in r.items()}))
