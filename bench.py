"""Benchmark: HR MPix/s per training step of 4x ESRGAN SR on synthetic 64->256 tiles (BASELINE.json).

Default workload = BASELINE config 3 (the metric's step, BASELINE.md §2 "both optimizer passes"): the full
ESRGAN GAN training step of ``GANLightningModule.training_step`` (pl_gan.py:63-97) -- generator pass (G
forward, RFB discriminator on hr and sr, VGG19 perceptual + relativistic adversarial + L1 losses, G backward,
AdamW_G), then the discriminator pass (fresh G forward, D on hr and sr.detach(), D backward, AdamW_D) and both
OneCycleLR steps -- with the RRDB generator (nf 64, nb 11, gc 16; conf/generator/esrgan.yaml), per-GPU batch
32, bf16 MFMA compute, fp32 master weights / optimiser state.  Each step segment is captured once as a hipGraph
and replayed.  The config-2 L1 pre-training step is measured in the same run and reported as ``config2``.

Multi-GPU: ``--gpus N`` launches N ranks itself (one process per GPU, RANK / LOCAL_RANK / WORLD_SIZE /
MASTER_ADDR=127.0.0.1 / MASTER_PORT in each child's environment; the launcher never touches the GPU) unless a
launcher (torchrun) already set WORLD_SIZE.  Per-rank seeded tiles (seed 42 + rank); the flat fp32 gradient
buffers are averaged over RCCL (DDP semantics, overlapped with the backward); every rank steps its own
replica.  Rank 0 prints ONE JSON line.
"""
import argparse
import functools
import json
import os
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_HBM_GBS = 8000.0
G_FWD_FLOP_PER_PX = 721_880  # 23,654,563,840 MAC per 64^2 sample / 65,536 HR px * 2
GAN_FLOP_PER_PX = 6_140_192  # (4 G + 9 D + 2 VGG) MAC * 2 / 65,536 at 256^2


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--median-steps", type=int, default=50,
                    help="extra steps timed one by one (HIP events) after the timed loop: median per-step time")
    ap.add_argument("--batch", type=int, default=32, help="per-GPU batch")
    ap.add_argument("--lr-size", type=int, default=64)
    ap.add_argument("--nb", type=int, default=11)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--no-config2", action="store_true", help="gan mode: skip the config-2 (L1 pretrain) sub-record")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--mode", choices=["pretrain", "gan", "infer"], default="gan",
                    help="gan = BASELINE config 3 (the metric's step: G + RFB-D + VGG19 perceptual, both optimizer passes); "
                         "pretrain = config 2 (L1 pre-training); infer = config 5 (whole-grid inference)")
    ap.add_argument("--model", choices=["rcan", "esrgan"], default="rcan",
                    help="infer mode: RCAN 10x20 (conf/inference.yaml's default) or the ESRGAN generator")
    ap.add_argument("--grid-h", type=int, default=360, help="infer mode: LR grid rows (CRU-TS 0.5 deg: 360)")
    ap.add_argument("--grid-w", type=int, default=720, help="infer mode: LR grid columns (720)")
    return ap.parse_args(argv)


# ------------------------------------------------------------------------------------------- launcher
def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def child_envs(n: int, port: int, base=None):
    """Environment of each of the n ranks (torchrun's variables; one node, rendezvous on 127.0.0.1)."""
    base = dict(os.environ if base is None else base)
    envs = []
    for r in range(n):
        e = dict(base)
        e.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        e.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver (RCCL)
        envs.append(e)
    return envs


LAUNCH_TIMEOUT_S = float(os.environ.get("CLIMSR_LAUNCH_TIMEOUT", "1200"))


def launch(n: int, cmd, timeout=LAUNCH_TIMEOUT_S) -> int:
    """Start n child processes of ``cmd`` (one per GPU) and wait for all of them.  Rank 0's stdout is passed
    through; every rank's stderr is inherited.  If a rank fails, the others are killed (by PID) and its exit
    code is returned.  A run still going after ``timeout`` seconds (default 1200, CLIMSR_LAUNCH_TIMEOUT; None =
    no limit) is killed rank by rank and returns 124, so one hung rank cannot hang the launcher.  The launcher
    itself never initialises the GPU."""
    port = free_port()
    procs = []
    for r, env in enumerate(child_envs(n, port)):
        procs.append(subprocess.Popen(cmd, env=env, stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    t0 = time.time()
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.kill()
        if timeout is not None and time.time() - t0 > timeout:
            for q in live:
                q.kill()
            for q in live:
                q.wait()
            print(f"[bench] launcher: ranks still running after {timeout:.0f} s were killed", file=sys.stderr, flush=True)
            return rc or 124
        time.sleep(0.05)
    return rc


def cpu_info():
    """Host CPU model, affinity cores and the cgroup CPU quota (the GPU box shows the whole machine's CPUs but
    grants one GPU a share of them)."""
    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return {"cpu_model": model, "affinity_cores": aff, "cgroup_quota_cores": quota,
            "threads": min(aff, quota) if quota else aff}


@functools.lru_cache(maxsize=None)
def _lib_sha256(path):
    """sha256 of the HIP library (hashed once per process: 9 MB)."""
    import hashlib

    return hashlib.sha256(open(path, "rb").read()).hexdigest()


def pmc_traffic(kernel, mode):
    """HBM bytes per launch of `kernel` from the newest committed rocprofv3 PMC summary of this workload
    (profiles/r*_<mode>_pmc_traffic.json: separate FETCH_SIZE / WRITE_SIZE passes of this bench,
    FETCH_SIZE x2 gfx950 correction, MI355X_MICROARCH.md).  The summary carries the sha256 of the library it
    profiled; counters of any other build describe other code, so they are refused: (None, reason)."""
    import glob
    import re

    from climsr_amd import _lib

    def build_key(path):  # r02_v11 after r02_v9: (round, version) as numbers, not as text
        m = re.match(r"r(\d+)_v(\d+)_", os.path.basename(path))
        return (int(m.group(1)), int(m.group(2))) if m else (-1, -1)

    files = sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_{mode}_pmc_traffic.json")), key=build_key)
    if not files:
        return None, "no PMC summary for this workload under profiles/"
    running = _lib_sha256(_lib.LIB_PATH)
    for f in reversed(files):
        try:
            doc = json.load(open(f))
        except (OSError, ValueError):
            continue
        if doc.get("lib_sha256") != running:
            continue
        rec = doc.get("kernels", {}).get(kernel)
        if not rec:
            return None, f"{os.path.basename(f)} (this build) has no record of {kernel}"
        return rec["hbm_bytes_per_launch"], os.path.basename(f)
    return None, f"no PMC summary under profiles/ was taken on this build (libclimsr_hip.so sha256 {running[:16]})"


class KernelTimer:
    """HIP-event timer around individual launches (ops.PROFILER hook), grouped by kernel name."""

    def __init__(self):
        self.rec = []
        self.fns = {}

    def __call__(self, name, flops, fn, tag="", nbytes=0):
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        fn()
        e.record()
        self.rec.append((name, flops, s, e, tag, nbytes))
        self.fns.setdefault(name, []).append(fn)

    def graph_us(self, name, reps=3):
        """Average launch duration of `name` with its launches of one step replayed back to back from a
        hipGraph (HIP events around the replay): the per-launch event pairs above also time the dispatch gap,
        which dominates for short kernels."""
        fns = self.fns[name]
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        gr = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            with torch.cuda.graph(gr, stream=side):
                for fn in fns:
                    fn()
        torch.cuda.synchronize()
        gr.replay()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(reps):
            gr.replay()
        e.record()
        torch.cuda.synchronize()
        return s.elapsed_time(e) * 1e3 / (reps * len(fns))

    def by_tag(self, top=25):
        torch.cuda.synchronize()
        agg = {}
        for name, flops, s, e, tag, _b in self.rec:
            key = name + " | " + ".".join(t for t in tag.split(".") if not t.isdigit() and not t.startswith("RDB"))
            a = agg.setdefault(key, [0, 0.0, 0])
            a[0] += 1
            a[1] += s.elapsed_time(e)
            a[2] += flops
        rows = sorted(agg.items(), key=lambda kv: -kv[1][1])[:top]
        return {k: {"n": v[0], "ms": round(v[1], 3), "tflops": round(v[2] / (v[1] / 1e3) / 1e12, 1)} for k, v in rows}

    def summary(self):
        """{kernel: [launches, ms, algorithmic flops, algorithmic bytes]}"""
        torch.cuda.synchronize()
        agg = {}
        for name, flops, s, e, _tag, nbytes in self.rec:
            a = agg.setdefault(name, [0, 0.0, 0, 0])
            a[0] += 1
            a[1] += s.elapsed_time(e)
            a[2] += flops
            a[3] += nbytes
        return agg


def roofline_entry(name, cnt, tot_ms, flops, nbytes, graph_us=None):
    """Roofline of one kernel: bound = the resource its algorithmic intensity saturates first (MFMA when
    flops/bytes >= the ridge 2500 TFLOP/s / 8 TB/s = 312 FLOP/B, else HBM); achieved = algorithmic work per
    launch / average launch time, in that resource's unit."""
    # The headline launch time is the per-launch HIP event pair on the launch stream, inside the eager step (an upper
    # bound: it includes the dispatch gap; it agrees with the rocprofv3 kernel-trace average of the bench run within a
    # few %).  The isolated hipGraph replay of the kernel's launches runs on operands the step has just touched (hot
    # caches) and is kept only as a diagnostic.
    eager_s = tot_ms / cnt / 1e3
    avg_s = eager_s
    ridge = PEAK_BF16_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9)
    ai = flops / nbytes if nbytes else float("inf")
    out = {"kernel": name, "launches_per_step": cnt, "avg_launch_us": round(avg_s * 1e6, 2),
           "avg_launch_us_source": "per-launch HIP events on the launch stream (eager step)",
           "eager_event_us": round(eager_s * 1e6, 2),
           "graph_replay_us_diagnostic": round(graph_us, 2) if graph_us else None, "flop_per_launch": flops // cnt,
           "bytes_per_launch": nbytes // cnt, "intensity_flop_per_byte": round(ai, 1) if nbytes else None,
           "tflops": round(flops / cnt / avg_s / 1e12, 2), "gbs": round(nbytes / cnt / avg_s / 1e9, 1) if nbytes else None}
    if ai >= ridge:
        out.update(bound="mfma", achieved=out["tflops"], peak=PEAK_BF16_TFLOPS, unit="TFLOP/s")
    else:
        out.update(bound="hbm", achieved=out["gbs"], peak=PEAK_HBM_GBS, unit="GB/s")
    out["frac"] = round(out["achieved"] / out["peak"], 4)
    return out


def cpu_baseline(args, hr, mode):
    """Oracle (PyTorch-CPU fp32 eager restatement of the same step, oracle/climsr_ref.py) on the host cores,
    bounded sample: batch 2 at the benchmark's tile size, ~args.cpu_seconds of steps after one warm-up step."""
    from oracle import climsr_ref as ref
    from tests.helpers import gen_params, rfb_d_params, vgg_params

    info = cpu_info()
    threads = info["threads"]
    torch.set_num_threads(threads)
    b = 2
    p = {k: v.float() for k, v in gen_params(args.nb, torch.float32).items()}
    opt = ref.AdamWState(p, list(p.keys()), lr=1e-4, total_steps=1000)
    bt = ref.synthetic_batch(b, hr)
    if mode == "pretrain":
        fn = lambda: ref.pretrain_step(p, opt, bt, args.nb)  # noqa: E731
        what = "L1-pretrain step (config 2)"
    else:
        dp = {k: (v.float() if v.is_floating_point() else v) for k, v in rfb_d_params().items()}
        vp = {k: v.float() for k, v in vgg_params().items()}
        opt_d = ref.AdamWState(dp, ref.trainable_keys(dp), lr=1e-4, total_steps=1000)
        fn = lambda: ref.gan_step(p, dp, vp, opt, opt_d, bt, args.nb)  # noqa: E731
        what = "full GAN step (config 3: G + RFB-D + VGG19 perceptual, both optimizer passes)"
    def timed(fn, seconds):
        fn()  # warm-up
        t0 = time.perf_counter()
        n = 0
        while True:
            fn()
            n += 1
            if time.perf_counter() - t0 >= seconds or n >= 50:
                break
        return (time.perf_counter() - t0) / n, n

    dt, n = timed(fn, args.cpu_seconds)
    # BASELINE config 1 exactly (configs[0]: RRDB nb 11 pixel-loss-only, 32 -> 128, batch 2: the reference's own CPU
    # case; pl_generator_pre_training.py:18-33), a few seconds of it
    p1 = {k: v.float() for k, v in gen_params(11, torch.float32).items()}
    opt1 = ref.AdamWState(p1, list(p1.keys()), lr=1e-4, total_steps=1000)
    bt1 = ref.synthetic_batch(2, 128)
    dt1, n1 = timed(lambda: ref.pretrain_step(p1, opt1, bt1, 11), max(3.0, args.cpu_seconds / 3))
    return {"value": round(b * hr * hr / 1e6 / dt, 5), "unit": "HR MPix/s", "cores": threads, "kind": "port",
            "sample": f"oracle {what}, fp32 PyTorch-CPU eager, batch {b}, {hr // 4}->{hr}, nb={args.nb}, "
                      f"{n} steps ({dt * 1e3:.0f} ms/step)",
            "cpu_model": info["cpu_model"], "affinity_cores": info["affinity_cores"],
            "cgroup_quota_cores": info["cgroup_quota_cores"],
            "config1": {"value": round(2 * 128 * 128 / 1e6 / dt1, 5), "unit": "HR MPix/s", "ms_per_step": round(dt1 * 1e3, 1),
                        "sample": f"oracle L1-pretrain step (BASELINE config 1: nb 11, batch 2, 32->128), fp32 PyTorch-CPU "
                                  f"eager, {n1} steps", "cores": threads, "kind": "port"}}


def run_infer(args, world, rank, dev):
    """BASELINE config 5: one whole CRU-TS grid (LR 720x360 -> HR 2880x1440) per step, forward only, one replica
    per GPU (the path does not shard within a grid: `scaling` weak, every rank infers its own grid)."""
    from climsr_amd import ops
    from climsr_amd.core.init import init_state, spec_from_shapes

    H, W = args.grid_h, args.grid_w
    if args.model == "rcan":
        from climsr_amd.models.rcan import RCAN

        net = RCAN(n_resgroups=10, n_resblocks=20, n_feats=64, reduction=16, scaling_factor=4, in_channels=3, out_channels=1)
        desc = "RCAN 10 groups x 20 RCABs, nf64, x4 (conf/generator/rcan.yaml)"
    else:
        from climsr_amd.models.esrgan import ESRGANGenerator

        net = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=args.nb, gc=16, scale_factor=4)
        desc = f"ESRGAN nf64 nb{args.nb} gc16 x4"
    st = init_state(spec_from_shapes({k: tuple(v.shape) for k, v in net.state_dict().items()}))
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    net = net.to(dev).eval()
    gen = torch.Generator(device="cpu").manual_seed(42 + rank)
    hh, ww = 4 * H, 4 * W
    t = torch.rand((1, 1, hh, ww), generator=gen) * 2 - 1
    e = torch.rand((1, 1, hh, ww), generator=gen) * 2 - 1
    m = (torch.rand((1, 1, hh, ww), generator=gen) < 0.7).float()
    lr = torch.cat([t, e, m], 1)[:, :, ::4, ::4].contiguous().to(dev)
    e, m = e.to(dev), m.to(dev)
    out = {}

    def fwd():
        out["sr"] = net(lr, e, m)

    with torch.no_grad():
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            fwd()
            fwd()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        run = fwd
        if not args.no_graph:
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                fwd()
            run = gr.replay
        for _ in range(args.warmup):
            run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            run()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if world > 1:
            tt = torch.tensor([elapsed], device=dev, dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            elapsed = float(tt.item())
        ms = elapsed / args.steps * 1e3
        mpix = world * hh * ww / 1e6 / (elapsed / args.steps)
        roof, kern = None, {}
        if not args.no_kernel_timing:
            timer = KernelTimer()
            ops.PROFILER = timer
            fwd()
            ops.PROFILER = None
            agg = timer.summary()
            name, (cnt, tot_ms, flops, nbytes) = max(agg.items(), key=lambda kv: kv[1][1])
            r = roofline_entry(name, cnt, tot_ms, flops, nbytes, timer.graph_us(name))
            roof = {"bound": r["bound"], "achieved": r["achieved"], "peak": r["peak"], "unit": r["unit"], "frac": r["frac"],
                    "traffic": None}
            roof.update({k: v for k, v in r.items() if k not in roof})
            tb, src = pmc_traffic(name, f"infer_{args.model}")
            if tb is None:
                roof["traffic_note"] = src
            else:
                roof.update(traffic=round(tb / 1e6, 2), traffic_unit="MB/launch", traffic_source=src,
                            traffic_over_algorithmic=round(tb / max(1, r["bytes_per_launch"]), 2))
            kern = {k: {"launches": v[0], "ms_total": round(v[1], 3), "tflops": round(v[2] / (v[1] / 1e3) / 1e12, 1),
                        "gbs": round(v[3] / (v[1] / 1e3) / 1e9, 1) if v[3] else None}
                    for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])}
            flop_fwd = sum(v[2] for v in agg.values())
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline_infer(args, {k: v.detach().cpu().float() for k, v in net.state_dict().items()})
    if rank == 0:
        res = {
            "metric": "HR MPix/s whole-grid inference (config 5: 720x360 -> 2880x1440, 4x SR)",
            "value": round(mpix, 3), "unit": "HR MPix/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic grid (seed 42+rank: U(-1,1) temp/elev, Bernoulli(0.7) mask, LR = HR[::4,::4]); deterministic init",
            "config": {"workload": f"config 5: whole-grid inference, LR {W}x{H} -> HR {ww}x{hh}, one grid per GPU per step",
                       "model": desc, "batch": 1, "parallelism": f"replicas{world}", "hip_graph": not args.no_graph,
                       "mode": "infer"},
            "pmc_summary": (roof or {}).get("traffic_source") or (roof or {}).get("traffic_note"),
            "roofline": roof,
            "step_mfma": ({"algorithmic_tflop_per_step": round(flop_fwd / 1e12, 3),
                           "achieved_tflops": round(flop_fwd / (ms / 1e3) / 1e12, 1),
                           "frac": round(flop_fwd / (ms / 1e3) / 1e12 / PEAK_BF16_TFLOPS, 4)} if roof else None),
            "cpu_baseline": cpu,
            "kernels": kern,
        }
        print(json.dumps(res))
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline_infer(args, state):
    """Oracle fp32 PyTorch-CPU forward of the same network on a bounded crop of the grid (LR 45x90)."""
    from oracle import climsr_ref as ref

    threads = cpu_info()["threads"]
    torch.set_num_threads(threads)
    h, w = 45, 90
    g = torch.Generator().manual_seed(7)
    x = torch.rand((1, 3, h, w), generator=g)
    e = torch.rand((1, 1, 4 * h, 4 * w), generator=g)
    m = torch.rand((1, 1, 4 * h, 4 * w), generator=g)
    if args.model == "rcan":
        fn = lambda: ref.rcan_forward(state, x, e, m, 10, 20, 4)  # noqa: E731
    else:
        fn = lambda: ref.generator_forward(state, x, e, m, args.nb)  # noqa: E731
    with torch.no_grad():
        fn()
        t0 = time.perf_counter()
        n = 0
        while True:
            fn()
            n += 1
            if time.perf_counter() - t0 >= args.cpu_seconds or n >= 20:
                break
    dt = (time.perf_counter() - t0) / n
    return {"value": round(16 * h * w / 1e6 / dt, 5), "unit": "HR MPix/s", "cores": threads, "kind": "port",
            "sample": f"oracle {args.model} forward (fp32 PyTorch-CPU), LR {w}x{h} crop of the grid, {n} runs ({dt * 1e3:.0f} ms each)"}


def build_train(args, mode, world, dev):
    """Models, optimisers, synthetic batch and the step segments of one training workload."""
    from climsr_amd.core.init import init_state, spec_from_shapes
    from climsr_amd.core.optim import GraphedAdamW
    from climsr_amd.losses.l1 import l1_loss
    from climsr_amd.models.esrgan import ESRGANGenerator

    rank = int(os.environ.get("RANK", "0"))
    B, lr_size = args.batch, args.lr_size
    hr = 4 * lr_size
    total_steps = max(1000, 2 * (args.warmup + args.steps + args.median_steps) + 10)
    g = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=args.nb, gc=16, scale_factor=4)
    st = init_state(spec_from_shapes({k: tuple(v.shape) for k, v in g.state_dict().items()}))
    g.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    g = g.to(dev)
    task = d = opt_d = None
    if mode == "gan":
        from climsr_amd.task.pl_gan import GANLightningModule

        task = GANLightningModule(generator=g, discriminator={"_target_": "climsr_amd.models.rfb_esrgan.RFBESRGANDiscriminator",
                                                              "in_channels": 1})
        d = task.discriminator
        dst = init_state(spec_from_shapes({k: tuple(v.shape) for k, v in d.state_dict().items()},
                                          [n_ for n_, m_ in d.named_modules() if isinstance(m_, torch.nn.BatchNorm2d)]))
        d.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in dst.items()})
        task = task.to(dev)
        g, d = task.generator, task.discriminator
        opt_d = GraphedAdamW(d, lr=1e-4, total_steps=total_steps, weight_decay=1e-4)
    opt_g = GraphedAdamW(g, lr=1e-4, total_steps=total_steps, weight_decay=1e-4)

    gen = torch.Generator(device="cpu").manual_seed(42 + rank)
    t = torch.rand((B, 1, hr, hr), generator=gen) * 2 - 1
    e = torch.rand((B, 1, hr, hr), generator=gen) * 2 - 1
    m = (torch.rand((B, 1, hr, hr), generator=gen) < 0.7).float()
    lr = torch.cat([t, e, m], 1)[:, :, ::4, ::4].contiguous()
    batch = {k: v.to(dev) for k, v in {"lr": lr, "hr": t, "elevation": e, "mask": m}.items()}
    loss_buf = torch.zeros(2, device=dev)

    def toggle(net_on):
        for net in (g, d):
            for p in net.parameters():
                p.requires_grad_(net is net_on)

    if mode == "pretrain":
        def seg_g():
            for p in g.parameters():
                p.grad = None  # zero_grad(set_to_none=True): backward overwrites the flat grad buffer
            sr = g(batch["lr"], batch["elevation"], batch["mask"])
            loss = l1_loss(sr, batch["hr"])
            loss.backward()
            loss_buf[0].copy_(loss.detach())

        segments = [(seg_g, g), (opt_g.step, None)]
    else:
        def seg_g():  # optimizer_idx 0 (pl_gan.py:63-79): D frozen
            toggle(g)
            for p in g.parameters():
                p.grad = None
            _hr, sr = task.common_step(batch)
            _perc, _adv, _pix, lg = task.loss_g(batch["hr"], sr)
            lg.backward()
            loss_buf[0].copy_(lg.detach())

        def seg_d():  # AdamW_G, then optimizer_idx 1 (pl_gan.py:81-97): fresh G forward, D update
            opt_g.step()
            toggle(d)
            for p in d.parameters():
                p.grad = None
            _hr, sr = task.common_step(batch)
            ld = task.loss_d(batch["hr"], sr)
            ld.backward()
            loss_buf[1].copy_(ld.detach())

        segments = [(seg_g, g), (seg_d, d), (opt_d.step, None)]
    return dict(g=g, d=d, segments=segments, loss_buf=loss_buf, B=B, hr=hr, lr_size=lr_size, batch=batch)


def make_runner(w, world, dev, use_graph=True):
    """The step of a workload from ``build_train`` as the bench times it: two eager warm-up steps, then every segment
    captured as hipGraph(s) and ``run()`` replaying them, with the DDP gradient average of each network after its
    segment (overlapped with the backward for N > 1).  ``tests/test_gpu_timed_step.py`` drives this same function and
    compares its steps with the eager ``Trainer`` + ``core.optim.AdamW`` + torch ``OneCycleLR`` path.
    Returns dict(run, step_eager, graphs, overlap)."""
    from climsr_amd.core.ddp import GradAllReducer, OverlappedGradAllReducer, broadcast_module

    g, d, segments = w["g"], w["d"], w["segments"]
    nets = [n_ for n_ in (g, d) if n_ is not None]

    reducers = {}
    # Overlapped DDP (default for N > 1; CLIMSR_DDP_OVERLAP=0 restores the all-reduce after the backward;
    # CLIMSR_DDP_OVERLAP_TEST=1 runs the overlapped structure at N = 1 with no-op reductions, to check it):
    # the backward reports finished gradient slices through the modules' grad-ready hooks, each slice is
    # all-reduced asynchronously while the rest of the backward runs, and the hipGraph of a segment is split
    # at those points so the replay can launch them in the same places.
    overlap = (world > 1 and os.environ.get("CLIMSR_DDP_OVERLAP", "1") != "0") or os.environ.get("CLIMSR_DDP_OVERLAP_TEST") == "1"
    ov = {id(n_): OverlappedGradAllReducer(n_) for n_ in nets} if overlap else {}
    # backward calls per step that accumulate into a network's gradients: D gets two in loss_d (real and
    # fake, pl_gan.py:51-61); G one (pass 0)
    hook_calls = {id(d): 2} if d is not None else {}

    def set_hook(net, fn):
        if net is d:
            net.set_grad_ready_hook(fn, calls_per_step=hook_calls[id(d)])
        else:
            net.set_grad_ready_hook(fn)

    for net in nets:
        set_hook(net, ov[id(net)].ready if overlap else None)

    def allreduce(net):
        if overlap:
            ov[id(net)].finish()
        elif world > 1:  # DDP gradient average of the flat fp32 buffer over RCCL/xGMI, 256 MB buckets
            if id(net) not in reducers:
                reducers[id(net)] = GradAllReducer(net)
            reducers[id(net)]()

    if world > 1:
        for net in nets:
            broadcast_module(net)

    def step_eager():
        for fn, net in segments:
            fn()
            if net is not None:
                allreduce(net)

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            step_eager()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graphs = []
    if use_graph:
        pool = torch.cuda.graph_pool_handle()
        cap = torch.cuda.Stream()
        for fn, net in segments:
            # one segment = one or more graphs: with the overlapped DDP the grad-ready hook (it runs on the
            # autograd thread, on the capture stream) ends the current capture and begins the next one
            # ("relaxed" capture: begin and end may be on different threads)
            subs, los = [torch.cuda.CUDAGraph()], []

            def split(lo, subs=subs, los=los):
                subs[-1].capture_end()
                los.append(lo)
                subs.append(torch.cuda.CUDAGraph())
                subs[-1].capture_begin(pool=pool, capture_error_mode="relaxed")

            if net is not None and overlap:
                set_hook(net, split)
            torch.cuda.synchronize()
            cap.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(cap):
                subs[0].capture_begin(pool=pool, capture_error_mode="relaxed")
                fn()
                subs[-1].capture_end()
            torch.cuda.current_stream().wait_stream(cap)
            if net is not None and overlap:
                set_hook(net, ov[id(net)].ready)
            graphs.append((list(zip(subs, los + [None])), net))

        def run():
            for subs, net in graphs:
                for gr, lo in subs:
                    gr.replay()
                    if lo is not None:
                        ov[id(net)].ready(lo)  # this slice's all-reduce overlaps the next graph
                if net is not None:
                    allreduce(net)
    else:
        run = step_eager
    return dict(run=run, step_eager=step_eager, graphs=graphs, overlap=overlap)


def measure_train(args, mode, world, rank, dev, kernel_timing=True):
    """Capture the step of ``mode`` (hipGraph segments), run W warm-up steps, time exactly K steps between a barrier +
    synchronize on both sides (max over ranks), then ``median_steps`` more steps one HIP-event pair each."""
    from climsr_amd import ops

    w = build_train(args, mode, world, dev)
    loss_buf, B, hr = w["loss_buf"], w["B"], w["hr"]
    use_graph = not args.no_graph
    rn = make_runner(w, world, dev, use_graph)
    run, step_eager, graphs, overlap = rn["run"], rn["step_eager"], rn["graphs"], rn["overlap"]

    def barrier_sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(v):
        if world == 1:
            return v
        tt = torch.tensor([v], device=dev, dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        return float(tt.item())

    for _ in range(args.warmup):
        run()
    barrier_sync()
    t0 = time.perf_counter()
    for i in range(args.steps):
        run()
        if rank == 0 and args.steps >= 20 and (i + 1) % max(1, args.steps // 4) == 0:
            print(f"[bench] {mode} step {i + 1}/{args.steps}", file=sys.stderr, flush=True)
    barrier_sync()
    elapsed = max_over_ranks(time.perf_counter() - t0)
    ms = elapsed / args.steps * 1e3
    mpix = world * B * hr * hr / 1e6 / (elapsed / args.steps)

    med = None
    if args.median_steps > 0:  # per-step HIP events on the replay stream, back to back
        evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.median_steps + 1)]
        evs[0].record()
        for i in range(args.median_steps):
            run()
            evs[i + 1].record()
        torch.cuda.synchronize()
        per = [evs[i].elapsed_time(evs[i + 1]) for i in range(args.median_steps)]
        med_ms = max_over_ranks(statistics.median(per))
        med = {"steps": args.median_steps, "after_warmup_steps": args.warmup + args.steps, "ms_per_step": round(med_ms, 3),
               "value": round(world * B * hr * hr / 1e6 / (med_ms / 1e3), 3), "min_ms": round(min(per), 3),
               "max_ms": round(max(per), 3), "source": "per-step HIP events (median over steps, max over ranks)"}
    loss_val = [float(v) for v in loss_buf.cpu()]

    flop_px = 3 * G_FWD_FLOP_PER_PX if mode == "pretrain" else GAN_FLOP_PER_PX
    flop_step = flop_px * B * hr * hr  # SURVEY §8d algorithmic FLOPs per HR pixel
    step_tflops = flop_step / (ms / 1e3) / 1e12
    rec = {"mode": mode, "ms": ms, "mpix": mpix, "median": med, "loss_last": [round(v, 6) for v in loss_val],
           "use_graph": use_graph, "overlap": overlap, "graph_segments": [len(sg) for sg, _n in graphs] if use_graph else None,
           "B": B, "hr": hr, "lr_size": w["lr_size"],
           "step_mfma": {"algorithmic_tflop_per_step": round(flop_step / 1e12, 3), "achieved_tflops": round(step_tflops, 1),
                         "frac": round(step_tflops / PEAK_BF16_TFLOPS, 4)}}
    if kernel_timing:
        rec.update(kernel_profile(step_eager, mode, ops))
    return rec


def kernel_profile(step, mode, ops):
    """Every native launch of one eager step timed with HIP events on its stream (ops.PROFILER sees each C-ABI
    call: convs, BN, linear, pooling, losses, AdamW, weight packing); the launch with the largest total time
    names the roofline kernel, whose average launch time is re-measured from a hipGraph replay of its launches.
    ``unattributed_ms`` = eager step time - sum of the timed launches (torch fills / copies, launch gaps)."""
    timer = KernelTimer()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ops.PROFILER = timer
    try:
        s.record()
        step()
        e.record()
    finally:
        ops.PROFILER = None
    torch.cuda.synchronize()
    eager_ms = s.elapsed_time(e)
    agg = timer.summary()
    name, (cnt, tot_ms, flops, nbytes) = max(agg.items(), key=lambda kv: kv[1][1])
    r = roofline_entry(name, cnt, tot_ms, flops, nbytes, timer.graph_us(name))
    roof = {"bound": r["bound"], "achieved": r["achieved"], "peak": r["peak"], "unit": r["unit"], "frac": r["frac"], "traffic": None}
    roof.update({k: v for k, v in r.items() if k not in roof})
    tb, src = pmc_traffic(name, mode)
    if tb is None:
        roof["traffic_note"] = src
    else:  # HBM bytes per launch (PMC) and the bandwidth they imply at the measured launch time
        roof.update(traffic=round(tb / 1e6, 2), traffic_unit="MB/launch", traffic_source=src,
                    traffic_gbs=round(tb / (r["avg_launch_us"] / 1e6) / 1e9, 1),
                    traffic_over_algorithmic=round(tb / max(1, r["bytes_per_launch"]), 2))
    timed = sum(v[1] for v in agg.values())
    kern = {k: {"launches": v[0], "ms_total": round(v[1], 3),
                "tflops": round(v[2] / (v[1] / 1e3) / 1e12, 1) if v[2] else None,
                "gbs": round(v[3] / (v[1] / 1e3) / 1e9, 1) if v[3] else None}
            for k, v in sorted(agg.items(), key=lambda kv: -kv[1][1])}
    if os.environ.get("CLIMSR_BENCH_DETAIL"):
        print(json.dumps(timer.by_tag(top=60), indent=0), file=sys.stderr)
    return {"roofline": roof, "kernels": kern,
            "profile": {"eager_step_ms": round(eager_ms, 3), "timed_launch_ms": round(timed, 3),
                        "unattributed_ms": round(eager_ms - timed, 3), "native_launches": sum(v[0] for v in agg.values())}}


WORKLOAD = {"pretrain": "config 2: RRDB generator L1 pre-training step (fwd+L1+bwd+AdamW+OneCycleLR)",
            "gan": "config 3: full ESRGAN GAN step (pl_gan.py:63-97: G pass = G fwd + D(hr), D(sr) + VGG19 perceptual + "
                   "L1 + G bwd + AdamW_G; D pass = G fwd + D(hr), D(sr) + D bwd + AdamW_D; OneCycleLR x2)"}


def main(argv=None):
    args = parse(argv)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # the driver's `bench.py --gpus N` without a launcher: fan out N ranks ourselves (no GPU touched here)
        return launch(args.gpus, [sys.executable, "-u", os.path.abspath(__file__)] + (sys.argv[1:] if argv is None else argv))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    rccl_world = dist.get_world_size() if dist.is_initialized() else 1

    import climsr_amd  # noqa: F401

    if args.mode == "infer":
        return run_infer(args, world, rank, dev)
    rec = measure_train(args, args.mode, world, rank, dev, kernel_timing=not args.no_kernel_timing)
    sub = None
    if args.mode == "gan" and not args.no_config2:
        r2 = measure_train(args, "pretrain", world, rank, dev, kernel_timing=not args.no_kernel_timing)
        sub = {"metric": "HR MPix/s per training step (4x SR, 64->256 tiles)", "workload": WORKLOAD["pretrain"],
               "value": round(r2["mpix"], 3), "ms_per_step": round(r2["ms"], 3), "median": r2["median"],
               "step_mfma": r2["step_mfma"], "roofline": r2.get("roofline"), "loss_last": r2["loss_last"]}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args, rec["hr"], args.mode)

    if rank == 0:
        out = {
            "metric": "HR MPix/s per training step (4x SR, 64->256 tiles)",
            "value": round(rec["mpix"], 3), "unit": "HR MPix/s", "n_gpus": world, "rccl_world": rccl_world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(rec["ms"], 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16",
            "data": "synthetic (seed 42+rank: U(-1,1) temp/elev, Bernoulli(0.7) mask, LR = HR[::4,::4]); deterministic init",
            "config": {"workload": WORKLOAD[args.mode], "generator": f"ESRGAN nf64 nb{args.nb} gc16 x4",
                       "discriminator": "RFBESRGANDiscriminator" if args.mode == "gan" else None,
                       "global_batch": world * rec["B"], "per_gpu_batch": rec["B"], "lr_tile": rec["lr_size"], "hr_tile": rec["hr"],
                       "parallelism": f"dp{world}", "hip_graph": rec["use_graph"], "ddp_overlap": rec["overlap"],
                       "graph_segments": rec["graph_segments"], "mode": args.mode},
            "median": rec["median"],
            # the PMC summary roofline.traffic comes from (matched on the library sha256), or why there is none
            "pmc_summary": (rec.get("roofline") or {}).get("traffic_source") or (rec.get("roofline") or {}).get("traffic_note"),
            "roofline": rec.get("roofline"),
            "step_mfma": rec["step_mfma"],
            "cpu_baseline": cpu,
            "loss_last": rec["loss_last"],
            "config2": sub,
            "profile": rec.get("profile"),
            "kernels": rec.get("kernels", {}),
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
