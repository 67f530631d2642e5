"""A/B of two launch fusions at the GAN step's shapes (GPU box only), one JSON line:
  - the discriminator stem (features.0 + features.2 in one launch, csrc/stem.hip) vs per layer: D forward + backward
    of 32 images 1 x 256^2 (rfb_esrgan.py engine flag fuse_stem);
  - VGG19 conv + ReLU + 2x2 max pool in one launch vs conv then pool: the perceptual features of 64 images 256^2
    (losses/perceptual.py flag fuse_pool).
    python tools/perf_stem.py <label>"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import _lib  # noqa: E402
from climsr_amd.losses.perceptual import PerceptualLoss  # noqa: E402
from climsr_amd.models.rfb_esrgan import RFBESRGANDiscriminator  # noqa: E402


def evt_time(fn, reps=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / reps * 1e3, 1)  # us


dev = "cuda"
torch.manual_seed(0)
res = {"label": sys.argv[1] if len(sys.argv) > 1 else "", "lib": _lib.LIB_PATH}
d = RFBESRGANDiscriminator(1).to(dev)
x = torch.randn(32, 1, 256, 256, device=dev, requires_grad=True)


def d_step():
    d.zero_grad(set_to_none=True)
    d(x).sum().backward()


for fuse in (True, False, True, False):
    d.engine().fuse_stem = fuse
    res.setdefault(f"d_fwd_bwd_stem{int(fuse)}_us", []).append(evt_time(d_step))
del d, x
torch.cuda.empty_cache()
pl = PerceptualLoss().to(dev)
a = torch.rand(32, 1, 256, 256, device=dev)
b = torch.rand(32, 1, 256, 256, device=dev)
for fuse in (True, False, True, False):
    pl.fuse_pool = fuse
    res.setdefault(f"perceptual_pool{int(fuse)}_us", []).append(evt_time(lambda: pl(a, b), 5))
print(json.dumps(res), flush=True)
