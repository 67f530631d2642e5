"""Time the discriminator stem (features.0 + features.2 in one launch, csrc/stem.hip, rfb_esrgan.py:28-31) at the GAN
step's shape (B=32, 1 x 256^2) under one libclimsr_hip.so (CLIMSR_HIP_LIB selects an A/B build): the keep form (a0
written for the backward, BatchNorm partials) and the no-keep form, hipGraph replay.  One JSON line.
    CLIMSR_HIP_LIB=... python tools/perf_dstem.py <label>"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import climsr_amd  # noqa: E402,F401
from climsr_amd import _lib, ops  # noqa: E402
from climsr_amd.models.rfb_esrgan import RFBESRGANDiscriminator  # noqa: E402
from tools.perf_conv_timing import timeit  # noqa: E402

dev, n, h, w = "cuda", 32, 256, 256
res = {"label": sys.argv[1] if len(sys.argv) > 1 else "", "lib": _lib.LIB_PATH}
torch.manual_seed(0)
d = RFBESRGANDiscriminator(1).to(dev)
eng = d.engine()
eng.ensure_packed()
(c0, _b0, _p0), (_c1, _b1, p1) = eng.layers[0], eng.layers[1]
x8 = torch.zeros((n, h, w, 8), dtype=torch.bfloat16, device=dev)
x8[..., 0] = torch.rand((n, h, w), device=dev).to(torch.bfloat16)
a0 = torch.empty((n, h, w, 64), dtype=torch.bfloat16, device=dev)
z = torch.empty((n, h // 2, w // 2, 64), dtype=torch.bfloat16, device=dev)
parts = ops.d_stem_s2_bn_parts(n, h, w)
part = torch.empty((parts * 2 * 64,), dtype=torch.float64, device=dev)
for rep in range(2):
    res.setdefault("stem_keep_us", []).append(round(timeit(lambda: ops.d_stem_s2(x8, 8, c0.weight, p1, a0, z, part, n, h, w), 10), 2))
    res.setdefault("stem_nokeep_us", []).append(round(timeit(lambda: ops.d_stem_s2(x8, 8, c0.weight, p1, None, z, part, n, h, w), 10), 2))
print(json.dumps(res), flush=True)
