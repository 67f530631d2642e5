"""Generate tests/golden/rcan.npz by running the REFERENCE's own RCAN (climsr/models/rcan.py) on CPU in fp64.

Run in the build container (needs /root/reference; never on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_rcan_golden.py

Weights: the deterministic initializer of ``climsr_amd.core.init`` keyed by state_dict name (the same one the
GPU test loads into the native RCAN).  Inputs: the seeded synthetic tile batch of make_golden.py.
"""
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402
import torch  # noqa: E402

from climsr.models.rcan import RCAN  # noqa: E402  (reference)

from climsr_amd.core.init import init_state, spec_from_shapes  # noqa: E402

torch.set_num_threads(8)
CONFIGS = {  # name: (n_resgroups, n_resblocks, scaling_factor, batch, lr size)
    "rcan_g2b2_x4": (2, 2, 4, 2, 16),
    "rcan_g2b2_x2": (2, 2, 2, 1, 24),
    "rcan_g10b20_x4": (10, 20, 4, 1, 16),
}


def batch(b, hr, seed=42, scale=4):
    g = torch.Generator().manual_seed(seed)
    t = torch.rand((b, 1, hr, hr), generator=g) * 2 - 1
    e = torch.rand((b, 1, hr, hr), generator=g) * 2 - 1
    m = (torch.rand((b, 1, hr, hr), generator=g) < 0.7).float()
    lr = torch.cat([t, e, m], 1)[:, :, ::scale, ::scale].contiguous()
    return lr, e, m


out = {}
for name, (ng, nb, sf, b, lr_size) in CONFIGS.items():
    net = RCAN(n_resgroups=ng, n_resblocks=nb, n_feats=64, reduction=16, scaling_factor=sf, in_channels=3, out_channels=1)
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    st = init_state(spec_from_shapes(shapes))
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()}, strict=True)
    net = net.double().eval()
    lr, e, m = batch(b, lr_size * sf, scale=sf)
    with torch.no_grad():
        sr = net(lr.double(), e.double(), m.double())
    out[name] = sr.numpy()
    print(name, tuple(sr.shape), float(sr.std()))
np.savez_compressed(os.path.join(HERE, "rcan.npz"), **out)
