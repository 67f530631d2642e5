"""Generate tests/golden/rcan.npz by running the REFERENCE's own RCAN (climsr/models/rcan.py) on CPU in fp64, and
tests/golden/rcan_train.json: the reference RCAN's L1 pre-training gradients (the task's loss, task.py:141 nn.L1Loss on
the generator output vs hr; rcan_pre_training.yaml) as per-tensor (sum, L2 norm) checksums, fp64.

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

import json  # noqa: E402

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

# training: L1(sr, hr) gradients of the reference module in fp64 (hr = the full-resolution temperature tile of batch())
TRAIN = {"rcan_g2b2_x4": (2, 2, 4, 2, 16), "rcan_g1b2_x2": (1, 2, 2, 2, 12), "rcan_g1b1_x3": (1, 1, 3, 1, 10)}
rec = {}
for name, (ng, nb, sf, b, lr_size) in TRAIN.items():
    net = RCAN(n_resgroups=ng, n_resblocks=nb, n_feats=64, reduction=16, scaling_factor=sf, in_channels=3, out_channels=1)
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    st = init_state(spec_from_shapes(shapes))
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()}, strict=True)
    net = net.double().train()
    hrs = lr_size * sf
    g = torch.Generator().manual_seed(7)
    hr = torch.rand((b, 1, hrs, hrs), generator=g, dtype=torch.float64) * 2 - 1
    e = torch.rand((b, 1, hrs, hrs), generator=g, dtype=torch.float64) * 2 - 1
    m = (torch.rand((b, 1, hrs, hrs), generator=g) < 0.7).double()
    lr = torch.cat([hr, e, m], 1)[:, :, ::sf, ::sf].contiguous()
    net.zero_grad()
    loss = torch.nn.L1Loss()(net(lr, e, m), hr)
    loss.backward()
    rec[name] = {"loss": float(loss), "grads": {k: [float(p.grad.double().sum()), float(p.grad.double().norm())]
                                                for k, p in net.named_parameters()}}
    print(name, "loss", float(loss))
with open(os.path.join(HERE, "rcan_train.json"), "w") as f:
    json.dump(rec, f)
