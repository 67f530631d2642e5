"""Shared test helpers: deterministic parameter dicts for the oracle, keyed like the reference."""
import numpy as np
import torch

from climsr_amd.core.init import init_state, spec_from_shapes
from oracle import climsr_ref as ref


def gen_params(nb=1, dtype=torch.float64, in_channels=3):
    shapes = ref.generator_shapes(in_channels=in_channels, nb=nb)
    st = init_state(spec_from_shapes(shapes))
    return {k: torch.from_numpy(np.asarray(v)).to(dtype) for k, v in st.items()}


def rfb_d_params(dtype=torch.float64):
    shapes = ref.rfb_discriminator_shapes()
    st = init_state(spec_from_shapes(shapes, ref.rfb_bn_prefixes()))
    return {k: (torch.from_numpy(np.asarray(v)).to(dtype) if np.asarray(v).dtype != np.int64 else torch.from_numpy(np.asarray(v)))
            for k, v in st.items()}


def plain_d_params(dtype=torch.float64):
    shapes = ref.plain_discriminator_shapes()
    st = init_state(spec_from_shapes(shapes, ref.plain_bn_prefixes()))
    return {k: (torch.from_numpy(np.asarray(v)).to(dtype) if np.asarray(v).dtype != np.int64 else torch.from_numpy(np.asarray(v)))
            for k, v in st.items()}


def vgg_params(dtype=torch.float64):
    shapes = ref.vgg19_shapes()
    st = init_state(spec_from_shapes(shapes), gain=float(np.sqrt(6.0)))
    return {k: torch.from_numpy(np.asarray(v)).to(dtype) for k, v in st.items()}


def psnr(a, b, data_range=None):
    a = a.double()
    b = b.double()
    if data_range is None:
        data_range = float(b.max() - b.min())
    mse = float(((a - b) ** 2).mean())
    return float("inf") if mse == 0 else 10 * np.log10(data_range ** 2 / mse)
