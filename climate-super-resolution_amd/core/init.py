"""Deterministic, counter-seeded parameter initializer.

The reference initialises with torch's default ``kaiming_uniform_(a=sqrt(5))`` (bound
``1/sqrt(fan_in)``) drawn from the global torch RNG (``climsr/models/esrgan.py:22-26``,
``rfb_esrgan.py:28-61``), which makes weights depend on construction order.  Here every tensor
is drawn from its own PCG64 stream seeded by ``crc32(state_dict key) ^ seed``, so the same
weights can be regenerated anywhere (oracle, golden fixtures, GPU box, every DDP rank) from
the key alone without shipping checkpoints.  Bounds follow torch's defaults:

* conv / linear weight and bias: U(-1/sqrt(fan_in), 1/sqrt(fan_in))
* BatchNorm: weight 1, bias 0, running_mean 0, running_var 1, num_batches_tracked 0
* ``gain`` > 1 scales the bound (used for the random-weight VGG19 so activations keep O(1)
  scale through 16 ReLU convs; the ImageNet weights of ``perceptual.py:15`` cannot be fetched
  offline).
"""
from __future__ import annotations

import math
import zlib
from typing import Dict, Iterable, Tuple

import numpy as np

DEFAULT_SEED = 42  # conf/training/default.yaml:5


def _stream(key: str, seed: int) -> np.random.Generator:
    s = (zlib.crc32(key.encode("utf-8")) ^ ((seed * 0x9E3779B1) & 0xFFFFFFFF)) & 0xFFFFFFFF
    return np.random.Generator(np.random.PCG64(s))


def det_uniform(key: str, shape: Tuple[int, ...], bound: float, seed: int = DEFAULT_SEED) -> np.ndarray:
    return _stream(key, seed).uniform(-bound, bound, size=shape).astype(np.float32)


def init_tensor(key: str, shape: Tuple[int, ...], fan_in: int, seed: int = DEFAULT_SEED, gain: float = 1.0) -> np.ndarray:
    if key.endswith("running_var"):
        return np.ones(shape, np.float32)
    if key.endswith("running_mean"):
        return np.zeros(shape, np.float32)
    if key.endswith("num_batches_tracked"):
        return np.zeros(shape, np.int64)
    bound = gain / math.sqrt(max(fan_in, 1))
    return det_uniform(key, shape, bound, seed)


def init_state(spec: Iterable[Tuple[str, Tuple[int, ...], int, str]], seed: int = DEFAULT_SEED, gain: float = 1.0) -> Dict[str, np.ndarray]:
    """spec rows: (key, shape, fan_in, kind) with kind in {"conv", "bn_w", "bn_b", "buf"}."""
    out = {}
    for key, shape, fan_in, kind in spec:
        if kind == "bn_w":
            out[key] = np.ones(shape, np.float32)
        elif kind == "bn_b":
            out[key] = np.zeros(shape, np.float32)
        else:
            out[key] = init_tensor(key, shape, fan_in, seed, gain)
    return out


def spec_from_shapes(shapes: Dict[str, Tuple[int, ...]], bn_prefixes: Iterable[str] = ()) -> list:
    """Build an init spec from ``{state_dict key: shape}``; fan_in is inferred from the weight
    shape of the same layer (bias uses its layer's weight fan_in, as torch does)."""
    bn_prefixes = set(bn_prefixes)
    rows = []
    for key, shape in shapes.items():
        layer, _, leaf = key.rpartition(".")
        if layer in bn_prefixes:
            kind = {"weight": "bn_w", "bias": "bn_b"}.get(leaf, "buf")
            rows.append((key, tuple(shape), 1, kind))
            continue
        wshape = shapes.get(layer + ".weight", shape)
        fan_in = int(np.prod(wshape[1:])) if len(wshape) > 1 else int(wshape[0])
        rows.append((key, tuple(shape), fan_in, "conv"))
    return rows
