"""Batch-level, on-device ``ClimateDataset``.

The reference builds every training sample on the CPU inside DataLoader workers
(climsr/data/sr/climate_dataset.py:220-275): read the tile, MinMax-normalise it with the per-file or
global min/max (or z-score it), NaN -> 0, derive the land mask, randomly v-flip / h-flip / rot90
(:144-189), decimate to LR with INTER_NEAREST and concatenate ``[lr, elevation_lr, mask_lr]``
(:95-118).  ``DeviceTilePipeline`` does that for a whole batch of raw tiles already resident in HBM
with two launches of ``libclimsr_hip.so`` (``climsr_tile_minmax_f32`` for the elevation's own
nanmin/nanmax, ``climsr_tile_prepare`` for everything else), so host workers only move raw float32
tiles.  The random draws are made on the host with ``random.Random`` in the reference's order
(v-flip, h-flip, rotation, then ``randint(0, 3)``), so a seeded pipeline reproduces a seeded
reference worker's transform sequence exactly.

No CPU fallback: inputs must be CUDA tensors and the HIP library must load.
"""
from __future__ import annotations

import ctypes
import random
from dataclasses import dataclass
from typing import Dict, Mapping, Optional, Sequence, Tuple, Union

import torch
from torch import Tensor

from .. import _lib
from .._lib import TileDesc, check, ptr

ELEVATION_MISSING_INDICATOR = -32768.0  # climsr/consts/world_clim.py:24


@dataclass
class TransformsCfg:
    """climsr/core/config.py:53-56."""
    v_flip: bool = True
    h_flip: bool = True
    random_90_rotation: bool = True


def _cuda_f32(t: Tensor, name: str) -> Tensor:
    if not isinstance(t, Tensor) or not t.is_cuda:
        raise RuntimeError(f"DeviceTilePipeline: `{name}` must be a CUDA tensor (the pipeline runs in libclimsr_hip.so only)")
    if t.dtype != torch.float32:
        raise RuntimeError(f"DeviceTilePipeline: `{name}` must be float32 (raw tiles), got {t.dtype}")
    return t.contiguous()


class DeviceTilePipeline:
    """Turns raw tiles ``[n, h, w]`` (NaN = sea) + raw elevation into the reference's batch dict.

    Args mirror ``ClimateDataset.__init__`` (climate_dataset.py:23-40): ``generator_type``
    ("esrgan" | "srcnn" | ...), ``stage`` ("train" draws transforms; "val"/"test" add the
    ``elevation_lr``/``nearest``/``cubic``/``original_data``/``min``/``max`` items),
    ``scaling_factor``, ``normalize`` / ``standardize`` (+ ``standardize_stats`` mapping with
    ``hr_mean, hr_std, hr_nan_sub, elev_mean, elev_std, elev_nan_sub``), ``normalize_range``,
    ``use_elevation``, ``use_mask``, ``transforms_cfg``; ``seed`` seeds the host RNG of the draws.
    """

    def __init__(self, generator_type: str = "esrgan", stage: str = "train", scaling_factor: int = 4, normalize: bool = True,
                 standardize: bool = False, standardize_stats: Optional[Mapping[str, float]] = None,
                 normalize_range: Tuple[float, float] = (-1.0, 1.0), use_elevation: bool = True, use_mask: bool = True,
                 transforms_cfg: Optional[TransformsCfg] = None, seed: Optional[int] = None):
        self.generator_type = generator_type
        self.stage = stage
        self.scaling_factor = int(scaling_factor)
        self.normalize = normalize
        self.standardize = standardize
        if standardize and standardize_stats is None:
            raise ValueError("standardize=True needs standardize_stats (hr/elev mean, std, nan_sub)")
        self.standardize_stats = dict(standardize_stats or {})
        self.normalize_range = tuple(float(v) for v in normalize_range)
        self.use_elevation = use_elevation
        self.use_mask = use_mask
        self.transforms_cfg = transforms_cfg or TransformsCfg()
        self.rng = random.Random(seed)

    @property
    def method(self) -> int:
        return 1 if self.standardize else (0 if self.normalize else 2)

    def draw_transforms(self, n: int) -> list:
        """Per-sample codes (bit0 flipud, bit1 fliplr, bits2-3 rot90 k) drawn like climate_dataset.py:149-166."""
        cfg, codes = self.transforms_cfg, []
        for _ in range(n):
            c = 0
            if cfg.v_flip and self.rng.random() > 0.5:
                c |= 1
            if cfg.h_flip and self.rng.random() > 0.5:
                c |= 2
            if cfg.random_90_rotation and self.rng.random() > 0.5:
                c |= self.rng.randint(0, 3) << 2
            codes.append(c)
        return codes

    def __call__(self, hr_raw: Tensor, elevation_raw: Optional[Tensor] = None,
                 hr_min: Optional[Union[Tensor, Sequence[float]]] = None, hr_max: Optional[Union[Tensor, Sequence[float]]] = None,
                 transforms: Optional[Sequence[int]] = None) -> Dict[str, Tensor]:
        hr_raw = _cuda_f32(hr_raw, "hr_raw")
        if hr_raw.dim() == 4:
            hr_raw = hr_raw.reshape(hr_raw.shape[0], hr_raw.shape[2], hr_raw.shape[3])
        n, h, w = hr_raw.shape
        dev = hr_raw.device
        s = self.scaling_factor
        if h % s or w % s:
            raise ValueError(f"tile {h}x{w} is not a multiple of scaling_factor {s}")
        use_elev = bool(self.use_elevation)
        if use_elev:
            if elevation_raw is None:
                raise ValueError("use_elevation=True needs elevation_raw")
            elevation_raw = _cuda_f32(elevation_raw, "elevation_raw").reshape(n, h, w)
        method = self.method
        mn = mx = None
        if method == 0:
            if hr_min is None or hr_max is None:
                raise ValueError("min-max normalisation needs hr_min / hr_max (per-file or global stats)")
            mn = torch.as_tensor(hr_min, dtype=torch.float64).to(dev).reshape(n).contiguous()
            mx = torch.as_tensor(hr_max, dtype=torch.float64).to(dev).reshape(n).contiguous()
        train = self.stage == "train"
        xform = None
        if train:
            codes = list(transforms) if transforms is not None else self.draw_transforms(n)
            if len(codes) != n:
                raise ValueError("one transform code per tile")
            xform = torch.tensor(codes, dtype=torch.int32).pin_memory().to(dev, non_blocking=True)
        srcnn = self.generator_type == "srcnn"
        lr_c = 1 + int(use_elev) + int(self.use_mask)
        lh, lw = (h, w) if srcnn else (h // s, w // s)
        new = lambda *shape: torch.empty(shape, dtype=torch.float32, device=dev)  # noqa: E731
        out = {"lr": new(n, lr_c, lh, lw), "hr": new(n, 1, h, w), "mask": new(n, 1, h, w)}
        if use_elev:
            out["elevation"] = new(n, 1, h, w)
        if not train:
            out["nearest"] = new(n, 1, h, w)
            out["hr_lr"] = new(n, 1, h // s, w // s)
            if use_elev:
                out["elevation_lr"] = new(n, 1, h // s, w // s)
        elev_mm = None
        L = _lib.load()
        stream = _lib.stream_ptr(dev)
        if use_elev and method == 0:
            elev_mm = torch.empty((n, 2), dtype=torch.float32, device=dev)
            check(L.climsr_tile_minmax_f32(ptr(elevation_raw), n, h * w, ELEVATION_MISSING_INDICATOR, 1, ptr(elev_mm), stream),
                  "tile_minmax")
        z = self.standardize_stats
        d = TileDesc(hr_raw=ptr(hr_raw), elev_raw=ptr(elevation_raw) if use_elev else None, hr_min=ptr(mn), hr_max=ptr(mx),
                     elev_minmax=ptr(elev_mm), xform=ptr(xform), lr=ptr(out["lr"]), hr=ptr(out["hr"]),
                     elev=ptr(out.get("elevation")), mask=ptr(out["mask"]), nearest=ptr(out.get("nearest")),
                     elev_lr=ptr(out.get("elevation_lr")), hr_lr=ptr(out.get("hr_lr")),
                     range_a=self.normalize_range[0], range_b=self.normalize_range[1], eps=1e-8, nan_sub=0.0,
                     zs_hr_mean=float(z.get("hr_mean", 0.0)), zs_hr_std=float(z.get("hr_std", 1.0)),
                     zs_hr_nan_sub=float(z.get("hr_nan_sub", 0.0)), zs_elev_mean=float(z.get("elev_mean", 0.0)),
                     zs_elev_std=float(z.get("elev_std", 1.0)), zs_elev_nan_sub=float(z.get("elev_nan_sub", 0.0)),
                     elev_missing=ELEVATION_MISSING_INDICATOR, method=method, n=n, h=h, w=w, scale=s, lr_c=lr_c,
                     srcnn=int(srcnn), use_elev=int(use_elev), use_mask=int(self.use_mask))
        check(L.climsr_tile_prepare(ctypes.byref(d), stream), "tile_prepare")
        if train:
            return out
        cubic = new(n, 1, h, w)  # upscale_cubic of the LR temperature (climate_dataset.py:194-195)
        check(L.climsr_resize_cubic_f32(ptr(out["hr_lr"]), n, h // s, w // s, ptr(cubic), h, w, stream), "resize_cubic")
        out["cubic"] = cubic
        out["original_data"] = hr_raw.reshape(n, 1, h, w)
        if mn is not None:
            out["min"], out["max"] = mn, mx
        return out
