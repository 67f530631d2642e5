"""Whole-image inference driver (mirror of ``climsr/inference/inference.py:27-113``).

``inference_on_full_images`` runs the generator on each full grid, denormalises the SR map with the grid's
min / max and puts NaN over the sea on the device (``climsr_denormalize_mask``), then hands the float32 raster
to a writer.  The reference writes GeoTIFFs through rasterio with the land-mask file's profile; rasterio is not
part of this image, so the default writer stores ``<filename>.npy`` and a rasterio writer is used when the
module is importable and a ``profile`` is given.
"""
from __future__ import annotations

import os
from typing import Callable, Dict, Iterable, Optional, Tuple

import numpy as np
import torch
from torch import Tensor

from . import _lib
from ._lib import check, ptr


def denormalize_mask(sr: Tensor, mask: Optional[Tensor], mins, maxes, normalization_range=(-1.0, 1.0)) -> Tensor:
    """[n,1,h,w] fp32 SR map -> denormalised fp32 with NaN where mask == 0 (inference.py:73-76), on the device."""
    if not sr.is_cuda:
        raise RuntimeError("denormalize_mask runs in libclimsr_hip.so: CUDA tensors only")
    n = sr.shape[0]
    hw = sr[0].numel()
    s = sr.detach().float().contiguous()
    m = mask.detach().float().contiguous() if mask is not None else None
    mn = torch.as_tensor(mins, dtype=torch.float64).reshape(n).to(sr.device)
    mx = torch.as_tensor(maxes, dtype=torch.float64).reshape(n).to(sr.device)
    out = torch.empty_like(s)
    check(_lib.load().climsr_denormalize_mask(ptr(s), ptr(m), ptr(mn), ptr(mx), float(normalization_range[0]),
                                              float(normalization_range[1]), n, hw, ptr(out), _lib.stream_ptr(sr.device)),
          "denormalize_mask")
    return out


def npy_writer(path: str, arr: np.ndarray, profile: Optional[dict] = None) -> str:
    path = os.path.splitext(path)[0] + ".npy"
    np.save(path, arr)
    return path


def default_writer() -> Callable[..., str]:
    try:  # pragma: no cover - rasterio is not installed in the build image
        import rasterio as rio

        def tif_writer(path: str, arr: np.ndarray, profile: Optional[dict] = None) -> str:
            if profile is None:
                return npy_writer(path, arr)
            with rio.open(path, "w", **profile) as raster:
                raster.write(arr, 1)
            return path

        return tif_writer
    except ImportError:
        return npy_writer


def inference_on_full_images(model, batches: Iterable[Dict[str, Tensor]], out_dir: str,
                             normalization_range: Tuple[float, float] = (-1.0, 1.0), profile: Optional[dict] = None,
                             writer: Optional[Callable[..., str]] = None) -> list:
    """Batch keys as the reference's inference datasets: lr, elevation, mask (CUDA), min, max, filename."""
    os.makedirs(out_dir, exist_ok=True)
    writer = writer or default_writer()
    written = []
    with torch.no_grad():
        for batch in batches:
            sr = model(batch["lr"], batch["elevation"], batch["mask"])
            den = denormalize_mask(sr, batch["mask"], batch["min"], batch["max"], normalization_range).cpu().numpy()
            names = batch["filename"]
            names = [names] if isinstance(names, str) else list(names)
            for i, name in enumerate(names):
                written.append(writer(os.path.join(out_dir, name), den[i, 0], profile))
    return written
