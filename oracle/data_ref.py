"""ORACLE — test infrastructure only.  numpy restatement of the reference's data pipeline and metrics.

Only ``tests/`` and ``__graft_entry__.smoke()`` import this module, as the checker of the device
tile pipeline / metrics in ``climsr_amd.data`` and ``climsr_amd.metrics``.  The product never
imports it.

Follows (file:line in /root/reference):
  * ``MinMaxScaler._normalize`` / ``_denormalize``  climsr/data/normalization.py:37-84
  * ``StandardScaler._normalize`` / ``_denormalize``  climsr/data/normalization.py:99-116
  * ``ClimateDataset.__getitem__`` normalisation + land mask  climsr/data/sr/climate_dataset.py:220-275
  * ``ClimateDataset._get_training_sample`` flips / rot90 / LR  climate_dataset.py:144-189
  * ``ClimateDataset._get_val_test_sample``  climate_dataset.py:191-218
  * ``ClimateDataset._concat_if_needed``  climate_dataset.py:95-118
  * ``common_val_test_step`` / ``compute_metrics``  climsr/core/task.py:262-294, 336-372
  * ``RegressionAccuracy``  climsr/metrics/regression_accuracy.py:6-22

Pinning: the scalers are checked against the reference's own ``climsr.data.normalization`` (imported
read-only when generating ``tests/golden/pipeline.npz``, ``tests/golden/make_pipeline_golden.py``);
the flip / rot90 / decimation index maps are numpy's own ``flipud`` / ``fliplr`` / ``rot90`` and
slicing; ``RegressionAccuracy`` is pinned by the reference's KATs (tests/metrics/
test_regresion_accuracy.py).  The torchmetrics PSNR / SSIM / MAE / MSE / MAPE / SMAPE / R2 formulas
(the reference's unpinned ``torchmetrics`` dependency, era 0.6) are restated from its published
definitions: parity unpinned (torchmetrics is not importable here).  cv2's INTER_CUBIC is restated
from OpenCV's published algorithm (cv2 absent): parity unpinned.
"""
from __future__ import annotations

import random
from typing import Dict, Optional, Sequence

import numpy as np

ELEV_MISSING = -32768.0  # consts.world_clim.elevation_missing_indicator
ACC_EPS = (0.1, 0.25, 0.5, 0.75, 1.0, 1.25, 1.5, 2.0)  # task.py:297-304
METRIC_KEYS = ("acc@0.1", "acc@0.25", "acc@0.5", "acc@0.75", "acc@1", "acc@01.25", "acc@1.5", "acc@2", "psnr", "ssim",
               "mae", "mse", "rmse", "mape", "smape", "r2")


# ----------------------------------------------------------------------------------------------
# scalers (numpy >= 2 / NEP 50 promotion, the numpy the reference runs with in this container)
# ----------------------------------------------------------------------------------------------
def minmax_normalize(arr: np.ndarray, mn=None, mx=None, a: float = -1.0, b: float = 1.0, eps: float = 1e-8,
                     missing_indicator: Optional[float] = None, nan_substitution: float = 0.0) -> np.ndarray:
    out = arr.copy()
    if missing_indicator:
        out[arr == missing_indicator] = np.nan
    if mn is None or mx is None:
        mx = np.nanmax(out)
        mn = np.nanmin(out)
    data_range = mx - mn
    scale = (b - a) / (data_range + eps)
    shift = a - mn * scale
    out = out * scale
    out += shift
    out[np.isnan(out)] = nan_substitution
    return out.astype(np.float32)


def zscore_normalize(arr: np.ndarray, mean, std, eps: float = 1e-8, missing_indicator: Optional[float] = None,
                     nan_substitution=None) -> np.ndarray:
    arr = arr.copy()
    if missing_indicator:
        arr[arr == missing_indicator] = np.nan
    out = (arr - mean) / (std + eps)
    if nan_substitution:
        out[np.isnan(out)] = nan_substitution
    return out.astype(np.float32)


def minmax_denormalize(arr: np.ndarray, mn: np.ndarray, mx: np.ndarray, a: float = -1.0, b: float = 1.0,
                       eps: float = 1e-8) -> np.ndarray:
    """Per-sample (arr [n,1,h,w]) float64 denormalisation of normalization.py:63-84 (torch branch)."""
    mn = np.asarray(mn, np.float64)
    mx = np.asarray(mx, np.float64)
    scale = (b - a) / ((mx - mn) + eps)
    shift = a - mn * scale
    return ((arr.astype(np.float64).transpose(1, 2, 3, 0) - shift) / scale).transpose(3, 0, 1, 2)


# ----------------------------------------------------------------------------------------------
# per-sample transforms
# ----------------------------------------------------------------------------------------------
def draw_transforms(rng: random.Random, n: int, v_flip: bool = True, h_flip: bool = True, rot: bool = True) -> np.ndarray:
    """Random draws in the order of climate_dataset.py:149-166 -> codes (bit0 v, bit1 h, bits2-3 k)."""
    codes = np.zeros(n, np.int32)
    for i in range(n):
        c = 0
        if v_flip and rng.random() > 0.5:
            c |= 1
        if h_flip and rng.random() > 0.5:
            c |= 2
        if rot and rng.random() > 0.5:
            c |= rng.randint(0, 3) << 2
        codes[i] = c
    return codes


def apply_transform(img: np.ndarray, code: int) -> np.ndarray:
    if code & 1:
        img = np.flipud(img)
    if code & 2:
        img = np.fliplr(img)
    k = (code >> 2) & 3
    if k:
        img = np.rot90(img, k)
    return np.ascontiguousarray(img)


def cubic_resize(img: np.ndarray, dh: int, dw: int) -> np.ndarray:
    """cv2.resize(INTER_CUBIC) restated: A=-0.75, replicate border, horizontal then vertical (float32)."""
    sh, sw = img.shape
    A = np.float32(-0.75)

    def coeffs(x):
        x = np.float32(x)
        c0 = ((A * (x + 1) - 5 * A) * (x + 1) + 8 * A) * (x + 1) - 4 * A
        c1 = ((A + 2) * x - (A + 3)) * x * x + 1
        c2 = ((A + 2) * (1 - x) - (A + 3)) * (1 - x) * (1 - x) + 1
        return np.array([c0, c1, c2, np.float32(1) - c0 - c1 - c2], np.float32)

    out = np.zeros((dh, dw), np.float32)
    for dy in range(dh):
        fy = np.float32((dy + 0.5) * (sh / dh) - 0.5)
        y0 = int(np.floor(fy))
        cy = coeffs(fy - y0)
        for dx in range(dw):
            fx = np.float32((dx + 0.5) * (sw / dw) - 0.5)
            x0 = int(np.floor(fx))
            cx = coeffs(fx - x0)
            acc = np.float32(0)
            for i in range(4):
                row = img[min(max(y0 - 1 + i, 0), sh - 1)]
                r = np.float32(0)
                for j in range(4):
                    r = np.float32(r + np.float32(row[min(max(x0 - 1 + j, 0), sw - 1)] * cx[j]))
                acc = np.float32(acc + np.float32(r * cy[i]))
            out[dy, dx] = acc
    return out


def prepare_batch(hr_raw: np.ndarray, elev_raw: np.ndarray, hr_min: Sequence[float], hr_max: Sequence[float],
                  codes: Optional[np.ndarray] = None, generator_type: str = "esrgan", scale: int = 4,
                  normalize_range=(-1.0, 1.0), use_elevation: bool = True, use_mask: bool = True, method: str = "minmax",
                  zscore_stats: Optional[Dict[str, float]] = None, stage: str = "train") -> Dict[str, np.ndarray]:
    """Batch of ClimateDataset samples (hr_raw/elev_raw [n,h,w] float32) -> the collated batch dict."""
    a, b = normalize_range
    n, h, w = hr_raw.shape
    out = {k: [] for k in ("lr", "hr", "elevation", "mask", "nearest", "elevation_lr", "hr_lr")}
    for t in range(n):
        original = hr_raw[t]
        if method == "minmax":
            img_hr = minmax_normalize(original, np.float64(hr_min[t]), np.float64(hr_max[t]), a, b)
            img_elev = minmax_normalize(elev_raw[t], a=a, b=b, missing_indicator=ELEV_MISSING)
        elif method == "zscore":
            z = zscore_stats
            img_hr = zscore_normalize(original, np.float64(z["hr_mean"]), np.float64(z["hr_std"]),
                                      nan_substitution=np.float64(z["hr_nan_sub"]))
            img_elev = zscore_normalize(elev_raw[t], np.float64(z["elev_mean"]), np.float64(z["elev_std"]),
                                        missing_indicator=ELEV_MISSING, nan_substitution=np.float64(z["elev_nan_sub"]))
        else:
            img_hr, img_elev = original.copy(), elev_raw[t].copy()
        mask = ~np.isnan(original)
        code = int(codes[t]) if (codes is not None and stage == "train") else 0
        img_hr = apply_transform(img_hr, code)
        img_elev = apply_transform(img_elev, code)
        mask = apply_transform(mask, code)
        hr_lr = img_hr[::scale, ::scale]                         # A.Resize(INTER_NEAREST), integer ratio
        elev_lr = img_elev[::scale, ::scale]
        mask_lr = mask[::scale, ::scale].astype(np.float32)
        nearest = np.repeat(np.repeat(hr_lr, scale, 0), scale, 1)  # upscale_nearest
        if generator_type == "srcnn":
            chans = [nearest] + ([img_elev] if use_elevation else []) + ([mask.astype(np.float32)] if use_mask else [])
        else:
            chans = [hr_lr] + ([elev_lr] if use_elevation else []) + ([mask_lr] if use_mask else [])
        out["lr"].append(np.stack(chans))
        out["hr"].append(img_hr[None])
        out["elevation"].append(img_elev[None])
        out["mask"].append(mask.astype(np.float32)[None])
        out["nearest"].append(nearest[None])
        out["elevation_lr"].append(elev_lr[None])
        out["hr_lr"].append(hr_lr[None])
    return {k: np.stack(v).astype(np.float32) for k, v in out.items()}


# ----------------------------------------------------------------------------------------------
# metrics (torchmetrics ~0.6 definitions, restated)
# ----------------------------------------------------------------------------------------------
def regression_accuracy(preds: np.ndarray, target: np.ndarray, eps: float) -> float:
    d = np.abs(preds.astype(np.float32) - target.astype(np.float32))
    return float(np.sum(d <= np.float32(eps))) / target.size


def _gaussian(k: int = 11, sigma: float = 1.5) -> np.ndarray:
    dist = np.arange((1 - k) / 2, (1 + k) / 2, 1, dtype=np.float64)
    g = np.exp(-((dist / sigma) ** 2) / 2)
    return g / g.sum()


def ssim(preds: np.ndarray, target: np.ndarray, k: int = 11, sigma: float = 1.5) -> float:
    """torchmetrics _ssim_compute with data_range=None, over [n,1,h,w]; valid (cropped) region mean."""
    p = preds.astype(np.float64)[:, 0]
    t = target.astype(np.float64)[:, 0]
    dr = max(p.max() - p.min(), t.max() - t.min())
    c1, c2 = (0.01 * dr) ** 2, (0.03 * dr) ** 2
    g = _gaussian(k, sigma)
    r = k // 2

    def filt(x):  # valid separable 2D filtering == cropped output of the reflect-padded conv
        h = sum(g[i] * x[:, :, i:x.shape[2] - 2 * r + i] for i in range(k))
        return sum(g[i] * h[:, i:h.shape[1] - 2 * r + i, :] for i in range(k))

    mp, mt = filt(p), filt(t)
    spp = filt(p * p) - mp * mp
    stt = filt(t * t) - mt * mt
    spt = filt(p * t) - mp * mt
    idx = ((2 * mp * mt + c1) * (2 * spt + c2)) / ((mp * mp + mt * mt + c1) * (spp + stt + c2))
    return float(idx.mean())


def sr_metrics(sr: np.ndarray, hr: np.ndarray, original: np.ndarray, mask: np.ndarray, mn, mx,
               normalize_range=(-1.0, 1.0)) -> Dict[str, float]:
    """common_val_test_step (task.py:262-294) + compute_metrics (task.py:336-372), minmax method."""
    a, b = normalize_range
    land = mask.astype(bool)
    den = minmax_denormalize(sr, mn, mx, a, b)
    sr_n = np.where(land, sr, 0).astype(np.float32)
    hr_n = np.where(land, hr, 0).astype(np.float32)
    p = np.where(land, den, 0.0)
    t = np.where(land, original.astype(np.float64), 0.0)
    n = p.size
    d = p - t
    res = {}
    for key, e in zip(METRIC_KEYS[:8], ACC_EPS):
        res[key] = float(np.sum(np.abs(d) <= e)) / n
    mse = float(np.sum(d * d)) / n
    res["psnr"] = 10.0 * np.log10((t.max() - t.min()) ** 2 / mse)
    res["ssim"] = ssim(sr_n, hr_n)
    res["mae"] = float(np.sum(np.abs(d))) / n
    res["mse"] = mse
    res["rmse"] = float(np.sqrt(mse))
    res["mape"] = float(np.sum(np.abs(sr_n - hr_n) / np.maximum(np.abs(hr_n), np.float32(1.17e-6)))) / n
    res["smape"] = 2.0 * float(np.sum(np.abs(d) / np.maximum(np.abs(t) + np.abs(p), 1.17e-6))) / n
    res["r2"] = 1.0 - float(np.sum(d * d)) / (float(np.sum(t * t)) - float(np.sum(t)) * float(np.sum(t)) / n)
    res["normalized_loss"] = float(np.mean(np.abs(sr_n.astype(np.float64) - hr_n)))
    return res
