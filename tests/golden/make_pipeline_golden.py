"""Generate tests/golden/pipeline.npz with the REFERENCE's own scalers (climsr.data.normalization).

Run in the build container (needs /root/reference; never on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_pipeline_golden.py

``climsr.data.normalization`` imports only numpy/torch, so it runs here read-only.  The rest of
``ClimateDataset`` (climsr/data/sr/climate_dataset.py) needs albumentations / cv2 / PIL, which are
absent, so its per-sample steps are written out below exactly in the order the reference applies
them (:236-275 normalise + mask, :149-166 flips / rot90, :169 nearest decimation == [::4, ::4] for
INTER_NEAREST with an integer ratio, :95-118 channel concatenation).
"""
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402

from climsr.data.normalization import MinMaxScaler, StandardScaler  # noqa: E402  (reference)

N, H, S = 8, 32, 4
MISSING = -32768.0
rs = np.random.RandomState(7)

# raw tiles: temperature-like values with a NaN "sea" region, elevation with missing-indicator holes
hr_raw = (rs.rand(N, H, H).astype(np.float32) * 50.0 - 20.0)
yy, xx = np.mgrid[0:H, 0:H]
for t in range(N):
    sea = (xx + (t * 7) % 11) + 0.5 * yy > 35 + 2 * t
    hr_raw[t][sea] = np.nan
hr_raw[5] = np.nan                                      # an all-sea tile
hr_raw[6][5:10, 15:20] = np.nan
elev_raw = (rs.rand(N, H, H).astype(np.float32) * 3000.0).astype(np.float32)
elev_raw[:, :3, :] = MISSING
elev_raw[3][20:, 20:] = MISSING
hr_min = np.array([np.nanmin(hr_raw[t]) if not np.all(np.isnan(hr_raw[t])) else -20.0 for t in range(N)], np.float64) - 1.5
hr_max = np.array([np.nanmax(hr_raw[t]) if not np.all(np.isnan(hr_raw[t])) else 30.0 for t in range(N)], np.float64) + 2.25
codes = np.array([0, 1, 2, 3, 4, 9, 14, 15], np.int32)  # every flip combination and rot90 k = 1, 2, 3
zs = dict(hr_mean=3.25, hr_std=11.5, hr_nan_sub=-0.75, elev_mean=812.0, elev_std=640.5, elev_nan_sub=-1.25)


def transform(img, code):
    if code & 1:
        img = np.flipud(img)
    if code & 2:
        img = np.fliplr(img)
    if (code >> 2) & 3:
        img = np.rot90(img, (code >> 2) & 3)
    return np.ascontiguousarray(img)


def batch(method, srcnn, stage):
    keys = ("lr", "hr", "elevation", "mask", "nearest", "elevation_lr", "hr_lr")
    out = {k: [] for k in keys}
    scaler = MinMaxScaler(feature_range=(-1.0, 1.0))
    elev_scaler = MinMaxScaler(feature_range=(-1.0, 1.0))
    if method == "zscore":
        scaler = StandardScaler(mean=np.float64(zs["hr_mean"]), std=np.float64(zs["hr_std"]),
                                nan_substitution=np.float64(zs["hr_nan_sub"]))
        elev_scaler = StandardScaler(mean=np.float64(zs["elev_mean"]), std=np.float64(zs["elev_std"]), missing_indicator=MISSING,
                                     nan_substitution=np.float64(zs["elev_nan_sub"]))
    for t in range(N):
        original = hr_raw[t].copy()
        if method == "minmax":
            img_hr = scaler.normalize(original.copy(), np.float64(hr_min[t]), np.float64(hr_max[t]))
            img_elev = elev_scaler.normalize(elev_raw[t].copy(), missing_indicator=MISSING)
        else:
            img_hr = scaler.normalize(arr=original.copy())
            img_elev = elev_scaler.normalize(arr=elev_raw[t].copy())
        mask = ~np.isnan(original)
        code = int(codes[t]) if stage == "train" else 0
        img_hr, img_elev, mask = transform(img_hr, code), transform(img_elev, code), transform(mask, code)
        hr_lr, elev_lr, mask_lr = img_hr[::S, ::S], img_elev[::S, ::S], mask[::S, ::S].astype(np.float32)
        nearest = np.repeat(np.repeat(hr_lr, S, 0), S, 1)
        if srcnn:
            lr = np.stack([nearest, img_elev, mask.astype(np.float32)])
        else:
            lr = np.stack([hr_lr, elev_lr, mask_lr])
        for k, v in zip(keys, (lr, img_hr[None], img_elev[None], mask.astype(np.float32)[None], nearest[None], elev_lr[None],
                               hr_lr[None])):
            out[k].append(v)
    return {k: np.stack(v).astype(np.float32) for k, v in out.items()}


arrays = dict(hr_raw=hr_raw, elev_raw=elev_raw, hr_min=hr_min, hr_max=hr_max, codes=codes,
              zscore=np.array([zs[k] for k in ("hr_mean", "hr_std", "hr_nan_sub", "elev_mean", "elev_std", "elev_nan_sub")]))
for name, (method, srcnn, stage) in {"train_esrgan": ("minmax", False, "train"), "train_srcnn": ("minmax", True, "train"),
                                     "val_esrgan": ("minmax", False, "val"), "train_zscore": ("zscore", False, "train")}.items():
    for k, v in batch(method, srcnn, stage).items():
        arrays[f"{name}/{k}"] = v
np.savez_compressed(os.path.join(HERE, "pipeline.npz"), **arrays)
print("wrote", os.path.join(HERE, "pipeline.npz"), sum(v.nbytes for v in arrays.values()) // 1024, "KiB raw")
