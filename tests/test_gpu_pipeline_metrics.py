"""GPU parity of the on-device tile pipeline and validation metrics.

* ``DeviceTilePipeline`` (climsr_tile_minmax_f32 + climsr_tile_prepare) vs tests/golden/pipeline.npz,
  generated with the reference's own scalers: bit-exact for every item (index maps are integer work;
  the normalisation follows numpy's rounding step by step);
* at the training size (32 tiles of 128x128) vs the numpy oracle: bit-exact;
* cv2-style cubic upscale vs the restated oracle: |diff| <= 1e-5 (parity unpinned: cv2 absent);
* RegressionAccuracy on device vs the reference's KATs: exact;
* SRMetrics vs the oracle restatement of task.py:262-372 (torchmetrics formulas): rel 1e-6 for
  sums / counts (fp64 accumulation), 1e-5 for SSIM (fp32 Gaussian filtering); deterministic.
"""
import os

import numpy as np
import pytest
import torch

from oracle import data_ref as dr

pytestmark = pytest.mark.gpu
DEV = "cuda"
CASES = {"train_esrgan": ("minmax", "esrgan", "train"), "train_srcnn": ("minmax", "srcnn", "train"),
         "val_esrgan": ("minmax", "esrgan", "val"), "train_zscore": ("zscore", "esrgan", "train")}


@pytest.fixture(scope="module")
def golden(golden_dir):
    return np.load(os.path.join(golden_dir, "pipeline.npz"))


def run_pipeline(hr_raw, elev_raw, mn, mx, codes, method, gen, stage, zs=None):
    from climsr_amd.data import DeviceTilePipeline

    p = DeviceTilePipeline(generator_type=gen, stage=stage, normalize=method == "minmax", standardize=method == "zscore",
                           standardize_stats=zs)
    out = p(torch.from_numpy(hr_raw).to(DEV), torch.from_numpy(elev_raw).to(DEV), torch.from_numpy(np.asarray(mn)),
            torch.from_numpy(np.asarray(mx)), transforms=[int(c) for c in codes] if stage == "train" else None)
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


def bits_equal(a, b):
    return a.shape == b.shape and np.array_equal(np.ascontiguousarray(a, np.float32).view(np.uint32),
                                                  np.ascontiguousarray(b, np.float32).view(np.uint32))


def describe(a, b):
    if a.shape != b.shape:
        return f"shape {a.shape} vs {b.shape}"
    bad = np.argwhere(np.ascontiguousarray(a, np.float32).view(np.uint32) != np.ascontiguousarray(b, np.float32).view(np.uint32))
    first = tuple(bad[0])
    return f"{len(bad)} of {a.size} differ; first {first}: {a[first]!r} vs {b[first]!r}; max|d| {np.nanmax(np.abs(a - b))}"


@pytest.mark.parametrize("case", list(CASES))
def test_pipeline_matches_reference_golden(golden, case):
    method, gen, stage = CASES[case]
    zs = dict(zip(("hr_mean", "hr_std", "hr_nan_sub", "elev_mean", "elev_std", "elev_nan_sub"), golden["zscore"].tolist()))
    got = run_pipeline(golden["hr_raw"], golden["elev_raw"], golden["hr_min"], golden["hr_max"], golden["codes"], method, gen,
                       stage, zs)
    keys = ["lr", "hr", "elevation", "mask"] + (["nearest", "elevation_lr", "hr_lr"] if stage != "train" else [])
    for k in keys:
        assert bits_equal(got[k], golden[f"{case}/{k}"]), f"{case}/{k}: {describe(got[k], golden[f'{case}/{k}'])}"
    if stage != "train":
        assert np.array_equal(np.isnan(got["original_data"][:, 0]), np.isnan(golden["hr_raw"]))


def test_pipeline_training_size_matches_oracle():
    rs = np.random.RandomState(11)
    n, h = 32, 128
    hr = (rs.rand(n, h, h).astype(np.float32) * 40 - 10)
    hr[rs.rand(n, h, h) < 0.3] = np.nan
    elev = (rs.rand(n, h, h) * 2500).astype(np.float32)
    elev[rs.rand(n, h, h) < 0.05] = dr.ELEV_MISSING
    mn = np.full(n, -12.5)
    mx = np.full(n, 31.0)
    codes = rs.randint(0, 16, n).astype(np.int32)
    got = run_pipeline(hr, elev, mn, mx, codes, "minmax", "esrgan", "train")
    want = dr.prepare_batch(hr, elev, mn, mx, codes)
    for k in ("lr", "hr", "elevation", "mask"):
        assert bits_equal(got[k], want[k]), f"{k}: {describe(got[k], want[k])}"


def test_cubic_upscale_matches_restated_cv2():
    from climsr_amd import _lib
    from climsr_amd._lib import check, ptr

    rs = np.random.RandomState(12)
    src = rs.rand(2, 8, 8).astype(np.float32)
    s = torch.from_numpy(src).to(DEV)
    d = torch.empty(2, 32, 32, device=DEV)
    check(_lib.load().climsr_resize_cubic_f32(ptr(s), 2, 8, 8, ptr(d), 32, 32, _lib.stream_ptr()), "cubic")
    got = d.cpu().numpy()
    for t in range(2):
        assert np.abs(got[t] - dr.cubic_resize(src[t], 32, 32)).max() <= 1e-5


SHAPE = (3, 128, 128)


@pytest.mark.parametrize("eps,kind,expected", [(0.1, "zeros_ones", 0.0), (0.1, "ones", 1.0), (0.1, "near", 1.0),
                                               (1.0, "zeros_twos", 0.0), (1.0, "ones", 1.0), (1.0, "near", 1.0),
                                               (0.25, "zeros_ones", 0.0), (0.25, "ones", 1.0), (0.25, "near", 1.0)])
def test_regression_accuracy_reference_kats(eps, kind, expected):
    from climsr_amd.metrics import RegressionAccuracy

    ones = torch.ones(SHAPE, device=DEV)
    preds = {"zeros_ones": torch.zeros(SHAPE, device=DEV), "zeros_twos": torch.zeros(SHAPE, device=DEV), "ones": ones,
             "near": ones - torch.rand(SHAPE, device=DEV) / 100}[kind]
    target = ones + 1 if kind == "zeros_twos" else ones
    sut = RegressionAccuracy(eps=eps)
    acc = sut(preds, target)
    assert acc.item() == expected
    sut.update(preds, target)
    assert sut.compute().item() == expected


def make_val_batch(n=4, h=64, seed=13):
    rs = np.random.RandomState(seed)
    original = (rs.rand(n, 1, h, h).astype(np.float32) * 30 - 5)
    original[rs.rand(n, 1, h, h) < 0.25] = np.nan
    mask = (~np.isnan(original)).astype(np.float32)
    mn, mx = np.full(n, -6.0) - rs.rand(n), np.full(n, 26.0) + rs.rand(n)
    hr = np.stack([dr.minmax_normalize(original[t], np.float64(mn[t]), np.float64(mx[t])) for t in range(n)])
    sr = np.clip(hr + rs.randn(n, 1, h, h).astype(np.float32) * 0.05, -1, 1).astype(np.float32)
    return sr, hr, original, mask, mn, mx


def test_sr_metrics_match_oracle():
    from climsr_amd.metrics import METRIC_KEYS, SRMetrics

    sr, hr, original, mask, mn, mx = make_val_batch()
    want = dr.sr_metrics(sr, hr, original, mask, mn, mx)
    m = SRMetrics()
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(DEV)  # noqa: E731
    got = m(t(sr), t(hr), t(original), t(mask), torch.from_numpy(mn), torch.from_numpy(mx), prefix="val")
    for k in METRIC_KEYS:
        g, w = got[f"val/{k}"].item(), want[k]
        tol = 1e-5 if k == "ssim" else 1e-6
        assert abs(g - w) <= tol * max(1.0, abs(w)), f"{k}: {g} vs {w}"
    assert abs(got["val/normalized_loss"].item() - want["normalized_loss"]) <= 1e-6
    again = m.raw(t(sr), t(hr), t(original), t(mask), torch.from_numpy(mn), torch.from_numpy(mx))
    assert torch.equal(again, m.raw(t(sr), t(hr), t(original), t(mask), torch.from_numpy(mn), torch.from_numpy(mx)))


def test_validation_step_through_task():
    from climsr_amd.task.pl_generator_pre_training import SuperResolutionLightningModule

    task = SuperResolutionLightningModule(generator={"_target_": "climsr_amd.models.esrgan.ESRGANGenerator", "nb": 1, "gc": 16,
                                                     "in_channels": 3, "out_channels": 1},
                                          normalization_method="minmax", normalization_range=(-1.0, 1.0))
    task.to(DEV)
    rs = np.random.RandomState(14)
    n, h = 2, 64
    raw = (rs.rand(n, h, h).astype(np.float32) * 30 - 5)
    raw[:, :10, :] = np.nan
    elev = (rs.rand(n, h, h) * 1000).astype(np.float32)
    from climsr_amd.data import DeviceTilePipeline

    batch = DeviceTilePipeline(stage="val")(torch.from_numpy(raw).to(DEV), torch.from_numpy(elev).to(DEV), [-6.0, -6.0],
                                           [26.0, 26.0])
    with torch.no_grad():
        out = task.validation_step(batch, 0)
    for k in ("val/rmse", "val/psnr", "val/ssim", "val/acc@01.25", "val/r2", "val/loss", "val/normalized_loss"):
        assert k in out and torch.isfinite(out[k]).item()
    assert float(batch["hr"][:, :, :10].abs().max()) == 0.0  # hr masked in place like task.py:290
    task.validation_epoch_end([out, out])
    assert abs(task.logged["hp_metric"].item() - out["val/rmse"].item()) < 1e-12


def test_inference_denormalize_mask_and_writer(tmp_path):
    """inference.py:73-80: float64 denormalisation of the SR map, NaN over the sea, one raster per grid."""
    from climsr_amd.inference import denormalize_mask, inference_on_full_images

    rs = np.random.RandomState(21)
    sr = rs.rand(2, 1, 12, 20).astype(np.float32) * 2 - 1
    mask = (rs.rand(2, 1, 12, 20) > 0.3).astype(np.float32)
    mn, mx = np.array([-7.25, 1.5]), np.array([31.0, 17.75])
    got = denormalize_mask(torch.from_numpy(sr).to(DEV), torch.from_numpy(mask).to(DEV), mn, mx).cpu().numpy()
    want = np.where(mask > 0, dr.minmax_denormalize(sr, mn, mx), np.nan).astype(np.float32)
    assert np.array_equal(np.isnan(got), np.isnan(want))
    assert bits_equal(np.nan_to_num(got), np.nan_to_num(want))

    class Identity(torch.nn.Module):
        def forward(self, lr, elev, mask):
            return lr[:, :1]

    batch = {"lr": torch.from_numpy(sr).to(DEV), "elevation": torch.zeros(2, 1, 12, 20, device=DEV),
             "mask": torch.from_numpy(mask).to(DEV), "min": mn, "max": mx, "filename": ["a.tif", "b.tif"]}
    paths = inference_on_full_images(Identity(), [batch], str(tmp_path))
    assert len(paths) == 2 and bits_equal(np.nan_to_num(np.load(paths[1])), np.nan_to_num(want[1, 0]))
