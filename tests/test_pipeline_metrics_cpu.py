"""CPU checks of the data-pipeline / metrics oracle (oracle/data_ref.py) and host logic.

* the numpy restatement of ClimateDataset's per-sample work reproduces tests/golden/pipeline.npz
  (made with the reference's own climsr.data.normalization scalers) bit for bit;
* the device pipeline's host-side random draws follow the reference's draw order;
* RegressionAccuracy reproduces the reference's own KATs (tests/metrics/test_regresion_accuracy.py);
* SSIM / cubic sanity properties of the restated (parity-unpinned) torchmetrics / cv2 algorithms.
"""
import os
import random

import numpy as np
import pytest
import torch

from oracle import data_ref as dr

CASES = {"train_esrgan": ("minmax", "esrgan", "train"), "train_srcnn": ("minmax", "srcnn", "train"),
         "val_esrgan": ("minmax", "esrgan", "val"), "train_zscore": ("zscore", "esrgan", "train")}


@pytest.fixture(scope="module")
def golden(golden_dir):
    return np.load(os.path.join(golden_dir, "pipeline.npz"))


def zscore_stats(g):
    return dict(zip(("hr_mean", "hr_std", "hr_nan_sub", "elev_mean", "elev_std", "elev_nan_sub"), g["zscore"].tolist()))


@pytest.mark.parametrize("case", list(CASES))
def test_oracle_pipeline_matches_reference_scalers(golden, case):
    method, gen, stage = CASES[case]
    got = dr.prepare_batch(golden["hr_raw"], golden["elev_raw"], golden["hr_min"], golden["hr_max"], golden["codes"],
                           generator_type=gen, method=method, zscore_stats=zscore_stats(golden), stage=stage)
    for k, v in got.items():
        want = golden[f"{case}/{k}"]
        assert v.shape == want.shape, k
        assert np.array_equal(v.view(np.uint32), want.view(np.uint32)), f"{case}/{k} not bit-exact"


def test_golden_covers_edge_cases(golden):
    hr = golden["hr_raw"]
    assert np.all(np.isnan(hr[5]))                       # an all-sea tile
    assert (golden["elev_raw"] == dr.ELEV_MISSING).any()  # missing elevation
    assert sorted({int(c) & 3 for c in golden["codes"]}) == [0, 1, 2, 3]
    assert sorted({(int(c) >> 2) & 3 for c in golden["codes"]}) == [0, 1, 2, 3]


def test_host_draw_order_matches_reference():
    from climsr_amd.data import DeviceTilePipeline, TransformsCfg

    p = DeviceTilePipeline(seed=1234)
    assert p.draw_transforms(64) == dr.draw_transforms(random.Random(1234), 64).tolist()
    p = DeviceTilePipeline(seed=5, transforms_cfg=TransformsCfg(v_flip=False))
    assert p.draw_transforms(16) == dr.draw_transforms(random.Random(5), 16, v_flip=False).tolist()


def test_pipeline_refuses_cpu_tensors():
    from climsr_amd.data import DeviceTilePipeline

    with pytest.raises(RuntimeError, match="CUDA"):
        DeviceTilePipeline()(torch.zeros(2, 16, 16), torch.zeros(2, 16, 16), [0, 0], [1, 1])


SHAPE = (3, 128, 128)


@pytest.mark.parametrize("eps,preds,target,expected", [
    (0.1, np.zeros(SHAPE), np.ones(SHAPE), 0.0),
    (0.1, np.ones(SHAPE), np.ones(SHAPE), 1.0),
    (0.1, np.ones(SHAPE) - np.random.RandomState(0).rand(*SHAPE) / 100, np.ones(SHAPE), 1.0),
    (1.0, np.zeros(SHAPE), np.ones(SHAPE) + 1, 0.0),
    (1.0, np.ones(SHAPE), np.ones(SHAPE), 1.0),
    (1.0, np.ones(SHAPE) - np.random.RandomState(1).rand(*SHAPE) / 100, np.ones(SHAPE), 1.0),
    (0.25, np.zeros(SHAPE), np.ones(SHAPE), 0.0),
    (0.25, np.ones(SHAPE), np.ones(SHAPE), 1.0),
    (0.25, np.ones(SHAPE) - np.random.RandomState(2).rand(*SHAPE) / 100, np.ones(SHAPE), 1.0),
])
def test_oracle_regression_accuracy_reference_kats(eps, preds, target, expected):
    assert dr.regression_accuracy(preds.astype(np.float32), target.astype(np.float32), eps) == expected


def test_oracle_ssim_and_cubic_properties():
    rs = np.random.RandomState(3)
    x = rs.rand(2, 1, 24, 24).astype(np.float32)
    assert abs(dr.ssim(x, x) - 1.0) < 1e-12
    assert dr.ssim(x, rs.rand(2, 1, 24, 24).astype(np.float32)) < 0.5
    c = np.full((5, 7), 2.5, np.float32)
    assert np.allclose(dr.cubic_resize(c, 20, 28), 2.5, atol=1e-6)


def test_oracle_metrics_identity():
    rs = np.random.RandomState(4)
    hr = rs.rand(2, 1, 16, 16).astype(np.float32) * 2 - 1
    mask = (rs.rand(2, 1, 16, 16) > 0.2).astype(np.float32)
    mn, mx = np.array([-5.0, 0.0]), np.array([20.0, 31.0])
    orig = dr.minmax_denormalize(hr, mn, mx).astype(np.float32)
    m = dr.sr_metrics(hr, hr, orig, mask, mn, mx)
    assert m["acc@0.1"] == 1.0 and m["mae"] < 1e-5 and m["normalized_loss"] == 0.0 and abs(m["ssim"] - 1) < 1e-9
