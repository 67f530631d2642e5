"""Validation / test metrics of the reference task, fused on device.

``SRMetrics`` reproduces ``TaskSuperResolutionModule.common_val_test_step`` + ``compute_metrics``
(climsr/core/task.py:262-294, 296-372): denormalise the SR map (MinMaxScaler with the batch's float64
per-sample min/max, or StandardScaler), zero sea pixels in sr / hr / denormalised sr / original,
then RegressionAccuracy at eps 0.1 ... 2, PSNR, SSIM and MAPE on the normalised maps where the
reference uses them (``ssim``, ``mape``), MAE / MSE / RMSE / SMAPE / PSNR / accuracy / R2 on the
denormalised ones, and the normalised L1.  One ``climsr_sr_metrics`` call = 4 launches
(fused reduction, fixed-order combine, SSIM, final) with fp64 accumulation; results stay on device as
0-d float64 tensors (views of one [17] buffer), so logging them does not sync the host.

torchmetrics (the reference's, unpinned ~0.6) is not importable here: the formulas are restated from
its published definitions (PSNR with data_range = target max - min, SSIM 11x11 / sigma 1.5 /
k1 0.01 / k2 0.03 with data_range = max of the two ranges, MAPE / SMAPE epsilon 1.17e-6, R2 uniform
average of one output) -- parity unpinned beyond the oracle restatement in oracle/data_ref.py.
"""
from __future__ import annotations

import ctypes
from typing import Dict, Optional, Sequence, Tuple

import torch
from torch import Tensor

from .. import _lib
from .._lib import MetricsDesc, check, ptr

ACC_EPS = (0.1, 0.25, 0.5, 0.75, 1.0, 1.25, 1.5, 2.0)  # task.py:297-304
METRIC_KEYS = ("acc@0.1", "acc@0.25", "acc@0.5", "acc@0.75", "acc@1", "acc@01.25", "acc@1.5", "acc@2", "psnr", "ssim",
               "mae", "mse", "rmse", "mape", "smape", "r2")  # task.py:313-330 (the reference's own key spelling)


class SRMetrics:
    def __init__(self, normalization_method: str = "minmax", normalization_range: Tuple[float, float] = (-1.0, 1.0),
                 zscore_mean: float = 0.0, zscore_std: float = 1.0, acc_eps: Sequence[float] = ACC_EPS):
        if len(acc_eps) != 8:
            raise ValueError("the reference logs exactly 8 RegressionAccuracy thresholds")
        self.method = {"minmax": 0, "zscore": 1, "none": 2}[normalization_method]
        self.range = tuple(float(v) for v in normalization_range)
        self.zscore = (float(zscore_mean), float(zscore_std))
        self.acc_eps = tuple(float(e) for e in acc_eps)
        self._ws = None

    def raw(self, sr: Tensor, hr: Tensor, original: Tensor, mask: Tensor, min_vals: Optional[Tensor] = None,
            max_vals: Optional[Tensor] = None) -> Tensor:
        """The [17] float64 device result vector (METRIC_KEYS + normalised L1)."""
        if not sr.is_cuda:
            raise RuntimeError("SRMetrics runs in libclimsr_hip.so: inputs must be CUDA tensors")
        n, c, h, w = sr.shape
        if c != 1:
            raise ValueError(f"SRMetrics expects single-channel [n, 1, h, w] maps (the reference's out_channels=1), got {tuple(sr.shape)}")
        dev = sr.device
        f32 = lambda t: t.detach().to(device=dev, dtype=torch.float32).reshape(n, 1, h, w).contiguous()  # noqa: E731
        sr_, hr_, orig_, mask_ = f32(sr), f32(hr), f32(original), f32(mask)
        mn = mx = None
        if self.method == 0:
            if min_vals is None or max_vals is None:
                raise ValueError("min-max denormalisation needs the batch's min / max")
            mn = torch.as_tensor(min_vals, dtype=torch.float64).to(dev).reshape(n).contiguous()
            mx = torch.as_tensor(max_vals, dtype=torch.float64).to(dev).reshape(n).contiguous()
        L = _lib.load()
        nbytes = L.climsr_sr_metrics_workspace()
        if self._ws is None or self._ws.device != dev:
            self._ws = torch.empty(nbytes // 8, dtype=torch.float64, device=dev)
        out = torch.empty(_lib.SR_METRICS, dtype=torch.float64, device=dev)
        d = MetricsDesc(sr=ptr(sr_), hr=ptr(hr_), original=ptr(orig_), mask=ptr(mask_), min=ptr(mn), max=ptr(mx),
                        workspace=ptr(self._ws), out=ptr(out), range_a=self.range[0], range_b=self.range[1], eps=1e-8,
                        zs_mean=self.zscore[0], zs_std=self.zscore[1], acc_eps=(ctypes.c_float * 8)(*self.acc_eps),
                        n=n, h=h, w=w, method=self.method)
        check(L.climsr_sr_metrics(ctypes.byref(d), _lib.stream_ptr(dev)), "sr_metrics")
        return out

    def __call__(self, sr: Tensor, hr: Tensor, original: Tensor, mask: Tensor, min_vals: Optional[Tensor] = None,
                 max_vals: Optional[Tensor] = None, prefix: str = "val") -> Dict[str, Tensor]:
        out = self.raw(sr, hr, original, mask, min_vals, max_vals)
        res = {f"{prefix}/{k}": out[i] for i, k in enumerate(METRIC_KEYS)}
        res[f"{prefix}/normalized_loss"] = out[16]
        res[f"{prefix}/loss"] = out[16]
        return res
