"""``RegressionAccuracy`` on device (mirror of climsr/metrics/regression_accuracy.py:6-22).

Same torchmetrics-style API: ``update(preds, target)`` accumulates ``correct += #(|p - t| <= eps)``
and ``total += numel`` in int64 device counters (``climsr_regression_accuracy_update``; exact and
order-independent), ``compute()`` returns ``correct / total`` as a 0-d float32 tensor, and calling
the metric returns the value of that batch alone while also accumulating (torchmetrics ``forward``).
No host synchronisation.  Inputs must be CUDA float tensors of equal shape.
"""
from __future__ import annotations

import torch
from torch import Tensor

from .. import _lib
from .._lib import check, ptr


class RegressionAccuracy:
    def __init__(self, eps: float = 1.0, dist_sync_on_step: bool = False):
        self.eps = eps
        self.dist_sync_on_step = dist_sync_on_step
        self._counts = None  # int64 [correct, total] on the inputs' device

    def reset(self) -> None:
        if self._counts is not None:
            self._counts.zero_()

    def _update_into(self, counts: Tensor, preds: Tensor, target: Tensor) -> None:
        assert preds.shape == target.shape
        if not (preds.is_cuda and target.is_cuda):
            raise RuntimeError("RegressionAccuracy runs in libclimsr_hip.so: preds / target must be CUDA tensors")
        p = preds.detach().to(torch.float32).contiguous()
        t = target.detach().to(torch.float32).contiguous()
        check(_lib.load().climsr_regression_accuracy_update(ptr(p), ptr(t), p.numel(), float(self.eps), ptr(counts),
                                                            _lib.stream_ptr(p.device)), "regression_accuracy")

    def update(self, preds: Tensor, target: Tensor) -> None:
        if self._counts is None:
            self._counts = torch.zeros(2, dtype=torch.int64, device=preds.device)
        self._update_into(self._counts, preds, target)

    @staticmethod
    def _ratio(counts: Tensor) -> Tensor:
        return counts[0].to(torch.float32) / counts[1]

    def compute(self) -> Tensor:
        if self._counts is None:
            raise RuntimeError("RegressionAccuracy.compute() before update()")
        if self.dist_sync_on_step and torch.distributed.is_available() and torch.distributed.is_initialized():
            c = self._counts.clone()
            torch.distributed.all_reduce(c)  # dist_reduce_fx="sum"
            return self._ratio(c)
        return self._ratio(self._counts)

    def __call__(self, preds: Tensor, target: Tensor) -> Tensor:
        batch = torch.zeros(2, dtype=torch.int64, device=preds.device)
        self._update_into(batch, preds, target)
        if self._counts is None:
            self._counts = torch.zeros(2, dtype=torch.int64, device=preds.device)
        self._counts += batch
        return self._ratio(batch)
