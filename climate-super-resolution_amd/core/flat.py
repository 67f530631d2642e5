"""Flat parameter / gradient storage for the native modules.

Every trainable parameter of a native module is a view into ONE contiguous fp32 buffer, and its
``.grad`` is a view into ONE contiguous fp32 gradient buffer.  The HIP backward writes gradients
straight into that buffer (no per-parameter autograd accumulation), the fused AdamW updates the
whole buffer in one launch, and the data-parallel all-reduce sends it in a few large RCCL buckets.
``state_dict`` keys and shapes stay identical to the reference (the views are ordinary Parameters).
"""
from __future__ import annotations

from typing import List, Tuple

import torch
import torch.nn as nn


class FlatParamsMixin:
    """Mixin for nn.Module subclasses; call ``_flatten()`` at the end of ``__init__``."""

    _flat: torch.Tensor
    _flat_grad: torch.Tensor
    _flat_index: List[Tuple[nn.Parameter, int, int]]

    def _flatten(self) -> None:
        params = [p for p in self.parameters()]
        total = sum(p.numel() for p in params)
        dev = params[0].device if params else torch.device("cpu")
        flat = torch.empty(total, dtype=torch.float32, device=dev)
        index = []
        off = 0
        for p in params:
            n = p.numel()
            flat[off:off + n].copy_(p.data.reshape(-1))
            index.append((p, off, n))
            off += n
        object.__setattr__(self, "_flat", flat)
        object.__setattr__(self, "_flat_grad", torch.zeros(total, dtype=torch.float32, device=dev))
        object.__setattr__(self, "_flat_index", index)
        self._rebind()

    def _rebind(self) -> None:
        for p, off, n in self._flat_index:
            p.data = self._flat[off:off + n].view(p.shape)

    def _flat_intact(self) -> bool:
        base = self._flat.data_ptr()
        for p, off, n in self._flat_index:
            if p.data_ptr() != base + 4 * off or p.dtype != torch.float32 or p.device != self._flat.device:
                return False
        return True

    def _ensure_flat(self) -> None:
        """Re-home parameters into the flat buffer if something replaced their storage."""
        if self._flat_intact():
            return
        dev = self._flat_index[0][0].device if self._flat_index else self._flat.device
        total = self._flat.numel()
        flat = torch.empty(total, dtype=torch.float32, device=dev)
        for p, off, n in self._flat_index:
            flat[off:off + n].copy_(p.data.reshape(-1).to(torch.float32))
        object.__setattr__(self, "_flat", flat)
        object.__setattr__(self, "_flat_grad", torch.zeros(total, dtype=torch.float32, device=dev))
        self._rebind()
        self._on_flat_moved()

    def _on_flat_moved(self) -> None:  # overridden by modules holding device plans
        pass

    def _apply(self, fn, recurse=True):  # keep the flat layout across .to()/.cuda()
        ret = super()._apply(fn, recurse)  # type: ignore[misc]
        if getattr(self, "_flat_index", None):
            self._ensure_flat()
        return ret

    def grads_as_views(self) -> bool:
        """Point every param.grad at its slice of the flat grad buffer.  Returns True if they
        already were (=> backward accumulates), False if (re)linked (=> backward overwrites)."""
        base = self._flat_grad.data_ptr()
        linked = True
        for p, off, n in self._flat_index:
            g = p.grad
            if g is None or g.data_ptr() != base + 4 * off:
                linked = False
                break
        if not linked:
            for p, off, n in self._flat_index:
                p.grad = self._flat_grad[off:off + n].view(p.shape)
        return linked
