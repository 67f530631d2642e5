"""L1 loss (mean) as a native autograd node: ``torch.nn.L1Loss`` of task.py:141 / pl_gan.py:20.

Forward: deterministic two-pass reduction (fp64 partials) in libclimsr_hip; backward:
``sign(a-b) * g / n`` with the upstream gradient read from device memory (graph-capturable).
"""
import torch

from .. import _lib
from .._lib import ptr
from ..ops import _launch


class _L1Fn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        a = a.contiguous().float()
        b = b.contiguous().float()
        assert a.shape == b.shape and a.is_cuda
        ws = torch.empty(1024, dtype=torch.float64, device=a.device)
        out = torch.empty((), dtype=torch.float32, device=a.device)
        _launch("l1_loss", lambda: _lib.load().climsr_l1_loss(ptr(a), ptr(b), a.numel(), ptr(ws), ptr(out), _lib.stream_ptr()),
                nbytes=8 * a.numel())
        ctx.save_for_backward(a, b)
        return out

    @staticmethod
    def backward(ctx, g):
        a, b = ctx.saved_tensors
        g = g.contiguous().float()
        ga = torch.empty_like(a) if ctx.needs_input_grad[0] else None
        gb = None
        if ga is not None:
            _launch("l1_grad", lambda: _lib.load().climsr_l1_loss_grad(ptr(a), ptr(b), a.numel(), ptr(g), ptr(ga), _lib.stream_ptr()),
                    nbytes=12 * a.numel())
        if ctx.needs_input_grad[1]:
            gb = torch.empty_like(b)
            _launch("l1_grad", lambda: _lib.load().climsr_l1_loss_grad(ptr(b), ptr(a), b.numel(), ptr(g), ptr(gb), _lib.stream_ptr()),
                    nbytes=12 * b.numel())
        return ga, gb


def l1_loss(a, b):
    return _L1Fn.apply(a, b)


class L1Loss(torch.nn.Module):
    """Drop-in for torch.nn.L1Loss() (reduction='mean')."""

    def forward(self, input, target):
        return l1_loss(input, target)
