"""Fused AdamW (+ device-side OneCycleLR for captured steps) over flat parameter buffers.

Replaces ``torch.optim.AdamW`` (conf/optimizers/adamw.yaml: lr, weight_decay=1e-4, betas
(0.9,0.999) with beta1 cycled by OneCycleLR, eps 1e-8) wired by
``climsr/core/instantiator.py:48-49`` and ``OneCycleLR`` (conf/schedulers/one_cycle_schedule.yaml,
instantiator.py:51-64).  One kernel updates a whole network's flat fp32 buffer.
"""
from __future__ import annotations

from typing import Iterable, List, Optional

import torch

from .. import _lib
from .._lib import ptr
from ..ops import _launch


def _flat_owner(params: List[torch.Tensor]):
    """If params are exactly the views of one flat buffer in order, return (flat, flat_grad_base_check)."""
    if not params:
        return None
    base = params[0]
    st = base.untyped_storage()
    off = base.storage_offset()
    for p in params:
        if p.untyped_storage().data_ptr() != st.data_ptr() or p.storage_offset() != off or p.dtype != torch.float32:
            return None
        off += p.numel()
    if off != st.nbytes() // 4:
        return None
    return torch.empty(0, dtype=torch.float32, device=base.device).set_(st, 0, (off,))


class AdamW(torch.optim.Optimizer):
    """Drop-in for torch.optim.AdamW (amsgrad=False) whose update runs in libclimsr_hip.

    Hyper-parameters are read from ``param_groups`` at every step, so torch's own
    ``OneCycleLR`` (which cycles lr and betas[0]) drives it unchanged.  When the params are the
    views of one flat buffer (climsr_amd modules) the whole group is one launch; the module's
    bf16 weight layouts are refreshed through ``owner.repack_weights()`` when given.
    """

    # torch.optim.AdamW options this fused update does not implement: accepted only at their default value
    _UNSUPPORTED = {"maximize": False, "foreach": None, "fused": None, "capturable": False, "differentiable": False}

    def __init__(self, params: Iterable, lr: float = 1e-3, betas=(0.9, 0.999), eps: float = 1e-8, weight_decay: float = 1e-2,
                 amsgrad: bool = False, owner=None, **kwargs):
        if amsgrad:
            raise ValueError("amsgrad is not supported")
        for k, v in kwargs.items():
            if k not in self._UNSUPPORTED:
                raise TypeError(f"AdamW got an unexpected keyword argument {k!r}")
            if v != self._UNSUPPORTED[k]:
                raise ValueError(f"AdamW option {k}={v!r} is not supported by the fused update (only {self._UNSUPPORTED[k]!r})")
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.owner = owner
        self._hp = None

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        lib = _lib.load()
        mirrored = False
        for group in self.param_groups:
            params = [p for p in group["params"] if p.grad is not None]
            if not params:
                continue
            st = self.state.setdefault("group%d" % self.param_groups.index(group), {})
            step = st.get("step", 0) + 1
            st["step"] = step
            lr = group["lr"]
            b1, b2 = group["betas"]
            bc1 = 1 - b1 ** step
            bc2 = 1 - b2 ** step
            hp = torch.tensor([lr, b1, b2, group["eps"], group["weight_decay"], lr / bc1, bc2 ** 0.5, 0.0],
                              dtype=torch.float32).to(params[0].device, non_blocking=True)
            flat = _flat_owner(group["params"]) if len(params) == len(group["params"]) else None
            if flat is not None:
                gflat = _flat_owner([p.grad for p in group["params"]])
                own = self.owner
                if gflat is None and own is not None and getattr(own, "_flat", None) is not None and \
                        own._flat.data_ptr() == flat.data_ptr() and own._flat.numel() == flat.numel():
                    # gradients delivered through autograd as separate tensors (torch DDP; a module called twice sums
                    # its nodes' gradients out of place): gather them into the module's flat gradient buffer (one
                    # multi-tensor copy) and keep the one-launch update
                    views = [own._flat_grad[off:off + n].view(p.shape) for p, off, n in own._flat_index]
                    torch._foreach_copy_(views, [p.grad for p in group["params"]])
                    gflat = own._flat_grad
                if gflat is None:
                    flat = None
            if flat is not None:
                if "m" not in st:
                    st["m"] = torch.zeros_like(flat)
                    st["v"] = torch.zeros_like(flat)
                _adamw_flat(lib, self.owner, flat, gflat, st["m"], st["v"], hp, _lib.stream_ptr())
                mirrored = True
            else:
                for p in params:
                    ps = self.state[p]
                    if "m" not in ps:
                        ps["m"] = torch.zeros_like(p)
                        ps["v"] = torch.zeros_like(p)
                    g = p.grad.contiguous()
                    _launch("adamw", lambda: lib.climsr_adamw_step(p.numel(), ptr(p), ptr(g), ptr(ps["m"]), ptr(ps["v"]), ptr(hp),
                                                                   _lib.stream_ptr()), nbytes=28 * p.numel())
        if self.owner is not None:
            if mirrored and _mirror_of(self.owner) is not None:
                self.owner.repack_weights(mirror_done=True)
            else:
                self.owner.repack_weights()
        return loss


def _mirror_of(module):
    """(offset, numel, bf16 buffer) of a weight the module reads as a bf16 copy of its flat buffer, or None."""
    fn = getattr(module, "bf16_mirror", None)
    return fn() if fn is not None else None


def _adamw_flat(lib, module, flat, gflat, m, v, hp, stream):
    """One fused AdamW launch over a flat buffer; when ``module`` mirrors part of it in bf16 (``bf16_mirror()``), the
    same pass writes that copy."""
    mir = _mirror_of(module) if module is not None else None
    if mir is None:
        _launch("adamw", lambda: lib.climsr_adamw_step(flat.numel(), ptr(flat), ptr(gflat), ptr(m), ptr(v), ptr(hp), stream),
                nbytes=28 * flat.numel())
    else:
        lo, n, buf = mir
        _launch("adamw", lambda: lib.climsr_adamw_step_mirror(flat.numel(), ptr(flat), ptr(gflat), ptr(m), ptr(v), ptr(hp), lo, n,
                                                              ptr(buf), stream), nbytes=28 * flat.numel() + 2 * n)


class GraphedAdamW:
    """AdamW + OneCycleLR with all scalars on the device, for hipGraph-captured training steps.

    ``step()`` launches: schedule kernel (lr, beta1, bias corrections from a device step counter),
    the fused update over the flat buffer, and the bf16 weight repack.  Semantics equal
    torch AdamW stepped before OneCycleLR.step() each iteration (Lightning interval="step").
    """

    def __init__(self, module, lr: float = 1e-4, total_steps: int = 1000, weight_decay: float = 1e-4, pct_start: float = 0.05,
                 div_factor: float = 2.0, final_div_factor: float = 100.0, betas=(0.9, 0.999), eps: float = 1e-8):
        self.module = module
        flat = module._flat
        self.m = torch.zeros_like(flat)
        self.v = torch.zeros_like(flat)
        self.state = torch.zeros(2, dtype=torch.float64, device=flat.device)
        self.hp = torch.zeros(8, dtype=torch.float32, device=flat.device)
        self.cfg = (int(total_steps), float(lr), float(pct_start), float(div_factor), float(final_div_factor), float(betas[1]),
                    float(eps), float(weight_decay))

    def step(self):
        lib = _lib.load()
        s = _lib.stream_ptr()
        ts, lr, pct, div, fdiv, b2, eps, wd = self.cfg
        _launch("adamw_hparams", lambda: lib.climsr_adamw_hparams(ptr(self.state), ts, lr, pct, div, fdiv, b2, eps, wd, ptr(self.hp),
                                                                  s))
        flat = self.module._flat
        _adamw_flat(lib, self.module, flat, self.module._flat_grad, self.m, self.v, self.hp, s)
        if _mirror_of(self.module) is not None:
            self.module.engine().repack(mirror_done=True)
        else:
            self.module.engine().repack()
