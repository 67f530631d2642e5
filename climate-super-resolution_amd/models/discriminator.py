"""Plain discriminator (drop-in for ``climsr.models.discriminator.Discriminator``).

Same constructor (``in_channels=1, out_channels=64, num_conv_block=4``), same ``feature_extraction`` /
``avgpool`` / ``classification`` submodules and ``state_dict`` keys (discriminator.py:6-40),
``forward(x: [N,C,H,W]) -> [N,1]`` raw scores (discriminator.py:42-46; like the reference it only works
where the flattened features are 8192 wide, i.e. 128x128 inputs with the defaults).  Honours
``.train()`` / ``.eval()``.  Arithmetic in libclimsr_hip:

* ``ReflectionPad2d(1)`` as an explicit bf16 pad launch (its backward folds the mirrored rows/columns);
* conv + bias + LeakyReLU(0.01) fused (implicit GEMM, stride 1/2, pad 0); the BatchNorm AFTER the
  activation with batch statistics (train) or running statistics (eval); its backward chains the LeakyReLU
  derivative (``climsr_bn_backward`` out_slope);
* the two valid 3x3 convs (LeakyReLU 0.2 between them), the NCHW flatten, ``classification.0``
  (8192->100, MFMA split-K, rows padded to 128) and ``classification.1`` (100->1, no sigmoid).
The ``avgpool`` member is constructed but unused, exactly as in the reference forward.
"""
from __future__ import annotations

from typing import Dict, List

import torch
import torch.nn as nn
from torch import Tensor

from .. import ops
from ..core.flat import FlatParamsMixin
from ..ops import ACT_LRELU, ACT_NONE, BatchedPacker, ConvPlan, Workspace

FC_PAD = 128  # classification.0 rows padded for the MFMA linear kernels (o % 64 == 0)


def _bf16(shape, dev):
    return torch.empty(shape, dtype=torch.bfloat16, device=dev)


def _f32(shape, dev):
    return torch.empty(shape, dtype=torch.float32, device=dev)


class _PlainDEngine:
    def __init__(self, d: "Discriminator"):
        self.d = d
        dev = d.classification[0].weight.device
        feats = list(d.feature_extraction)
        self.layers = []  # dict(conv, plan, rpad, slope, bn)
        for i, m in enumerate(feats):
            if not isinstance(m, nn.Conv2d):
                continue
            rpad = i > 0 and isinstance(feats[i - 1], nn.ReflectionPad2d)
            act = feats[i + 1] if i + 1 < len(feats) and isinstance(feats[i + 1], nn.LeakyReLU) else None
            bn = feats[i + 2] if act is not None and i + 2 < len(feats) and isinstance(feats[i + 2], nn.BatchNorm2d) else None
            plan = ConvPlan(m.in_channels, m.out_channels, 3, m.stride[0], 0, f"feature_extraction.{i}")
            plan.bind(m.weight, m.bias, need_t=True)
            self.layers.append(dict(conv=m, plan=plan, rpad=rpad, slope=(act.negative_slope if act is not None else None), bn=bn))
        self.packer = BatchedPacker([L["plan"] for L in self.layers], dev)
        fc0 = d.classification[0]
        self.feat = fc0.in_features
        self.hid = fc0.out_features
        assert self.hid <= FC_PAD
        self.w0 = torch.zeros((FC_PAD, self.feat), dtype=torch.bfloat16, device=dev)
        self.b0 = torch.zeros((FC_PAD,), dtype=torch.float32, device=dev)
        self.w1 = torch.zeros((FC_PAD,), dtype=torch.float32, device=dev)
        self.version = -1
        self.ws = Workspace()
        self.scratch: Dict[str, Tensor] = {}

    def ensure_packed(self):
        if self.d._flat._version != self.version:
            self.repack()

    def repack(self):
        d = self.d
        self.packer.run()
        fc0, fc1 = d.classification[0], d.classification[1]
        ops.f32_to_bf16(fc0.weight, self.w0[: self.hid])
        self.b0[: self.hid].copy_(fc0.bias)
        self.w1[: self.hid].copy_(fc1.weight.view(-1))
        self.version = d._flat._version

    def _scr(self, key, shape, dtype, dev):
        t = self.scratch.get(key)
        if t is None or tuple(t.shape) != tuple(shape) or t.device != dev:
            t = torch.zeros(shape, dtype=dtype, device=dev)
            self.scratch[key] = t
        return t

    # ------------------------------------------------------------------ forward
    def forward(self, x: Tensor, keep: bool, need_pt: bool):
        d = self.d
        n, cin, h, w = x.shape
        dev = x.device
        self.ensure_packed()
        cpad = (cin + 7) // 8 * 8
        a = torch.zeros((n, h, w, cpad), dtype=torch.bfloat16, device=dev)
        ops.nchw_to_nhwc(x.contiguous().float(), a, cpad, 0)
        cs, hh, ww = cpad, h, w
        saved = []
        for L in self.layers:
            plan = L["plan"]
            if L["rpad"]:
                xp = _bf16((n, hh + 2, ww + 2, cs), dev)
                ops.reflect_pad1(a, n, hh, ww, cs, xp)
                src, sh, sw = xp, hh + 2, ww + 2
            else:
                src, sh, sw = a, hh, ww
            oh, ow = plan.out_hw(sh, sw)
            if oh < 1 or ow < 1:  # the reference fails here too (kernel larger than the input)
                raise RuntimeError(f"Discriminator: {h}x{w} input leaves no pixels for {plan.name}; the reference architecture "
                                   f"only runs on inputs that flatten to 8192 (128x128), discriminator.py:42-46")
            c = plan.cout
            t = _bf16((n, oh, ow, c), dev)
            slope = L["slope"]
            plan.fwd(src, cs, 0, sh, sw, t, c, 0, n, act=(ACT_LRELU if slope is not None else ACT_NONE),
                     slope=(slope if slope is not None else 0.0))
            rec = dict(src=src, cs_in=cs, sh=sh, sw=sw, h_in=hh, w_in=ww, t=t, oh=oh, ow=ow, mean=None, rstd=None)
            bn = L["bn"]
            out = t
            if bn is not None:
                out = _bf16((n, oh, ow, c), dev)
                npix = n * oh * ow
                if d.training:
                    mean, rstd = _f32((c,), dev), _f32((c,), dev)
                    ops.bn_forward(t, npix, c, bn.weight, bn.bias, mean, rstd, out, ops.bn_workspace(npix, c, self.scratch, dev),
                                   bn.running_mean, bn.running_var, act=ACT_NONE, eps=bn.eps, momentum=bn.momentum,
                                   num_batches_tracked=bn.num_batches_tracked)
                    rec.update(mean=mean, rstd=rstd)
                else:
                    ops.bn_inference(t, npix, c, bn.running_mean, bn.running_var, bn.weight, bn.bias, out, act=ACT_NONE, eps=bn.eps)
            saved.append(rec)
            a, cs, hh, ww = out, c, oh, ow
        feat = cs * hh * ww
        if feat != self.feat:
            raise RuntimeError(f"Discriminator: flattened features {feat} != classification input {self.feat}; the reference "
                               f"architecture only runs on inputs that flatten to 8192 (128x128), discriminator.py:42-46")
        n_pad = (n + 31) // 32 * 32
        p = _bf16((n, feat), dev)
        p_t = torch.zeros((feat, n_pad), dtype=torch.bfloat16, device=dev) if need_pt else None
        ops.adaptive_pool_fwd(a, n, hh, ww, cs, hh, ww, p, p_t, n_pad)  # identity pool = torch's NCHW flatten
        hid = _f32((n, FC_PAD), dev)
        lin_ws = self._scr("linws", (1024 * n * FC_PAD,), torch.float32, dev)
        ops.linear_fwd(p, self.w0, self.b0, n, feat, FC_PAD, hid, lin_ws, act=ACT_NONE)
        s = _f32((n, 1), dev)
        ops.d_head_fwd(hid, self.w1, d.classification[1].bias, n, FC_PAD, s, sigmoid=False)
        sv = None
        if keep:
            sv = dict(n=n, h=h, w=w, layers=saved, p_t=p_t, hid=hid, s=s, n_pad=n_pad, feat=feat, hh=hh, ww=ww, c=cs)
        return s, sv

    # ------------------------------------------------------------------ backward
    def backward(self, ds: Tensor, sv: dict, need_w: bool, need_x: bool, accumulate: bool):
        d = self.d
        dev = ds.device
        n, n_pad, feat = sv["n"], sv["n_pad"], sv["feat"]
        fc0, fc1 = d.classification[0], d.classification[1]
        ds = ds.contiguous().float()
        acc = accumulate
        du0 = _bf16((n, FC_PAD), dev)
        du0_t = torch.zeros((FC_PAD, n_pad), dtype=torch.bfloat16, device=dev)
        dw1 = self._scr("dw1", (FC_PAD,), torch.float32, dev).zero_()  # scratch: the head kernel's accumulate flag
        db0 = self._scr("db0", (FC_PAD,), torch.float32, dev).zero_()  # must only affect the real bias gradient
        db1 = fc1.bias.grad if need_w else None
        ops.d_head_bwd(sv["hid"], sv["s"], ds, self.w1, n, FC_PAD, n_pad, dw1 if need_w else None, db1, db0 if need_w else None,
                       acc, du0, du0_t, slope=1.0, sigmoid=False)
        if need_w:
            dw0 = self._scr("dw0", (FC_PAD, feat), torch.float32, dev)
            ops.linear_wgrad(du0_t, sv["p_t"], n_pad, feat, FC_PAD, dw0, False)
            hd = self.hid
            if acc:
                fc0.weight.grad.add_(dw0[:hd])
                fc0.bias.grad.add_(db0[:hd])
                fc1.weight.grad.view(-1).add_(dw1[:hd])
            else:
                fc0.weight.grad.copy_(dw0[:hd])
                fc0.bias.grad.copy_(db0[:hd])
                fc1.weight.grad.view(-1).copy_(dw1[:hd])
        dp = self._scr("dp", (n, feat), torch.float32, dev)
        ops.linear_dgrad(du0, self.w0, n, feat, FC_PAD, dp)
        hh, ww, c = sv["hh"], sv["ww"], sv["c"]
        da = _f32((n, hh, ww, c), dev)
        ops.adaptive_pool_bwd(dp, n, hh, ww, c, hh, ww, da)
        coef = self._scr("bncoef", (3 * 512,), torch.float32, dev)
        dx = None
        for li in reversed(range(len(self.layers))):
            L = self.layers[li]
            R = sv["layers"][li]
            plan, conv, bn, slope = L["plan"], L["conv"], L["bn"], L["slope"]
            oh, ow, c = R["oh"], R["ow"], plan.cout
            npix = n * oh * ow
            cz = (c + 7) // 8 * 8
            dz = _bf16((n, oh, ow, cz), dev)
            if bn is not None:  # d(BN input) through the LeakyReLU that produced it
                ops.bn_backward(da, R["t"], R["t"], npix, c, R["mean"], R["rstd"], bn.weight, ops.bn_workspace(npix, c, self.scratch, dev), coef,
                                bn.weight.grad if need_w else None, bn.bias.grad if need_w else None, acc, dz, slope=1.0,
                                out_slope=slope)
            elif slope is not None:
                ops.act_grad(npix, c, da, c, 0, R["t"], c, 0, ACT_LRELU, dz, cz, slope=slope)
            else:
                ops.act_grad(npix, c, da, c, 0, None, 0, 0, ACT_NONE, dz, cz)
            if need_w:
                plan.gw = conv.weight.grad
                plan.gb = conv.bias.grad
                plan.wgrad(R["src"], R["cs_in"], 0, R["sh"], R["sw"], dz, cz, n, self.ws, acc)
            if li > 0 or need_x:
                gp = _f32((n, R["sh"], R["sw"], plan.cin), dev)
                plan.dgrad(dz, cz, oh, ow, gp, plan.cin, 0, n)
                if L["rpad"]:
                    g = _f32((n, R["h_in"], R["w_in"], plan.cin), dev)
                    ops.reflect_pad1_bwd(gp, n, R["h_in"], R["w_in"], plan.cin, g)
                else:
                    g = gp
                da = g
            if li == 0 and need_x:
                dx = torch.empty((n, 1, sv["h"], sv["w"]), dtype=torch.float32, device=dev)
                ops.nhwc_to_nchw(da, n, 1, sv["h"], sv["w"], plan.cin, 0, dx)
        return dx


class _PlainDFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, box, *params):
        engine, keep, need_pt, via_autograd = box
        s, sv = engine.forward(x, keep, need_pt)
        ctx.engine, ctx.sv, ctx.via_autograd = engine, sv, via_autograd
        return s

    @staticmethod
    def backward(ctx, ds):
        engine, sv = ctx.engine, ctx.sv
        if sv is None:
            raise RuntimeError("discriminator forward ran without saving activations")
        need_w = any(ctx.needs_input_grad[2:])
        need_x = ctx.needs_input_grad[0]
        if need_w and ctx.via_autograd:  # torch DDP: the gradients go through AccumulateGrad (and the reducer's hooks)
            buf, prev = engine.d._begin_autograd_grads()
            dx = engine.backward(ds, sv, need_w, need_x, False)
            ctx.sv = None
            return (dx, None) + engine.d._end_autograd_grads(buf, prev, ctx.needs_input_grad[2:])
        acc = engine.d.grads_as_views() if need_w else True
        dx = engine.backward(ds, sv, need_w, need_x, acc)
        ctx.sv = None
        return (dx, None) + tuple(None for _ in range(len(ctx.needs_input_grad) - 2))


class Discriminator(FlatParamsMixin, nn.Module):
    """discriminator.py:5-46 (same members, keys and forward contract)."""

    def __init__(self, in_channels=1, out_channels=64, num_conv_block=4):
        super().__init__()
        block: List[nn.Module] = []
        for _ in range(num_conv_block):
            block += [nn.ReflectionPad2d(1), nn.Conv2d(in_channels, out_channels, 3), nn.LeakyReLU(), nn.BatchNorm2d(out_channels)]
            in_channels = out_channels
            block += [nn.ReflectionPad2d(1), nn.Conv2d(in_channels, out_channels, 3, 2), nn.LeakyReLU()]
            out_channels *= 2
        out_channels //= 2
        in_channels = out_channels
        block += [nn.Conv2d(in_channels, out_channels, 3), nn.LeakyReLU(0.2), nn.Conv2d(out_channels, out_channels, 3)]
        self.feature_extraction = nn.Sequential(*block)
        self.avgpool = nn.AdaptiveAvgPool2d((512, 512))
        self.classification = nn.Sequential(nn.Linear(8192, 100), nn.Linear(100, 1))
        self._flatten()
        object.__setattr__(self, "_engine", None)

    def _on_flat_moved(self):
        object.__setattr__(self, "_engine", None)

    def _apply(self, fn, recurse=True):
        ret = super()._apply(fn, recurse)
        object.__setattr__(self, "_engine", None)
        return ret

    def engine(self) -> _PlainDEngine:
        self._ensure_flat()
        if self._engine is None:
            object.__setattr__(self, "_engine", _PlainDEngine(self))
        return self._engine

    def repack_weights(self) -> None:
        self.engine().repack()

    def forward(self, x: Tensor) -> Tensor:
        if not x.is_cuda:
            raise RuntimeError("climsr_amd.Discriminator runs on the GPU only (no CPU fallback)")
        eng = self.engine()
        params = [p for p, _o, _n in self._flat_index]
        grad_on = torch.is_grad_enabled()
        need_w = grad_on and any(p.requires_grad for p in params)
        keep = grad_on and (need_w or x.requires_grad)
        return _PlainDFn.apply(x, (eng, keep, need_w, need_w and self._route_grads_through_autograd()), *params)
