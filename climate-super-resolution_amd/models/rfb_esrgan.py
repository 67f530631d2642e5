"""RFB-ESRGAN discriminator (drop-in for ``climsr.models.rfb_esrgan.RFBESRGANDiscriminator``).

Same constructor (``in_channels=1``), same ``features`` / ``fc`` submodules and ``state_dict`` keys
(rfb_esrgan.py:26-61), ``forward(x: [N,1,H,W]) -> [N,1]`` in (0,1) (rfb_esrgan.py:63-69), honours
``.train()`` / ``.eval()`` (batch statistics + running-stat update vs running statistics).  All
arithmetic runs in libclimsr_hip: implicit-GEMM convs (stride 1/2; the stride-2 data gradient as a
stride-1 conv over the zero-inserted gradient), BatchNorm fused with LeakyReLU(0.2), the adaptive
16->14 average pool, fc.0 (100352->1024) on MFMA with split-K, and the LeakyReLU/fc.2/Sigmoid head.

Each call is one autograd node.  Weight/BN-affine gradients land in one flat fp32 buffer and are
only computed when the parameters require grad (Lightning toggles D off during the generator
update, pl_gan.py:63-79); the input gradient (into the generator) is computed when the input
requires grad.
"""
from __future__ import annotations

from typing import Dict, List

import torch
import torch.nn as nn
from torch import Tensor

from .. import ops
from ..core.flat import FlatParamsMixin
from ..ops import ACT_LRELU, ACT_LRELU_BWD, BatchedPacker, ConvPlan, Workspace

POOL = 14


def _bf16(shape, dev):
    return torch.empty(shape, dtype=torch.bfloat16, device=dev)


def _f32(shape, dev):
    return torch.empty(shape, dtype=torch.float32, device=dev)


class _DEngine:
    def __init__(self, d: "RFBESRGANDiscriminator"):
        self.d = d
        dev = d.fc[0].weight.device
        self.layers = []  # (conv module, bn module or None, ConvPlan)
        feats = list(d.features)
        for i, m in enumerate(feats):
            if isinstance(m, nn.Conv2d):
                bn = feats[i + 1] if i + 1 < len(feats) and isinstance(feats[i + 1], nn.BatchNorm2d) else None
                plan = ConvPlan(m.in_channels, m.out_channels, 3, m.stride[0], 1, f"features.{i}")
                plan.bind(m.weight, None, need_t=True)
                self.layers.append((m, bn, plan))
        self.packer = BatchedPacker([p for _c, _b, p in self.layers], dev)
        # fc.0's bf16 MFMA copy, row-major (written by the optimizer's AdamW pass, climsr_adamw_step_mirror)
        self.fc0_bf16 = torch.empty(tuple(d.fc[0].weight.shape), dtype=torch.bfloat16, device=dev)
        self.version = -1
        self.ws = Workspace()
        self.scratch: Dict[str, Tensor] = {}
        # the two D backwards of loss_d share one fc.0 weight-gradient launch (backward's defer)
        self._wpend = None

    def ensure_packed(self):
        v = self.d._flat._version
        if v != self.version:
            self.repack()

    def repack(self, mirror_done: bool = False):
        """mirror_done: the optimizer's AdamW pass already wrote fc0_bf16 (climsr_adamw_step_mirror)."""
        self.packer.run()
        if not mirror_done:
            ops.f32_to_bf16(self.d.fc[0].weight, self.fc0_bf16)
        self.version = self.d._flat._version

    def _scr(self, key, shape, dtype, dev):
        t = self.scratch.get(key)
        if t is None or tuple(t.shape) != tuple(shape) or t.device != dev:
            t = torch.empty(shape, dtype=dtype, device=dev)
            self.scratch[key] = t
        return t

    # ------------------------------------------------------------------ forward
    def forward(self, x: Tensor, keep: bool, need_pt: bool):
        d = self.d
        n, cin, h, w = x.shape
        dev = x.device
        self.ensure_packed()
        if keep:
            # a held fc.0 weight gradient still pending here belongs to a backward that never finished (the pass's
            # end-of-pass callback did not run): drop it, so it cannot merge into the next pass's gradient
            self._wpend = None
        cpad = (cin + 7) // 8 * 8
        xc = x.contiguous().float()
        if cpad == 8:  # channels 0..cin-1 + zero padding in one full-pixel pass
            x8 = torch.empty((n, h, w, 8), dtype=torch.bfloat16, device=dev)
            ops.pack_planes8([(xc, k) for k in range(cin)], n, h, w, x8)
        else:
            x8 = torch.zeros((n, h, w, cpad), dtype=torch.bfloat16, device=dev)
            ops.nchw_to_nhwc(xc, x8, cpad, 0)
        a_prev, cs_prev, hh, ww = x8, cpad, h, w
        saved = []
        training = d.training
        # features.0 + features.2 as one launch (csrc/stem.hip): features.0's 64-channel output is recomputed from the
        # image where features.2 reads it and written only when the backward needs it
        stem = None
        (c0, bn0, p0), (c1, bn1, p1) = self.layers[0], self.layers[1]
        if (cin == 1 and bn0 is None and bn1 is not None and p0.cout == 64 and p1.cin_real == 64 and p1.cout == 64 and p1.stride == 2
                and p1.kpk == 576):
            oh, ow = p1.out_hw(h, w)
            a0 = _bf16((n, h, w, 64), dev) if keep else None
            z = _bf16((n, oh, ow, 64), dev)
            nparts = ops.d_stem_s2_bn_parts(n, h, w) if training else 0
            part = self._scr("bnpart1", (max(nparts, 1) * 2 * 64,), torch.float64, dev) if nparts else None
            ops.d_stem_s2(x8, cpad, c0.weight, p1, a0, z, part, n, h, w, slope=0.2)
            saved.append(dict(a_in=x8, cs_in=cpad, h_in=h, w_in=w, z=None, a=a0, mean=None, rstd=None, oh=h, ow=w))
            stem = (z, part, nparts, oh, ow)
        for li, (conv, bn, plan) in enumerate(self.layers):
            if stem is not None and li == 0:
                a_prev, cs_prev = saved[0]["a"], 64  # (None when not kept: nothing reads it then)
                continue
            oh, ow = plan.out_hw(hh, ww)
            c = plan.cout
            if bn is None:
                a = _bf16((n, oh, ow, c), dev)
                plan.fwd(a_prev, cs_prev, 0, hh, ww, a, c, 0, n, act=ACT_LRELU, use_bias=False)
                saved.append(dict(a_in=a_prev, cs_in=cs_prev, h_in=hh, w_in=ww, z=None, a=a, mean=None, rstd=None, oh=oh, ow=ow))
            else:
                a = _bf16((n, oh, ow, c), dev)
                npix = n * oh * ow
                if stem is not None and li == 1:  # z and its BatchNorm partials came from the stem launch
                    z, part, nparts, _oh, _ow = stem
                else:
                    z = _bf16((n, oh, ow, c), dev)
                    # train mode: the conv epilogue emits the batch statistics' partial sums (no pass over z for them)
                    nparts = plan.bn_parts(cs_prev, hh, ww, n, c) if training else 0
                    part = self._scr(f"bnpart{len(saved)}", (max(nparts, 1) * 2 * c,), torch.float64, dev) if nparts else None
                    plan.fwd(a_prev, cs_prev, 0, hh, ww, z, c, 0, n, use_bias=False, bn_part=part)
                if training:
                    mean, rstd = _f32((c,), dev), _f32((c,), dev)
                    if nparts:
                        ops.bn_forward_parts(part, nparts, z, npix, c, bn.weight, bn.bias, mean, rstd, a, bn.running_mean,
                                             bn.running_var, eps=bn.eps, momentum=bn.momentum,
                                             num_batches_tracked=bn.num_batches_tracked)
                    else:
                        ops.bn_forward(z, npix, c, bn.weight, bn.bias, mean, rstd, a, ops.bn_workspace(npix, c, self.scratch, dev),
                                       bn.running_mean, bn.running_var, eps=bn.eps, momentum=bn.momentum,
                                       num_batches_tracked=bn.num_batches_tracked)
                else:
                    mean = rstd = None
                    ops.bn_inference(z, npix, c, bn.running_mean, bn.running_var, bn.weight, bn.bias, a, eps=bn.eps)
                saved.append(dict(a_in=a_prev, cs_in=cs_prev, h_in=hh, w_in=ww, z=z, a=a, mean=mean, rstd=rstd, oh=oh, ow=ow))
            a_prev, cs_prev, hh, ww = a, c, oh, ow
        c = cs_prev
        feat = c * POOL * POOL
        n_pad = (n + 31) // 32 * 32
        p = _bf16((n, feat), dev)
        p_t = torch.zeros((feat, n_pad), dtype=torch.bfloat16, device=dev) if need_pt else None
        ops.adaptive_pool_fwd(a_prev, n, hh, ww, c, POOL, POOL, p, p_t, n_pad)
        fc0, fc2 = d.fc[0], d.fc[2]
        hid = _f32((n, fc0.out_features), dev)
        nsplit_max = 3072 // ((fc0.out_features + 63) // 64) + 1
        lin_ws = self._scr("linws", (nsplit_max * n * fc0.out_features,), torch.float32, dev)
        ops.linear_fwd(p, self.fc0_bf16, fc0.bias, n, feat, fc0.out_features, hid, lin_ws, act=ACT_LRELU, slope=0.2)
        s = _f32((n, 1), dev)
        ops.d_head_fwd(hid, fc2.weight, fc2.bias, n, fc0.out_features, s)
        sv = None
        if keep:
            sv = dict(n=n, h=h, w=w, cpad=cpad, layers=saved, p_t=p_t, hid=hid, s=s, n_pad=n_pad, feat=feat, hh=hh, ww=ww, c=c)
        return s, sv

    # ------------------------------------------------------------------ backward
    def flush_wgrad(self):
        """Launch a held fc.0 weight gradient (backward's defer) that no second call of the pass picked up."""
        pend, self._wpend = self._wpend, None
        if pend is not None:
            du0_t, p_t, n_pad, w0g, acc, feat, o, stream = pend
            with torch.cuda.stream(stream):
                ops.linear_wgrad(du0_t, p_t, n_pad, feat, o, w0g, acc)

    def backward(self, ds: Tensor, sv: dict, need_w: bool, need_x: bool, accumulate: bool, defer: bool = False):
        d = self.d
        dev = ds.device
        n, n_pad, feat = sv["n"], sv["n_pad"], sv["feat"]
        fc0, fc2 = d.fc[0], d.fc[2]
        o = fc0.out_features
        ds = ds.contiguous().float()
        du0 = _bf16((n, o), dev)
        du0_t = torch.zeros((o, n_pad), dtype=torch.bfloat16, device=dev)
        acc = accumulate
        ops.d_head_bwd(sv["hid"], sv["s"], ds, fc2.weight, n, o, n_pad, fc2.weight.grad if need_w else None,
                       fc2.bias.grad if need_w else None, fc0.bias.grad if need_w else None, acc, du0, du0_t)
        # grad-ready reports (core/ddp.OverlappedGradAllReducer): only in the step's last weight-gradient backward
        # (loss_d runs D twice, pl_gan.py:51-61), where each slice below becomes final
        hook = d._grad_ready_hook if need_w else None
        if hook is not None:
            calls = d._ready_calls + 1
            object.__setattr__(d, "_ready_calls", 0 if calls >= d._ready_need else calls)
            if calls < d._ready_need:
                hook = None
        if need_w:
            w0g = fc0.weight.grad
            pend = self._wpend
            if pend is not None and (pend[3].data_ptr() != w0g.data_ptr() or pend[2] % 32 or n_pad % 32):
                self.flush_wgrad()
                pend = None
            if pend is not None:  # the pass's other D call: one weight-gradient launch for both batches
                self._wpend = None
                ops.linear_wgrad2(pend[0], pend[1], pend[2], du0_t, sv["p_t"], n_pad, feat, o, w0g, pend[4])
            elif defer and hook is None:
                # loss_d backpropagates through D twice in one pass (real and fake, pl_gan.py:51-61): hold this call's
                # fc.0 operands so the next call writes the 411 MB gradient once; a pass with no second call launches
                # it from the end-of-pass callback, on this call's stream
                self._wpend = (du0_t, sv["p_t"], n_pad, w0g, acc, feat, o, torch.cuda.current_stream(dev))
                torch.autograd.Variable._execution_engine.queue_callback(self.flush_wgrad)
            else:
                ops.linear_wgrad(du0_t, sv["p_t"], n_pad, feat, o, w0g, acc)
            if hook is not None:  # fc.0 / fc.2: the last flat entries, 103 M of 107 M parameters
                hook(d._fc_flat_lo())
        dp = self._scr("dp", (n, feat), torch.float32, dev)
        ops.linear_dgrad(du0, self.fc0_bf16, n, feat, o, dp)
        hh, ww, c = sv["hh"], sv["ww"], sv["c"]
        da = _f32((n, hh, ww, c), dev)
        ops.adaptive_pool_bwd(dp, n, hh, ww, c, POOL, POOL, da)
        coef = self._scr("bncoef", (3 * 512,), torch.float32, dev)
        dx = None
        dz_next = None  # layer 0's output gradient, written directly by layer 1's data gradient
        fused = {}  # layer -> (part, nparts): its BN backward statistics, from the next layer's data-gradient epilogue
        for li in reversed(range(len(self.layers))):
            conv, bn, plan = self.layers[li]
            L = sv["layers"][li]
            oh, ow, c = L["oh"], L["ow"], plan.cout
            npix = n * oh * ow
            cz = (c + 7) // 8 * 8
            if bn is not None:
                # lrelu'(a) recomputed from z: the activation is not read; da is the bf16 data gradient of the
                # next conv (fp32 only for the last layer, from the pooling backward)
                dz = _bf16((n, oh, ow, cz), dev)
                if li in fused:
                    part, nparts = fused.pop(li)
                    ops.bn_backward_parts(part, nparts, da, L["z"], npix, c, L["mean"], L["rstd"], bn.weight, bn.bias, coef,
                                          bn.weight.grad if need_w else None, bn.bias.grad if need_w else None, acc, dz)
                else:
                    ops.bn_backward_z(da, L["z"], npix, c, L["mean"], L["rstd"], bn.weight, bn.bias,
                                      ops.bn_workspace(npix, c, self.scratch, dev), coef,
                                      bn.weight.grad if need_w else None, bn.bias.grad if need_w else None, acc, dz)
            elif dz_next is not None:
                dz = dz_next
            else:
                dz = _bf16((n, oh, ow, cz), dev)
                ops.act_grad(npix, c, da, c, 0, L["a"], c, 0, ACT_LRELU, dz, cz)
            if need_w:
                plan.gw = conv.weight.grad
                plan.gb = None
                plan.wgrad(L["a_in"], L["cs_in"], 0, L["h_in"], L["w_in"], dz, cz, n, self.ws, acc)
                if hook is not None and li in d._ready_layers:  # this layer group's conv + BN gradients are final
                    hook(d._layer_flat_lo(li))
            if li > 0 or need_x:
                prev_bn = self.layers[li - 1][1] if li > 0 else None
                if prev_bn is None and li > 0:
                    # the previous layer has no BN (layer 0): its LeakyReLU' (from its stored bf16 activation) goes
                    # into this data gradient's epilogue, which writes that layer's bf16 output gradient
                    P0 = sv["layers"][li - 1]
                    g = _bf16((n, L["h_in"], L["w_in"], plan.cin), dev)
                    plan.dgrad(dz, cz, oh, ow, g, plan.cin, 0, n, act=ACT_LRELU_BWD, res1=P0["a"], res1_cs=plan.cin, res1_co=0)
                    dz_next = g
                elif li > 0:
                    g = _bf16((n, L["h_in"], L["w_in"], plan.cin), dev)  # bf16: read by the previous layer's BN backward
                    P = sv["layers"][li - 1]
                    # that BN's backward statistics (sum d, sum d * xhat) come from this data gradient's epilogue
                    # where its kernel supports them: the separate statistics pass over g and z is skipped
                    nparts = plan.dgrad_bn_parts(cz, oh, ow, plan.cin, n, plan.cin) if P["mean"] is not None else 0
                    if nparts:
                        part = self._scr(f"bnbwd{li - 1}", (nparts * 2 * plan.cin,), torch.float64, dev)
                        plan.dgrad(dz, cz, oh, ow, g, plan.cin, 0, n,
                                   bn_bwd=(part, P["z"], plan.cin, P["mean"], P["rstd"], prev_bn.weight, prev_bn.bias))
                        fused[li - 1] = (part, nparts)
                    else:
                        plan.dgrad(dz, cz, oh, ow, g, plan.cin, 0, n)
                else:
                    g = _f32((n, L["h_in"], L["w_in"], plan.cin), dev)
                    plan.dgrad(dz, cz, oh, ow, g, plan.cin, 0, n)
                da = g
            if li == 0 and need_x:
                dx = torch.empty((n, 1, sv["h"], sv["w"]), dtype=torch.float32, device=dev)
                ops.nhwc_to_nchw(da, n, 1, sv["h"], sv["w"], plan.cin, 0, dx)
        return dx


class _DFn(torch.autograd.Function):
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
        dx = engine.backward(ds, sv, need_w, need_x, acc, defer=True)
        ctx.sv = None
        return (dx, None) + tuple(None for _ in range(len(ctx.needs_input_grad) - 2))


class RFBESRGANDiscriminator(FlatParamsMixin, nn.Module):
    r"""The main architecture of the discriminator. Similar to VGG structure (rfb_esrgan.py:23-69)."""

    def __init__(self, in_channels=1):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2d(in_channels, 64, kernel_size=3, stride=1, padding=1, bias=False),
            nn.LeakyReLU(negative_slope=0.2, inplace=True),
            nn.Conv2d(64, 64, kernel_size=3, stride=2, padding=1, bias=False),
            nn.BatchNorm2d(64),
            nn.LeakyReLU(negative_slope=0.2, inplace=True),
            nn.Conv2d(64, 128, kernel_size=3, stride=1, padding=1, bias=False),
            nn.BatchNorm2d(128),
            nn.LeakyReLU(negative_slope=0.2, inplace=True),
            nn.Conv2d(128, 128, kernel_size=3, stride=2, padding=1, bias=False),
            nn.BatchNorm2d(128),
            nn.LeakyReLU(negative_slope=0.2, inplace=True),
            nn.Conv2d(128, 256, kernel_size=3, stride=1, padding=1, bias=False),
            nn.BatchNorm2d(256),
            nn.LeakyReLU(negative_slope=0.2, inplace=True),
            nn.Conv2d(256, 256, kernel_size=3, stride=2, padding=1, bias=False),
            nn.BatchNorm2d(256),
            nn.LeakyReLU(negative_slope=0.2, inplace=True),
            nn.Conv2d(256, 512, kernel_size=3, stride=1, padding=1, bias=False),
            nn.BatchNorm2d(512),
            nn.LeakyReLU(negative_slope=0.2, inplace=True),
            nn.Conv2d(512, 512, kernel_size=3, stride=2, padding=1, bias=False),
            nn.BatchNorm2d(512),
            nn.LeakyReLU(negative_slope=0.2, inplace=True),
        )
        self.avgpool = nn.AdaptiveAvgPool2d((POOL, POOL))
        self.fc = nn.Sequential(
            nn.Linear(512 * POOL * POOL, 1024),
            nn.LeakyReLU(negative_slope=0.2, inplace=True),
            nn.Linear(1024, 1),
            nn.Sigmoid(),
        )
        self._flatten()
        object.__setattr__(self, "_engine", None)
        object.__setattr__(self, "_grad_ready_hook", None)
        object.__setattr__(self, "_ready_calls", 0)
        object.__setattr__(self, "_ready_need", 1)
        # conv-tower slices reported during the last backward: layers 6-7 (3.5 M parameters), 3-5 (1.0 M); layers 0-2
        # (0.1 M) go with finish()
        object.__setattr__(self, "_ready_layers", (6, 3))

    def set_grad_ready_hook(self, fn, calls_per_step: int = 1) -> None:
        """Call ``fn(lo)`` during backward once the fc gradients (flat offsets >= lo; 103 M of the 107 M
        parameters, computed first) are final (core/ddp.OverlappedGradAllReducer): on the
        ``calls_per_step``-th weight-gradient backward of the step (the D loss backpropagates through two D
        calls, real and fake, pl_gan.py:51-61, so it passes 2).  ``fn=None`` removes it."""
        object.__setattr__(self, "_grad_ready_hook", fn)
        object.__setattr__(self, "_ready_calls", 0)
        object.__setattr__(self, "_ready_need", max(1, int(calls_per_step)))

    def bf16_mirror(self):
        """(flat offset, numel, bf16 buffer) of fc.0's weight: its row-major MFMA copy, written by the fused AdamW pass."""
        return self._fc_flat_lo(), self.fc[0].weight.numel(), self.engine().fc0_bf16

    def grad_ready_los(self):
        """The flat offsets the backward reports through the grad-ready hook, in its order (fc first, then the conv
        tower's layer groups from the top): every gradient at or above an offset is final when it is reported."""
        return [self._fc_flat_lo()] + [self._layer_flat_lo(li) for li in self._ready_layers]

    def _layer_flat_lo(self, li: int) -> int:
        """Flat offset of the li-th conv's weight (its BatchNorm follows it; later layers sit above it)."""
        convs = [m for m in self.features if isinstance(m, nn.Conv2d)]
        p = convs[li].weight
        for q, off, _n in self._flat_index:
            if q is p:
                return off
        raise KeyError(f"features conv {li} not in the flat parameter index")

    def _fc_flat_lo(self) -> int:
        p = self.fc[0].weight
        for q, off, _n in self._flat_index:
            if q is p:
                return off
        raise KeyError("fc.0.weight not in the flat parameter index")

    def _on_flat_moved(self):
        object.__setattr__(self, "_engine", None)

    def _apply(self, fn, recurse=True):
        ret = super()._apply(fn, recurse)
        object.__setattr__(self, "_engine", None)  # buffers (BN running stats) may have moved too
        return ret

    def engine(self) -> _DEngine:
        self._ensure_flat()
        if self._engine is None:
            object.__setattr__(self, "_engine", _DEngine(self))
        return self._engine

    def repack_weights(self, mirror_done: bool = False) -> None:
        self.engine().repack(mirror_done=mirror_done)

    def forward(self, input: Tensor) -> Tensor:
        if not input.is_cuda:
            raise RuntimeError("climsr_amd.RFBESRGANDiscriminator runs on the GPU only (no CPU fallback)")
        eng = self.engine()
        params = [p for p, _o, _n in self._flat_index]
        grad_on = torch.is_grad_enabled()
        need_w = grad_on and any(p.requires_grad for p in params)
        keep = grad_on and (need_w or input.requires_grad)
        return _DFn.apply(input, (eng, keep, need_w, need_w and self._route_grads_through_autograd()), *params)
