"""RCAN generator (drop-in for ``climsr.models.rcan.RCAN``) -- native inference and training.

Same constructor kwargs (``n_resgroups, n_resblocks, n_feats, reduction, scaling_factor, in_channels,
out_channels, conv, **kwargs``; rcan.py:138-150), same submodule tree and ``state_dict`` keys
(``head.0``, ``body.{g}.body.{b}.body.{0,2}``, ``body.{g}.body.{b}.body.3.conv_du.{0,2}``,
``body.{g}.body.{n_resblocks}``, ``body.{n_resgroups}``, ``tail.0.{0,2}``, ``tail.1``, ``srcnn.conv{1,2,3}``),
same ``forward(x, elev, mask)`` (rcan.py:181-192) and the reference's lenient ``load_state_dict``
(rcan.py:194-219: shape-mismatched ``tail`` upsampler weights are skipped).

The forward runs entirely in libclimsr_hip.so: every conv on the MFMA implicit-GEMM kernels (bf16
NHWC activations, fp32 accumulation), the residual stream in fp32 with a bf16 shadow for the next
conv, channel attention as ``climsr_channel_attention`` + ``climsr_ca_scale_add`` (pool, 1x1-ReLU-1x1-
sigmoid, ``x * y + x`` in one pass), the group / body skips fused into the conv epilogues, the
Upsampler's ``nn.PixelShuffle`` as ``climsr_pixel_shuffle_bf16`` (bit-exact index map) and the SRCNN
tail as in the ESRGAN generator.

Training (the reference pre-trains RCAN with the L1 task, conf/experiment/rcan_pre_training.yaml:7,10): the forward
keeps every RCAB's conv input, ReLU output, body output, attention scale and pooled mean; the backward is one autograd
node like the ESRGAN generator's (parameters are views of one flat fp32 buffer, gradients of one flat gradient
buffer, core/flat.py): the SRCNN tail's fused backward, the Upsampler's convs with ``climsr_pixel_unshuffle_bf16`` (the
inverse PixelShuffle index map, bit-exact), then the body in reverse -- per RCAB ``climsr_ca_backward`` (sigmoid' x
scale through the two 1x1 convs and the average pool, rcan.py:50-69) and the two convs' weight / data gradients, the
residual adds (rcan.py:100,134,186) as fp32 epilogue operands of the data gradients.
"""
from __future__ import annotations

import logging
import math
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn
from torch import Tensor

from .. import _lib
from .._lib import check, ptr
from ..core.flat import FlatParamsMixin
from ..ops import ACT_NONE, ACT_RELU, ACT_RELU_BWD, OUT_BF16, OUT_F32, BatchedPacker, ConvPlan, SrcnnTail, Workspace, _launch, axpby, \
    nchw_to_nhwc
from .esrgan import _GeneratorFn
from .srcnn import SRCNN


def default_conv(in_channels: int, out_channels: int, kernel_size: int, bias: bool = True) -> nn.Module:
    return nn.Conv2d(in_channels, out_channels, kernel_size, padding=kernel_size // 2, bias=bias)


class Upsampler(nn.Sequential):
    """rcan.py:17-47 (conv -> PixelShuffle per x2 stage, or one x3 stage)."""

    def __init__(self, conv, scale: int, n_feat: int, bn: bool = False, act=False, bias: bool = True):
        m: List[nn.Module] = []
        if (scale & (scale - 1)) == 0:
            for _ in range(int(math.log(scale, 2))):
                m.append(conv(n_feat, 4 * n_feat, 3, bias))
                m.append(nn.PixelShuffle(2))
        elif scale == 3:
            m.append(conv(n_feat, 9 * n_feat, 3, bias))
            m.append(nn.PixelShuffle(3))
        else:
            raise NotImplementedError
        if bn or act:
            raise NotImplementedError("RCAN's Upsampler is built with bn=False, act=False (rcan.py:166)")
        super().__init__(*m)


class CALayer(nn.Module):
    def __init__(self, channel: int, reduction: int = 16):
        super().__init__()
        self.avg_pool = nn.AdaptiveAvgPool2d(1)
        self.conv_du = nn.Sequential(nn.Conv2d(channel, channel // reduction, 1, padding=0, bias=True), nn.ReLU(inplace=True),
                                     nn.Conv2d(channel // reduction, channel, 1, padding=0, bias=True), nn.Sigmoid())


class RCAB(nn.Module):
    def __init__(self, conv, n_feat: int, kernel_size: int, reduction: int, act: nn.Module, bias: bool = True, bn: bool = False,
                 res_scale: int = 1):
        super().__init__()
        self.body = nn.Sequential(conv(n_feat, n_feat, kernel_size, bias=bias), act, conv(n_feat, n_feat, kernel_size, bias=bias),
                                  CALayer(n_feat, reduction))
        self.res_scale = res_scale


class ResidualGroup(nn.Module):
    def __init__(self, conv, n_feat: int, kernel_size: int, reduction: int, n_resblocks: int):
        super().__init__()
        body: List[nn.Module] = [RCAB(conv, n_feat, kernel_size, reduction, bias=True, bn=False, act=nn.ReLU(True), res_scale=1)
                                 for _ in range(n_resblocks)]
        body.append(conv(n_feat, n_feat, kernel_size))
        self.body = nn.Sequential(*body)


class RCAN(FlatParamsMixin, nn.Module):
    def __init__(self, n_resgroups: int = 10, n_resblocks: int = 20, n_feats: int = 64, reduction: int = 16,
                 scaling_factor: int = 4, in_channels: int = 3, out_channels: int = 1, conv=default_conv, **kwargs):
        super().__init__()
        self.n_resgroups, self.n_resblocks, self.n_feats = n_resgroups, n_resblocks, n_feats
        self.kernel_size = 3
        self.reduction = reduction
        self.scaling_factor = scaling_factor
        self.in_channels, self.out_channels = in_channels, out_channels
        self.head = nn.Sequential(conv(in_channels, n_feats, self.kernel_size))
        body: List[nn.Module] = [ResidualGroup(conv, n_feats, self.kernel_size, reduction, n_resblocks=n_resblocks)
                                 for _ in range(n_resgroups)]
        body.append(conv(n_feats, n_feats, self.kernel_size))
        self.body = nn.Sequential(*body)
        self.tail = nn.Sequential(Upsampler(conv, scaling_factor, n_feats, act=False), conv(n_feats, out_channels, self.kernel_size))
        self.srcnn = SRCNN(in_channels=3, out_channels=out_channels)
        self._flatten()
        object.__setattr__(self, "_engine", None)

    def load_state_dict(self, state_dict: dict, strict: bool = False):
        """rcan.py:194-219: copy matching names; a shape mismatch is tolerated only for ``tail`` keys."""
        own = self.state_dict()
        with torch.no_grad():
            for name, param in state_dict.items():
                if name in own:
                    if isinstance(param, nn.Parameter):
                        param = param.data
                    try:
                        own[name].copy_(param)
                    except Exception:
                        if name.find("tail") >= 0:
                            logging.info("Replace pre-trained upsampler to new one...")
                        else:
                            raise RuntimeError(f"While copying the parameter named {name}, whose dimensions in the model are "
                                               f"{own[name].size()} and whose dimensions in the checkpoint are {param.size()}.")
                elif strict and name.find("tail") == -1:
                    raise KeyError(f'unexpected key "{name}" in state_dict')
            self._flat.add_(0)  # bump the flat buffer's version: the engine re-packs its bf16 weights at the next forward
        if strict:
            missing = set(own.keys()) - set(state_dict.keys())
            if missing:
                raise KeyError(f'missing keys in state_dict: "{missing}"')

    def _on_flat_moved(self):
        object.__setattr__(self, "_engine", None)

    def engine(self) -> "_RcanEngine":
        self._ensure_flat()
        eng = self._engine
        if eng is None or eng.gen is not self or eng.device != self._flat.device:
            eng = _RcanEngine(self)
            object.__setattr__(self, "_engine", eng)
        return eng

    def repack_weights(self) -> None:
        """Refresh the bf16 MFMA weight layouts after an in-place update of the fp32 master weights."""
        self.engine().repack()

    def _flat_params(self) -> List[nn.Parameter]:
        return [p for p, _o, _n in self._flat_index]

    def forward(self, x: Tensor, elev: Tensor, mask: Tensor) -> Tensor:
        if not x.is_cuda:
            raise RuntimeError("RCAN runs in libclimsr_hip.so: inputs and parameters must be on a CUDA device")
        eng = self.engine()
        params = self._flat_params()
        keep = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        if not keep:
            return eng.forward(x, elev, mask, keep=False)[0]
        return _GeneratorFn.apply(x, elev, mask, (eng, True, self._route_grads_through_autograd()), *params)


class _RcanEngine:
    """Native forward (inference, or training with the activations the backward needs kept) and backward of one RCAN."""

    def __init__(self, m: RCAN):
        self.gen = m
        self.device = m._flat.device
        self.nf = m.n_feats
        assert self.nf % 8 == 0, "n_feats must be a multiple of 8"
        self.cin_pad = (m.in_channels + 7) // 8 * 8
        self.plans: Dict[str, ConvPlan] = {}
        mods = dict(m.named_modules())
        self.mods = mods
        for name, mod in mods.items():
            if isinstance(mod, nn.Conv2d) and ".conv_du." not in name:
                p = ConvPlan(mod.in_channels, mod.out_channels, mod.kernel_size[0], mod.stride[0], mod.padding[0], name)
                # transposed (data-gradient) weights for every conv the backward runs through (not the head: its input
                # is the data)
                p.bind(mod.weight, mod.bias, need_t=(name != "head.0"))
                self.plans[name] = p
        self.ups: List[Tuple[str, int]] = []  # (conv name, shuffle factor)
        up = m.tail[0]
        for i, mod in enumerate(up):
            if isinstance(mod, nn.PixelShuffle):
                self.ups.append((f"tail.0.{i - 1}", mod.upscale_factor))
        self.packer = BatchedPacker(list(self.plans.values()), self.device)
        self.version = None
        self.ca_ws = None
        self.cab_ws = None
        self.ws = Workspace()
        self.scratch: Dict[str, Tensor] = {}
        # the SRCNN tail as one launch (csrc/srcnn.hip, as models/esrgan.py) where its shape is the fused kernel's
        sc = [self.plans.get(f"srcnn.conv{i}") for i in (1, 2, 3)]
        self.srcnn = None
        if (all(c is not None and c.bias is not None for c in sc) and m.out_channels == 1 and sc[0].cin_real <= 4 and
                sc[0].cout == 64 and sc[0].ks == 9 and sc[1].cout == 32 and sc[1].ks == 1 and sc[2].cout == 1 and sc[2].ks == 5 and
                all(c.stride == 1 and c.pad == c.ks // 2 for c in sc)):
            self.srcnn = SrcnnTail(sc, "srcnn")

    def _params_version(self):
        return self.gen._flat._version, self.gen._flat.data_ptr()

    def repack(self):
        self.packer.run()
        if self.srcnn is not None:
            self.srcnn.pack()
        self.version = self._params_version()

    def ensure_packed(self):
        if self._params_version() != self.version:
            self.repack()

    def bind_grads(self):
        for name, p in self.plans.items():
            mod = self.mods[name]
            p.gw = mod.weight.grad
            p.gb = mod.bias.grad if mod.bias is not None else None

    def _scratch(self, key, shape, dtype, zero=False):
        t = self.scratch.get(key)
        if t is None or tuple(t.shape) != tuple(shape) or t.device != self.device:
            t = (torch.zeros if zero else torch.empty)(shape, dtype=dtype, device=self.device)
            self.scratch[key] = t
        return t

    def forward(self, x: Tensor, elev: Tensor, mask: Tensor, keep: bool = False):
        """Returns (sr, saved): saved (keep = training) holds what the backward reads, None otherwise."""
        m, P, nf = self.gen, self.plans, self.nf
        n, cin, h, w = x.shape
        dev = x.device
        sf = m.scaling_factor
        hh, ww = h * sf, w * sf
        assert elev.shape == (n, 1, hh, ww) and mask.shape == (n, 1, hh, ww), "elev/mask must be [N,1,sH,sW]"
        if keep and (m.n_resgroups < 1 or m.n_resblocks < 1 or self.srcnn is None):
            raise NotImplementedError("native RCAN training needs n_resgroups >= 1, n_resblocks >= 1 and the climate SRCNN tail "
                                      "(in_channels <= 4, out_channels = 1)")
        self.ensure_packed()
        L = _lib.load()
        st = _lib.stream_ptr()
        bf = lambda *s: torch.empty(s, dtype=torch.bfloat16, device=dev)  # noqa: E731
        f32 = lambda *s: torch.empty(s, dtype=torch.float32, device=dev)  # noqa: E731
        lr = torch.zeros((n, h, w, self.cin_pad), dtype=torch.bfloat16, device=dev)
        nchw_to_nhwc(x.contiguous().float(), lr, self.cin_pad, 0)
        head = f32(n, h, w, nf)
        xb = bf(n, h, w, nf)
        P["head.0"].fwd(lr, self.cin_pad, 0, h, w, head, nf, 0, n, out_mode=OUT_F32, aux=xb, aux_cs=nf)
        xres = head.clone()
        xb_alt = None if keep else bf(n, h, w, nf)
        gin = f32(n, h, w, nf)
        t = bf(n, h, w, nf)
        s = f32(n, nf)
        mean = None
        ws_bytes = L.climsr_channel_attention_workspace(n, nf)
        if self.ca_ws is None or self.ca_ws.numel() * 8 < ws_bytes or self.ca_ws.device != dev:
            self.ca_ws = torch.empty((ws_bytes + 7) // 8, dtype=torch.float64, device=dev)
        # the RCAB's second conv pools its own output for the channel attention (per-tile channel sums in its epilogue,
        # the register-resident 64 -> 64 conv) when it can; else the pooling pass re-reads u
        cp_rows, cp_tpi = P["body.0.body.0.body.2"].ch_parts(nf, h, w, n, nf)
        cpart = f32(max(cp_rows, 1), nf)
        # u (the RCAB body's output) in bf16 when the conv pools it itself: the attention's mean comes from the fp32
        # values in the epilogue, only the scale-add reads u (half the bytes of the fp32 round trip)
        u_bf16 = bool(cp_rows)
        u = bf(n, h, w, nf) if u_bf16 else f32(n, h, w, nf)
        rcabs: List[List[tuple]] = []
        tail_in: List[Tensor] = []
        for g in range(m.n_resgroups):
            gin.copy_(xres)
            grp = []
            for b in range(m.n_resblocks):
                pre = f"body.{g}.body.{b}.body"
                if keep:  # every RCAB's conv input (xb), ReLU output (t), body output (u), scale (s), pooled mean: kept
                    t, s, mean = bf(n, h, w, nf), f32(n, nf), f32(n, nf)
                    u = bf(n, h, w, nf) if u_bf16 else f32(n, h, w, nf)
                P[f"{pre}.0"].fwd(xb, nf, 0, h, w, t, nf, 0, n, act=ACT_RELU)
                ca = self.mods[f"{pre}.3"].conv_du
                w1, b1, w2, b2 = ca[0].weight, ca[0].bias, ca[2].weight, ca[2].bias
                if cp_rows:
                    P[f"{pre}.2"].fwd(t, nf, 0, h, w, u, nf, 0, n, ch_part=cpart)
                    check(L.climsr_channel_attention_parts_mean(ptr(cpart), n, cp_tpi, h * w, nf, ptr(w1), ptr(b1), ptr(w2), ptr(b2),
                                                                w1.shape[0], ptr(self.ca_ws), ptr(s), ptr(mean), st),
                          f"channel attention {pre}")
                else:
                    P[f"{pre}.2"].fwd(t, nf, 0, h, w, u, nf, 0, n, out_mode=OUT_F32)
                    check(L.climsr_channel_attention_mean(ptr(u), n, h * w, nf, nf, ptr(w1), ptr(b1), ptr(w2), ptr(b2), w1.shape[0],
                                                          ptr(self.ca_ws), ptr(s), ptr(mean), st), f"channel attention {pre}")
                xb_out = bf(n, h, w, nf) if keep else xb
                check(L.climsr_ca_scale_add(ptr(u), int(u_bf16), nf, ptr(s), ptr(xres), ptr(xb_out), nf, n, h * w, nf, st),
                      f"rcab residual {pre}")
                if keep:
                    grp.append((xb, t, u, s, mean))
                xb = xb_out
            rcabs.append(grp)
            tail_in.append(xb)
            # group tail conv + group skip (rcan.py:133-135), fp32 stream + bf16 shadow.  The shadow goes to another
            # buffer: written in place, a tile's aux store would race the halo reads of its neighbours.
            xb_next = bf(n, h, w, nf) if keep else xb_alt
            P[f"body.{g}.body.{m.n_resblocks}"].fwd(xb, nf, 0, h, w, xres, nf, 0, n, res1=gin, res1_cs=nf, out_mode=OUT_F32,
                                                   aux=xb_next, aux_cs=nf)
            if not keep:
                xb_alt = xb
            xb = xb_next
        # body conv + global skip (rcan.py:185-186); only its bf16 form feeds the tail
        feat = bf(n, h, w, nf)
        P[f"body.{m.n_resgroups}"].fwd(xb, nf, 0, h, w, feat, nf, 0, n, res1=head, res1_cs=nf, out_mode=OUT_BF16)
        cur, ch, cw = feat, h, w
        ups_in = []
        for name, r in self.ups:
            ups_in.append((cur, ch, cw))
            c4 = P[name].cout
            t4 = bf(n, ch, cw, c4)
            P[name].fwd(cur, nf, 0, ch, cw, t4, c4, 0, n)
            nxt = bf(n, ch * r, cw * r, nf)
            check(L.climsr_pixel_shuffle_bf16(ptr(t4), n, ch, cw, nf, r, c4, ptr(nxt), nf, st), f"pixel shuffle {name}")
            cur, ch, cw = nxt, ch * r, cw * r
        assert (ch, cw) == (hh, ww)
        tail8 = [] if keep else None
        out = srcnn_tail(P, "tail.1", cur, nf, n, hh, ww, m.out_channels, elev, mask, self.srcnn, keep_tail=tail8)
        if not keep:
            return out, None
        saved = dict(n=n, h=h, w=w, hh=hh, ww=ww, lr=lr, rcabs=rcabs, tail_in=tail_in, xb_final=xb, ups_in=ups_in, hr_feat=cur,
                     tail8=tail8[0], u_bf16=u_bf16)
        return out, saved

    def backward(self, gout: Tensor, sv: dict, accumulate: bool) -> None:
        m, P, nf = self.gen, self.plans, self.nf
        n, h, w, hh, ww = sv["n"], sv["h"], sv["w"], sv["hh"], sv["ww"]
        acc, ws = accumulate, self.ws
        L = _lib.load()
        st = _lib.stream_ptr()
        gout = gout.contiguous().float()
        bf = lambda key, *s: self._scratch(key, s, torch.bfloat16)  # noqa: E731
        f32 = lambda key, *s: self._scratch(key, s, torch.float32)  # noqa: E731
        # ---- SRCNN tail (srcnn.py:13-18): conv3 / conv2 gradients and dZ1 in one launch that recomputes the forward; then
        #      conv1's weight gradient and the gradient of its input channel 0 (tail.1's output; elev / mask need none)
        dz1 = bf("dz1", n, hh, ww, 64)
        self.srcnn.bwd(sv["tail8"], 8, 0, n, hh, ww, gout, dz1, ws, acc)
        P["srcnn.conv1"].wgrad(sv["tail8"], 8, 0, hh, ww, dz1, 64, n, ws, acc)
        dz8 = self._scratch("dz8", (n, hh, ww, 8), torch.bfloat16, zero=True)  # channels 1..7 stay 0
        P["srcnn.conv1"].dgrad(dz1, 64, hh, ww, dz8, 8, 0, n, cout_t=1)
        # ---- tail.1 (the last conv, rcan.py:175)
        P["tail.1"].wgrad(sv["hr_feat"], nf, 0, hh, ww, dz8, 8, n, ws, acc)
        g_cur = bf("g_hr", n, hh, ww, nf)
        P["tail.1"].dgrad(dz8, 8, hh, ww, g_cur, nf, 0, n)
        # ---- Upsampler (rcan.py:28-33): PixelShuffle backward (the inverse index map), then the conv's gradients
        g_feat = f32("g_feat", n, h, w, nf)
        gfb = bf("g_feat_b", n, h, w, nf)
        for idx in reversed(range(len(self.ups))):
            name, r = self.ups[idx]
            xin, ch, cw = sv["ups_in"][idx]
            c4 = P[name].cout
            gt4 = bf(f"gt4_{idx}", n, ch, cw, c4)
            _launch(f"pixel unshuffle {name}", lambda: L.climsr_pixel_unshuffle_bf16(ptr(g_cur), n, ch, cw, nf, r, nf, ptr(gt4), c4, st),
                    nbytes=n * ch * cw * c4 * 4)
            P[name].wgrad(xin, nf, 0, ch, cw, gt4, c4, n, ws, acc)
            if idx == 0:  # the body output's gradient: fp32 (it also feeds the global skip) + the bf16 copy the convs read
                P[name].dgrad(gt4, c4, ch, cw, g_feat, nf, 0, n, aux=gfb, aux_cs=nf)
            else:
                g_cur = bf(f"g_up_{idx}", n, ch, cw, nf)
                P[name].dgrad(gt4, c4, ch, cw, g_cur, nf, 0, n)
        # ---- body conv (rcan.py:170,185-186): res = conv(x) + head
        ng, nbk = m.n_resgroups, m.n_resblocks
        G = [f32(f"G{k}", n, h, w, nf) for k in range(3)]
        GB = [bf(f"GB{k}", n, h, w, nf) for k in range(2)]
        P[f"body.{ng}"].wgrad(sv["xb_final"], nf, 0, h, w, gfb, nf, n, ws, acc)
        io, ic, ii, bo = 0, 1, 2, 0
        P[f"body.{ng}"].dgrad(gfb, nf, h, w, G[io], nf, 0, n, aux=GB[bo], aux_cs=nf)
        hw = h * w
        cr = nf // m.reduction
        need = int(L.climsr_ca_backward_workspace(n, hw, nf, cr))
        if self.cab_ws is None or self.cab_ws.numel() < need or self.cab_ws.device != gout.device:
            self.cab_ws = torch.empty(need, dtype=torch.uint8, device=gout.device)
        gu, gt = bf("gu", n, h, w, nf), bf("gt", n, h, w, nf)
        for g in reversed(range(ng)):
            # ---- residual group (rcan.py:132-135): out = tail_conv(RCABs(x)) + x.  G[io] = dL/d(out), GB[bo] its bf16 copy
            tname = f"body.{g}.body.{nbk}"
            P[tname].wgrad(sv["tail_in"][g], nf, 0, h, w, GB[bo], nf, n, ws, acc)
            P[tname].dgrad(GB[bo], nf, h, w, G[ic], nf, 0, n)  # G[ic] = dL/d(output of the last RCAB)
            if g == 0:  # the head output also feeds the global skip (rcan.py:186): its gradient joins group 0's skip
                axpby(n * hw, nf, 1.0, g_feat, nf, 0, 1.0, G[io], nf, 0)
            for b in reversed(range(nbk)):
                pre = f"body.{g}.body.{b}.body"
                xb_in, t, u, s, mean = sv["rcabs"][g][b]
                ca = self.mods[f"{pre}.3"].conv_du
                w1, b1, w2 = ca[0].weight, ca[0].bias, ca[2].weight
                gw1, gb1, gw2, gb2 = ca[0].weight.grad, ca[0].bias.grad, ca[2].weight.grad, ca[2].bias.grad
                # RCAB (rcan.py:98-101): y = u * s + x.  dL/du (bf16) and the conv_du gradients from dL/dy = G[ic]
                _launch(f"ca backward {pre}", lambda: L.climsr_ca_backward(
                    ptr(G[ic]), nf, ptr(u), int(sv["u_bf16"]), nf, ptr(s), ptr(mean), n, hw, nf, ptr(w1), ptr(b1), ptr(w2), cr,
                    ptr(gw1), ptr(gb1), ptr(gw2), ptr(gb2), int(acc), ptr(self.cab_ws), ptr(gu), nf, st),
                    nbytes=n * hw * nf * (4 + 2 * u.element_size() + 4 + 2))
                P[f"{pre}.2"].wgrad(t, nf, 0, h, w, gu, nf, n, ws, acc)
                P[f"{pre}.2"].dgrad(gu, nf, h, w, gt, nf, 0, n, act=ACT_RELU_BWD, res1=t, res1_cs=nf, res1_co=0)
                P[f"{pre}.0"].wgrad(xb_in, nf, 0, h, w, gt, nf, n, ws, acc)
                if b > 0:  # dL/dx = dL/dy + conv0^T(gt): accumulated in place
                    P[f"{pre}.0"].dgrad(gt, nf, h, w, G[ic], nf, 0, n, accumulate=True)
                else:  # the group input's gradient = conv0^T(gt) + dL/dy + the group skip's, with its bf16 copy
                    P[f"{pre}.0"].dgrad(gt, nf, h, w, G[ii], nf, 0, n, res1=G[ic], res1_cs=nf, res2=G[io], res2_cs=nf,
                                        aux=GB[1 - bo], aux_cs=nf)
            io, ic, ii, bo = ii, io, ic, 1 - bo
        # ---- head (rcan.py:163,184): its output's gradient = group 0's input gradient (global skip included)
        P["head.0"].wgrad(sv["lr"], self.cin_pad, 0, h, w, GB[bo], nf, n, ws, acc)


def srcnn_tail(P: Dict[str, ConvPlan], last: str, feat: Tensor, feat_cs: int, n: int, hh: int, ww: int, oc: int, elev: Tensor,
               mask: Tensor, fused: Optional[SrcnnTail] = None, keep_tail: Optional[list] = None) -> Tensor:
    """Last conv into channels [0, oc) of an 8-channel buffer, elev / mask after them (the torch.cat of rcan.py:190),
    then SRCNN (srcnn.py:13-18) with fused ReLUs: one launch (``fused``, csrc/srcnn.hip) or three convs.  keep_tail:
    a list the 8-channel buffer is appended to (the training backward reads it)."""
    dev = feat.device
    tail = torch.zeros((n, hh, ww, 8), dtype=torch.bfloat16, device=dev)
    P[last].fwd(feat, feat_cs, 0, hh, ww, tail, 8, 0, n)
    nchw_to_nhwc(elev.contiguous().float(), tail, 8, oc)
    nchw_to_nhwc(mask.contiguous().float(), tail, 8, oc + 1)
    if keep_tail is not None:
        keep_tail.append(tail)
    if fused is not None and oc == 1:
        out = torch.empty((n, 1, hh, ww), dtype=torch.float32, device=dev)
        fused.fwd(tail, 8, 0, n, hh, ww, out)
        return out
    s1 = torch.empty((n, hh, ww, 64), dtype=torch.bfloat16, device=dev)
    P["srcnn.conv1"].fwd(tail, 8, 0, hh, ww, s1, 64, 0, n, act=ACT_RELU)
    s2 = torch.empty((n, hh, ww, 32), dtype=torch.bfloat16, device=dev)
    P["srcnn.conv2"].fwd(s1, 64, 0, hh, ww, s2, 32, 0, n, act=ACT_RELU)
    out = torch.empty((n, oc, hh, ww), dtype=torch.float32, device=dev)
    if oc == 1:
        P["srcnn.conv3"].fwd(s2, 32, 0, hh, ww, out, 1, 0, n, out_mode=OUT_F32)
    else:
        tmp = torch.empty((n, hh, ww, oc), dtype=torch.float32, device=dev)
        P["srcnn.conv3"].fwd(s2, 32, 0, hh, ww, tmp, oc, 0, n, out_mode=OUT_F32)
        out.copy_(tmp.permute(0, 3, 1, 2))
    return out
