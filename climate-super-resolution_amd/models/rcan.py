"""RCAN generator (drop-in for ``climsr.models.rcan.RCAN``) -- native inference.

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
tail as in the ESRGAN generator.  Inference only: the reference runs RCAN from ``inference.py`` with
``net.eval()``; calling it in training mode with gradients enabled raises (no silent non-training).
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
from ..ops import ACT_RELU, OUT_BF16, OUT_F32, BatchedPacker, ConvPlan, SrcnnTail, nchw_to_nhwc
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


class RCAN(nn.Module):
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
        self._engine = None

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
        if strict:
            missing = set(own.keys()) - set(state_dict.keys())
            if missing:
                raise KeyError(f'missing keys in state_dict: "{missing}"')

    def forward(self, x: Tensor, elev: Tensor, mask: Tensor) -> Tensor:
        if torch.is_grad_enabled() and self.training and any(p.requires_grad for p in self.parameters()):
            raise NotImplementedError("native RCAN is inference-only in this build: call .eval() (as inference.py does) "
                                      "or run under torch.no_grad()")
        if not x.is_cuda:
            raise RuntimeError("RCAN runs in libclimsr_hip.so: inputs and parameters must be on a CUDA device")
        eng = self._engine
        if eng is None or eng.device != x.device:
            eng = _RcanEngine(self)
            object.__setattr__(self, "_engine", eng)
        return eng.forward(x, elev, mask)


class _RcanEngine:
    def __init__(self, m: RCAN):
        self.m = m
        self.device = m.head[0].weight.device
        self.nf = m.n_feats
        assert self.nf % 8 == 0, "n_feats must be a multiple of 8"
        self.cin_pad = (m.in_channels + 7) // 8 * 8
        self.plans: Dict[str, ConvPlan] = {}
        mods = dict(m.named_modules())
        self.mods = mods
        for name, mod in mods.items():
            if isinstance(mod, nn.Conv2d) and ".conv_du." not in name:
                p = ConvPlan(mod.in_channels, mod.out_channels, mod.kernel_size[0], mod.stride[0], mod.padding[0], name)
                p.bind(mod.weight, mod.bias, need_t=False)
                self.plans[name] = p
        self.ups: List[Tuple[str, int]] = []  # (conv name, shuffle factor)
        up = m.tail[0]
        for i, mod in enumerate(up):
            if isinstance(mod, nn.PixelShuffle):
                self.ups.append((f"tail.0.{i - 1}", mod.upscale_factor))
        self.packer = BatchedPacker(list(self.plans.values()), self.device)
        self.version = None
        self.ca_ws = None
        # the SRCNN tail as one launch (csrc/srcnn.hip, as models/esrgan.py) where its shape is the fused kernel's
        sc = [self.plans.get(f"srcnn.conv{i}") for i in (1, 2, 3)]
        self.srcnn = None
        if (all(c is not None and c.bias is not None for c in sc) and m.out_channels == 1 and sc[0].cin_real <= 4 and
                sc[0].cout == 64 and sc[0].ks == 9 and sc[1].cout == 32 and sc[1].ks == 1 and sc[2].cout == 1 and sc[2].ks == 5 and
                all(c.stride == 1 and c.pad == c.ks // 2 for c in sc)):
            self.srcnn = SrcnnTail(sc, "srcnn")

    def _params_version(self):
        return tuple(p._version for p in self.m.parameters()) + tuple(p.data_ptr() for p in self.m.parameters())

    def ensure_packed(self):
        v = self._params_version()
        if v != self.version:
            for name, p in self.plans.items():  # rebind in case parameters were replaced
                mod = self.mods[name]
                p.bind(mod.weight, mod.bias, need_t=False)
            self.packer = BatchedPacker(list(self.plans.values()), self.device)
            self.packer.run()
            if self.srcnn is not None:
                self.srcnn.pack()
            self.version = v

    def forward(self, x: Tensor, elev: Tensor, mask: Tensor) -> Tensor:
        m, P, nf = self.m, self.plans, self.nf
        n, cin, h, w = x.shape
        dev = x.device
        sf = m.scaling_factor
        hh, ww = h * sf, w * sf
        assert elev.shape == (n, 1, hh, ww) and mask.shape == (n, 1, hh, ww), "elev/mask must be [N,1,sH,sW]"
        self.ensure_packed()
        L = _lib.load()
        st = _lib.stream_ptr()
        npx = n * h * w
        bf = lambda *s: torch.empty(s, dtype=torch.bfloat16, device=dev)  # noqa: E731
        f32 = lambda *s: torch.empty(s, dtype=torch.float32, device=dev)  # noqa: E731
        lr = torch.zeros((n, h, w, self.cin_pad), dtype=torch.bfloat16, device=dev)
        nchw_to_nhwc(x.contiguous().float(), lr, self.cin_pad, 0)
        head = f32(n, h, w, nf)
        xb = bf(n, h, w, nf)
        P["head.0"].fwd(lr, self.cin_pad, 0, h, w, head, nf, 0, n, out_mode=OUT_F32, aux=xb, aux_cs=nf)
        xres = head.clone()
        xb_alt = bf(n, h, w, nf)
        gin = f32(n, h, w, nf)
        t = bf(n, h, w, nf)
        s = f32(n, nf)
        ws_bytes = L.climsr_channel_attention_workspace(n, nf)
        if self.ca_ws is None or self.ca_ws.numel() * 8 < ws_bytes or self.ca_ws.device != dev:
            self.ca_ws = torch.empty((ws_bytes + 7) // 8, dtype=torch.float64, device=dev)
        # the RCAB's second conv pools its own output for the channel attention (per-tile channel sums in its epilogue,
        # the register-resident 64 -> 64 conv) when it can; else the pooling pass re-reads u
        cp_rows, cp_tpi = P["body.0.body.0.body.2"].ch_parts(nf, h, w, n, nf)
        cpart = f32(max(cp_rows, 1), nf)
        # u (the RCAB body's output) in bf16 when the conv pools it itself: the attention's mean comes from the fp32
        # values in the epilogue, only the scale-add reads u (half the bytes of the fp32 round trip)
        u = bf(n, h, w, nf) if cp_rows else f32(n, h, w, nf)
        for g in range(m.n_resgroups):
            gin.copy_(xres)
            for b in range(m.n_resblocks):
                pre = f"body.{g}.body.{b}.body"
                P[f"{pre}.0"].fwd(xb, nf, 0, h, w, t, nf, 0, n, act=ACT_RELU)
                ca = self.mods[f"{pre}.3"].conv_du
                w1, b1, w2, b2 = ca[0].weight, ca[0].bias, ca[2].weight, ca[2].bias
                if cp_rows:
                    P[f"{pre}.2"].fwd(t, nf, 0, h, w, u, nf, 0, n, ch_part=cpart)
                    check(L.climsr_channel_attention_parts(ptr(cpart), n, cp_tpi, h * w, nf, ptr(w1), ptr(b1), ptr(w2), ptr(b2),
                                                           w1.shape[0], ptr(self.ca_ws), ptr(s), st), f"channel attention {pre}")
                else:
                    P[f"{pre}.2"].fwd(t, nf, 0, h, w, u, nf, 0, n, out_mode=OUT_F32)
                    check(L.climsr_channel_attention(ptr(u), n, h * w, nf, nf, ptr(w1), ptr(b1), ptr(w2), ptr(b2), w1.shape[0],
                                                     ptr(self.ca_ws), ptr(s), st), f"channel attention {pre}")
                check(L.climsr_ca_scale_add(ptr(u), int(bool(cp_rows)), nf, ptr(s), ptr(xres), ptr(xb), nf, n, h * w, nf, st),
                      f"rcab residual {pre}")
            # group tail conv + group skip (rcan.py:133-135), fp32 stream + bf16 shadow.  The shadow goes to the other
            # buffer of a pair: written in place, a tile's aux store would race the halo reads of its neighbours.
            P[f"body.{g}.body.{m.n_resblocks}"].fwd(xb, nf, 0, h, w, xres, nf, 0, n, res1=gin, res1_cs=nf, out_mode=OUT_F32,
                                                   aux=xb_alt, aux_cs=nf)
            xb, xb_alt = xb_alt, xb
        # body conv + global skip (rcan.py:185-186); only its bf16 form feeds the tail
        feat = bf(n, h, w, nf)
        P[f"body.{m.n_resgroups}"].fwd(xb, nf, 0, h, w, feat, nf, 0, n, res1=head, res1_cs=nf, out_mode=OUT_BF16)
        cur, ch, cw = feat, h, w
        for name, r in self.ups:
            c4 = P[name].cout
            t4 = bf(n, ch, cw, c4)
            P[name].fwd(cur, nf, 0, ch, cw, t4, c4, 0, n)
            nxt = bf(n, ch * r, cw * r, nf)
            check(L.climsr_pixel_shuffle_bf16(ptr(t4), n, ch, cw, nf, r, c4, ptr(nxt), nf, st), f"pixel shuffle {name}")
            cur, ch, cw = nxt, ch * r, cw * r
        assert (ch, cw) == (hh, ww)
        return srcnn_tail(P, "tail.1", cur, nf, n, hh, ww, m.out_channels, elev, mask, self.srcnn)


def srcnn_tail(P: Dict[str, ConvPlan], last: str, feat: Tensor, feat_cs: int, n: int, hh: int, ww: int, oc: int, elev: Tensor,
               mask: Tensor, fused: Optional[SrcnnTail] = None) -> Tensor:
    """Last conv into channels [0, oc) of an 8-channel buffer, elev / mask after them (the torch.cat of rcan.py:190),
    then SRCNN (srcnn.py:13-18) with fused ReLUs: one launch (``fused``, csrc/srcnn.hip) or three convs."""
    dev = feat.device
    tail = torch.zeros((n, hh, ww, 8), dtype=torch.bfloat16, device=dev)
    P[last].fwd(feat, feat_cs, 0, hh, ww, tail, 8, 0, n)
    nchw_to_nhwc(elev.contiguous().float(), tail, 8, oc)
    nchw_to_nhwc(mask.contiguous().float(), tail, 8, oc + 1)
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
