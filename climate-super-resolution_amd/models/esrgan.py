"""ESRGAN RRDB generator (drop-in for ``climsr.models.esrgan.ESRGANGenerator``).

Same constructor kwargs (``in_channels, out_channels, nf, nb, gc, scaling_factor, **kwargs`` —
``scale_factor`` from conf/generator/default.yaml:3 is swallowed by **kwargs exactly as in the
reference, esrgan.py:58-67), same submodule names and ``state_dict`` keys, same
``forward(x, elev, mask)`` (esrgan.py:89-102).  The forward and backward run as one autograd
node whose arithmetic is entirely HIP (libclimsr_hip.so):

* one NHWC bf16 "dense" buffer of nf+4*gc channels per RDB holds x, x1..x4 (torch.cat of
  esrgan.py:34-37 is free: conv k reads channels [0, nf+(k-1)gc) and writes its gc outputs after
  them);
* conv5 fuses ``x5*0.2 + x`` (esrgan.py:38) and, in the third RDB of an RRDB, ``out*0.2 + x``
  (esrgan.py:54) into its epilogue; trunk_conv fuses the global skip (esrgan.py:91);
* the nearest x2 upsample (esrgan.py:94,97) is done on load by the following conv, and its
  backward (2x2 sum) in the dgrad epilogue;
* parameter gradients land in one flat fp32 buffer (core/flat.py).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.nn as nn
from torch import Tensor

from ..core.flat import FlatParamsMixin
from ..ops import (ACT_LRELU, ACT_LRELU_BWD, ACT_NONE, ACT_RELU, ACT_RELU_BWD, OUT_F32, BatchedPacker, ConvPlan, GroupedWgrad, PullPacker, PullPlan,
                   RdbChain, SrcnnTail, Workspace, act_grad, axpby, nchw_to_nhwc, pack_planes8)
from .srcnn import SRCNN


class ResidualDenseBlock(nn.Module):
    """Parameter container with the reference's names (esrgan.py:17-27)."""

    def __init__(self, nf=64, gc=32, bias=True):
        super().__init__()
        self.conv1 = nn.Conv2d(nf, gc, 3, 1, 1, bias=bias)
        self.conv2 = nn.Conv2d(nf + gc, gc, 3, 1, 1, bias=bias)
        self.conv3 = nn.Conv2d(nf + 2 * gc, gc, 3, 1, 1, bias=bias)
        self.conv4 = nn.Conv2d(nf + 3 * gc, gc, 3, 1, 1, bias=bias)
        self.conv5 = nn.Conv2d(nf + 4 * gc, nf, 3, 1, 1, bias=bias)
        self.lrelu = nn.LeakyReLU(negative_slope=0.2, inplace=True)

    def forward(self, x):  # pragma: no cover - the whole generator runs as one native node
        raise RuntimeError("ResidualDenseBlock runs inside ESRGANGenerator's native forward")


class ResidualInResidualDenseBlock(nn.Module):
    """esrgan.py:41-54."""

    def __init__(self, nf, gc=32):
        super().__init__()
        self.RDB1 = ResidualDenseBlock(nf, gc)
        self.RDB2 = ResidualDenseBlock(nf, gc)
        self.RDB3 = ResidualDenseBlock(nf, gc)

    def forward(self, x):  # pragma: no cover
        raise RuntimeError("ResidualInResidualDenseBlock runs inside ESRGANGenerator's native forward")


def _bf16(shape, dev):
    return torch.empty(shape, dtype=torch.bfloat16, device=dev)


def _f32(shape, dev):
    return torch.empty(shape, dtype=torch.float32, device=dev)


class _Engine:
    """Native forward/backward of one ESRGANGenerator (per device)."""

    def __init__(self, gen: "ESRGANGenerator"):
        self.gen = gen
        nf, gc, nb = gen.nf, gen.gc, gen.nb
        self.nf, self.gc, self.nb = nf, gc, nb
        self.dc = nf + 4 * gc
        assert nf % 8 == 0 and gc % 8 == 0, "nf and gc must be multiples of 8"
        self.cin = gen.in_channels
        self.cin_pad = (self.cin + 7) // 8 * 8
        self.plans: Dict[str, ConvPlan] = {}
        self.ws = Workspace()
        self.version = -1
        self.scratch: Dict[str, Tensor] = {}

        def add(name, conv: nn.Conv2d):
            p = ConvPlan(conv.in_channels, conv.out_channels, conv.kernel_size[0], conv.stride[0], conv.padding[0], name)
            self.plans[name] = p

        add("conv_first", gen.conv_first)
        for i, rrdb in enumerate(gen.RRDB_trunk):
            for r in (1, 2, 3):
                rdb = getattr(rrdb, f"RDB{r}")
                for c in range(1, 6):
                    add(f"RRDB_trunk.{i}.RDB{r}.conv{c}", getattr(rdb, f"conv{c}"))
        add("trunk_conv", gen.trunk_conv)
        add("upconv1", gen.upconv1)
        if gen.scale_factor == 4:
            add("upconv2", gen.upconv2)
        add("HRconv", gen.HRconv)
        add("conv_last", gen.conv_last)
        add("srcnn.conv1", gen.srcnn.conv1)
        add("srcnn.conv2", gen.srcnn.conv2)
        add("srcnn.conv3", gen.srcnn.conv3)
        self.modules = dict(gen.named_modules())
        self.bind()

    # ------------------------------------------------------------------ weights
    def bind(self):
        gen = self.gen
        nf, gc = self.nf, self.gc
        for name, p in self.plans.items():
            conv = self.modules[name]
            # RDB convs need no transposed weights: their data gradients run as pull convs (below)
            p.bind(conv.weight, conv.bias, need_t=(name != "conv_first" and ".RDB" not in name))
        dev = gen.conv_first.weight.device
        # conv1..conv4 of every RDB (and their pull gradients) as one fused row-streaming launch each (nf 64, gc 16:
        # csrc/rdb_chain.hip); other configurations run the four convs one by one (conv_n16)
        self.chains: List[RdbChain] = []
        if nf == 64 and gc == 16:
            for i in range(3 * self.nb):
                blk, r = divmod(i, 3)
                self.chains.append(RdbChain([self.plans[self.rdb_name(blk, r + 1, k)] for k in range(1, 6)],
                                            f"RRDB_trunk.{blk}.RDB{r + 1}"))
        self.packer = BatchedPacker(list(self.plans.values()), dev, [d for ch in self.chains for d in ch.pack_descs()])
        # Pull-form RDB backward: the dense concatenation's channel group j (0 = x, 1..4 = x1..x4) receives the
        # transposed convs of conv j+1..conv5, whose output gradients sit side by side in one buffer
        # dZ = [dZ1|dZ2|dZ3|dZ4|dZ5] (gc,gc,gc,gc,nf channels): group j's gradient is one conv over dZ[:, j*gc:].
        self.pulls: List[List[PullPlan]] = []
        for i in range(3 * self.nb):
            blk, r = divmod(i, 3)
            lst = []
            for j in range(5):
                segs = []
                for k in range(j + 1, 6):
                    w = self.modules[self.rdb_name(blk, r + 1, k)].weight
                    segs.append((w, gc if k < 5 else nf, nf + (k - 1) * gc))
                lst.append(PullPlan(segs, nf if j == 0 else gc, 0 if j == 0 else nf + (j - 1) * gc, 3,
                                    f"RRDB_trunk.{blk}.RDB{r + 1}.pull{j}"))
            self.pulls.append(lst)
        self.pull_packer = PullPacker([p for lst in self.pulls for p in (lst[:1] if self.chains else lst)], dev,
                                      [d for ch in self.chains for d in ch.pull_descs()])
        # the per-conv pulls 4..1 are packed only once a backward at a width the chain does not take needs them
        self.pull_packer_rest = PullPacker([p for lst in self.pulls for p in lst[1:]], dev) if self.chains else None
        self.pull_rest_on = False
        # the five weight gradients of an RDB: one GEMM over dZ (all dc channels) x the dense buffer (dc channels)
        self.rdb_wgrads: List[GroupedWgrad] = []
        for i in range(3 * self.nb if self.dc % 64 == 0 else 0):
            blk, r = divmod(i, 3)
            convs = [self.plans[self.rdb_name(blk, r + 1, k)] for k in range(1, 6)]
            self.rdb_wgrads.append(GroupedWgrad(convs, self.dc, f"RRDB_trunk.{blk}.RDB{r + 1}"))
        # the SRCNN tail as one launch (csrc/srcnn.hip) when its input is the climate cat[out, elev, mask] (<= 4 channels)
        tail = [self.plans[f"srcnn.conv{k}"] for k in (1, 2, 3)]
        self.srcnn_tail = SrcnnTail(tail) if tail[0].cin_real <= 4 and gen.out_channels == 1 and nf == 64 else None
        self.version = -1

    def bind_grads(self):
        for name, p in self.plans.items():
            conv = self.modules[name]
            p.gw = conv.weight.grad
            p.gb = conv.bias.grad if conv.bias is not None else None

    def ensure_packed(self):
        v = self.gen._flat._version
        if v != self.version:
            self.repack()

    def repack(self):
        self.packer.run()
        self.pull_packer.run()
        if self.pull_rest_on:
            self.pull_packer_rest.run()
        if self.srcnn_tail is not None:
            self.srcnn_tail.pack()
        self.version = self.gen._flat._version

    def chain_ok(self, w: int, n: int = 1, h: int = 1) -> bool:
        """The fused conv1-4 launch takes any image size whose buffers stay under 2 GiB (its 32-bit buffer offsets:
        climsr_rdb_chain rejects larger ones; the pull reads the dense buffer as its activation mask, same size);
        anything else runs conv by conv."""
        return bool(self.chains) and n * h * w * self.dc * 2 < (1 << 31)

    def _rdb_wgrad(self, i, src, dz, n, h, w, ws, acc):
        blk, r = divmod(i, 3)
        if self.dc % 64 == 0:
            self.rdb_wgrads[i].run(src, self.dc, 0, h, w, dz, self.dc, n, ws, acc)
        else:
            for k in range(1, 6):
                off = (k - 1) * self.gc
                self.plans[self.rdb_name(blk, r + 1, k)].wgrad(src, self.dc, 0, h, w, dz[..., off:], self.dc, n, ws, acc)

    def rdb_name(self, i, r, c):
        return f"RRDB_trunk.{i}.RDB{r}.conv{c}"

    def _scratch(self, key, shape, dtype, dev, zero=False):
        t = self.scratch.get(key)
        if t is None or tuple(t.shape) != tuple(shape) or t.device != dev:
            t = torch.zeros(shape, dtype=dtype, device=dev) if zero else torch.empty(shape, dtype=dtype, device=dev)
            self.scratch[key] = t
        return t

    # ------------------------------------------------------------------ forward
    def forward(self, x: Tensor, elev: Tensor, mask: Tensor, keep: bool):
        n, cin, h, w = x.shape
        dev = x.device
        nf, gc, dc, nb = self.nf, self.gc, self.dc, self.nb
        sf = self.gen.scale_factor
        h2, w2 = 2 * h, 2 * w
        hh, ww = (4 * h, 4 * w) if sf == 4 else (2 * h, 2 * w)
        assert elev.shape == (n, 1, hh, ww) and mask.shape == (n, 1, hh, ww), "elev/mask must be [N,1,sH,sW]"
        P = self.plans
        self.ensure_packed()
        x = x.contiguous().float()
        if self.cin_pad == 8:  # lr channels + zero padding in one full-pixel pass
            lr = torch.empty((n, h, w, 8), dtype=torch.bfloat16, device=dev)
            pack_planes8([(x, k) for k in range(x.shape[1])], n, h, w, lr)
        else:
            lr = torch.zeros((n, h, w, self.cin_pad), dtype=torch.bfloat16, device=dev)
            nchw_to_nhwc(x, lr, self.cin_pad, 0)
        # keep (training): every RDB's dense buffer is saved for the backward.  No-grad: a ring of three -- RDB i
        # reads ring[i % 3] and writes ring[(i + 1) % 3], so an RRDB's input ring[3 blk % 3] is still intact when its
        # third RDB's conv5 adds it (esrgan.py:54) and writes the result over it in place (the epilogue reads each
        # residual element before the same lane stores that element; conv5's conv input is another buffer)
        ndense = 3 * nb + 1 if keep else 3
        dense = [_bf16((n, h, w, dc), dev) for _ in range(ndense)]
        if keep:
            P["conv_first"].fwd(lr, self.cin_pad, 0, h, w, dense[0], dc, 0, n)
            fea = dense[0]
        else:  # fea (kept for the global skip, esrgan.py:91) and the first RDB's input in one launch (aux output)
            fea = _bf16((n, h, w, nf), dev)
            P["conv_first"].fwd(lr, self.cin_pad, 0, h, w, fea, nf, 0, n, aux=dense[0], aux_cs=dc, aux_co=0)
        for i in range(3 * nb):
            blk, r = divmod(i, 3)
            src = dense[i] if keep else dense[i % 3]
            dst = dense[i + 1] if keep else dense[(i + 1) % 3]
            if self.chain_ok(w, n, h):
                self.chains[i].forward(src, dc, n, h, w)
            else:
                for c in range(1, 5):
                    P[self.rdb_name(blk, r + 1, c)].fwd(src, dc, 0, h, w, src, dc, nf + (c - 1) * gc, n, act=ACT_LRELU)
            res2 = None
            if r == 2:
                res2 = dense[3 * blk] if keep else dense[(3 * blk) % 3]  # no-grad: == dst (in place)
            P[self.rdb_name(blk, r + 1, 5)].fwd(src, dc, 0, h, w, dst, dc, 0, n, res1=src, alpha1=0.2, res1_cs=dc, res1_co=0,
                                                 res2=res2, alpha2=0.2, res2_cs=dc, res2_co=0)
        last = dense[3 * nb] if keep else dense[(3 * nb) % 3]
        fea2 = _bf16((n, h, w, nf), dev)
        P["trunk_conv"].fwd(last, dc, 0, h, w, fea2, nf, 0, n, res1=fea, alpha1=1.0, res1_cs=(dc if keep else nf), res1_co=0)
        u1 = _bf16((n, h2, w2, nf), dev)
        P["upconv1"].fwd(fea2, nf, 0, h, w, u1, nf, 0, n, up=2, act=ACT_LRELU)
        if sf == 4:
            u2 = _bf16((n, hh, ww, nf), dev)
            P["upconv2"].fwd(u1, nf, 0, h2, w2, u2, nf, 0, n, up=2, act=ACT_LRELU)
        else:
            u2 = u1
        hr = _bf16((n, hh, ww, nf), dev)
        P["HRconv"].fwd(u2, nf, 0, hh, ww, hr, nf, 0, n, act=ACT_LRELU)
        tail = torch.zeros((n, hh, ww, 8), dtype=torch.bfloat16, device=dev)
        oc = self.gen.out_channels
        P["conv_last"].fwd(hr, nf, 0, hh, ww, tail, 8, 0, n)
        nchw_to_nhwc(elev.contiguous().float(), tail, 8, oc)
        nchw_to_nhwc(mask.contiguous().float(), tail, 8, oc + 1)
        out = torch.empty((n, oc, hh, ww), dtype=torch.float32, device=dev)
        s1 = s2 = None
        if self.srcnn_tail is not None:  # (its backward recomputes relu(conv1) / relu(conv2) from `tail`)
            self.srcnn_tail.fwd(tail, 8, 0, n, hh, ww, out)
        else:
            s1 = _bf16((n, hh, ww, 64), dev)
            P["srcnn.conv1"].fwd(tail, 8, 0, hh, ww, s1, 64, 0, n, act=ACT_RELU)
            s2 = _bf16((n, hh, ww, 32), dev)
            P["srcnn.conv2"].fwd(s1, 64, 0, hh, ww, s2, 32, 0, n, act=ACT_RELU)
            if oc == 1:
                P["srcnn.conv3"].fwd(s2, 32, 0, hh, ww, out, 1, 0, n, out_mode=OUT_F32)
            else:
                tmp = _f32((n, hh, ww, oc), dev)
                P["srcnn.conv3"].fwd(s2, 32, 0, hh, ww, tmp, oc, 0, n, out_mode=OUT_F32)
                out.copy_(tmp.permute(0, 3, 1, 2))
        saved = None
        if keep:
            saved = dict(n=n, h=h, w=w, hh=hh, ww=ww, lr=lr, dense=dense, fea2=fea2, u1=u1, u2=u2, hr=hr, tail=tail, s1=s1, s2=s2)
        return out, saved

    # ------------------------------------------------------------------ backward
    def backward(self, gout: Tensor, sv: dict, accumulate: bool) -> None:
        P = self.plans
        n, h, w, hh, ww = sv["n"], sv["h"], sv["w"], sv["hh"], sv["ww"]
        dev = gout.device
        nf, gc, dc, nb = self.nf, self.gc, self.dc, self.nb
        sf = self.gen.scale_factor
        h2, w2 = 2 * h, 2 * w
        acc = accumulate
        ws = self.ws
        oc = self.gen.out_channels
        assert oc == 1, "native backward implemented for out_channels=1 (the climate config)"
        npx_hr = n * hh * ww
        npx_lr = n * h * w
        gout = gout.contiguous().float()
        # HR-resolution output gradients stay bf16: every data gradient applies the next activation's
        # backward in its epilogue (no fp32 [N,4H,4W,64] intermediates, no separate act_grad passes)
        dzA = self._scratch("dzA", (n, hh, ww, nf), torch.bfloat16, dev)
        dzB = self._scratch("dzB", (n, hh, ww, nf), torch.bfloat16, dev)
        # ---- SRCNN tail (srcnn.py:13-18)
        if self.srcnn_tail is not None:
            # conv3 / conv2 gradients and dZ1 (into dzA) in one launch that recomputes the forward; dz8's channels 1..7
            # are never written (zero since allocation): conv1's data gradient below fills channel 0
            dz8 = self._scratch("dz8", (n, hh, ww, 8), torch.bfloat16, dev, zero=True)
            self.srcnn_tail.bwd(sv["tail"], 8, 0, n, hh, ww, gout, dzA, ws, acc)
        else:
            dz8 = self._scratch("dz8", (n, hh, ww, 8), torch.bfloat16, dev)
            dz32 = self._scratch("dz32", (n, hh, ww, 32), torch.bfloat16, dev)
            act_grad(npx_hr, 1, gout, 1, 0, None, 0, 0, ACT_NONE, dz8, 8)  # also zeroes dz8's pad channels
            P["srcnn.conv3"].wgrad(sv["s2"], 32, 0, hh, ww, dz8, 8, n, ws, acc)
            P["srcnn.conv3"].dgrad(dz8, 8, hh, ww, dz32, 32, 0, n, act=ACT_RELU_BWD, res1=sv["s2"], res1_cs=32, res1_co=0)
            P["srcnn.conv2"].wgrad(sv["s1"], 64, 0, hh, ww, dz32, 32, n, ws, acc)
            P["srcnn.conv2"].dgrad(dz32, 32, hh, ww, dzA, nf, 0, n, act=ACT_RELU_BWD, res1=sv["s1"], res1_cs=64, res1_co=0)
        P["srcnn.conv1"].wgrad(sv["tail"], 8, 0, hh, ww, dzA, 64, n, ws, acc)
        # only d(out) (tail channel 0) is needed; channels 1..7 of dz8 stay 0
        P["srcnn.conv1"].dgrad(dzA, 64, hh, ww, dz8, 8, 0, n, cout_t=1)
        # ---- conv_last / HRconv (esrgan.py:99)
        P["conv_last"].wgrad(sv["hr"], nf, 0, hh, ww, dz8, 8, n, ws, acc)
        P["conv_last"].dgrad(dz8, 8, hh, ww, dzA, nf, 0, n, act=ACT_LRELU_BWD, res1=sv["hr"], res1_cs=nf, res1_co=0)
        P["HRconv"].wgrad(sv["u2"], nf, 0, hh, ww, dzA, nf, n, ws, acc)
        # ---- upsampling (esrgan.py:94-97)
        dz_u1 = self._scratch("dz_u1", (n, h2, w2, nf), torch.bfloat16, dev)
        if sf == 4:
            P["HRconv"].dgrad(dzA, nf, hh, ww, dzB, nf, 0, n, act=ACT_LRELU_BWD, res1=sv["u2"], res1_cs=nf, res1_co=0)
            P["upconv2"].wgrad(sv["u1"], nf, 0, h2, w2, dzB, nf, n, ws, acc, up=2)
            P["upconv2"].dgrad(dzB, nf, hh, ww, dz_u1, nf, 0, n, down2=True, act=ACT_LRELU_BWD, res1=sv["u1"], res1_cs=nf,
                               res1_co=0)
        else:
            P["HRconv"].dgrad(dzA, nf, hh, ww, dz_u1, nf, 0, n, act=ACT_LRELU_BWD, res1=sv["u1"], res1_cs=nf, res1_co=0)
        g_fea2 = self._scratch("g_fea2", (n, h, w, nf), torch.float32, dev)
        dz64 = self._scratch("dz64", (n, h, w, nf), torch.bfloat16, dev)
        P["upconv1"].wgrad(sv["fea2"], nf, 0, h, w, dz_u1, nf, n, ws, acc, up=2)
        # fp32 gradient of fea2 (it also feeds the global skip) + its bf16 copy for trunk_conv's weight gradient
        P["upconv1"].dgrad(dz_u1, nf, h2, w2, g_fea2, nf, 0, n, down2=True, aux=dz64, aux_cs=nf, aux_co=0)
        # ---- trunk_conv + global skip (esrgan.py:90-91)
        dense = sv["dense"]
        L = 3 * nb
        P["trunk_conv"].wgrad(dense[L], dc, 0, h, w, dz64, nf, n, ws, acc)
        # G[k]: fp32 [n,h,w,nf] gradients at RDB boundaries (4-way rotation keeps each RRDB's skip gradient alive);
        # dZ[k]: bf16 [n,h,w,dc] output gradients of one RDB's five convs, side by side (ping-pong)
        G = [self._scratch(f"G{k}", (n, h, w, nf), torch.float32, dev) for k in range(4)]
        dZ = [self._scratch(f"dZ{k}", (n, h, w, dc), torch.bfloat16, dev) for k in range(2)]
        # the last RDB (r = 2) sees 0.2 * G at its output; its conv5 output gradient is 0.2 * that
        P["trunk_conv"].dgrad(dz64, nf, h, w, G[L % 4], nf, 0, n, aux=dZ[(L - 1) % 2], aux_cs=dc, aux_co=4 * gc, aux_scale=0.04)
        # ---- RRDB trunk, reverse (esrgan.py:32-54), pull form
        # (running RDB i's weight gradients on a second stream beside the pull-x / pull-chain launches measured 0.5 ms
        # SLOWER per GAN step than this serial order)
        for i in reversed(range(L)):
            blk, r = divmod(i, 3)
            s_o = 0.2 if r == 2 else 1.0  # RDB3's output enters the RRDB output scaled by 0.2 (esrgan.py:54)
            g_out, g_in, g_skip = G[(i + 1) % 4], G[i % 4], G[(3 * blk + 3) % 4]
            dz, src, pulls = dZ[i % 2], dense[i], self.pulls[i]
            # dZ_j = lrelu'(x_j) * sum_{k>j} conv_k^T(dZ_k)   (x_j = channels nf+(j-1)gc.. of the dense buffer)
            if self.chain_ok(w, n, h):
                self.chains[i].pull(dz, src, dc, n, h, w)
            else:
                if self.chains and not self.pull_rest_on:
                    self.pull_rest_on = True
                    self.pull_packer_rest.run()
                for j in (4, 3, 2, 1):
                    pulls[j].fwd(dz, dc, j * gc, h, w, dz, dc, (j - 1) * gc, n, act=ACT_LRELU_BWD, use_bias=False,
                                 res1=src, res1_cs=dc, res1_co=nf + (j - 1) * gc)
            # G_in = sum_k conv_k^T(dZ_k) + s_o * G_out (+ the RRDB skip gradient at its first RDB); the next
            # (earlier) RDB's conv5 output gradient dZ5 = 0.2 * s_o' * G_in is written alongside
            aux = dZ[(i - 1) % 2] if i > 0 else None
            pulls[0].fwd(dz, dc, 0, h, w, g_in, nf, 0, n, use_bias=False, out_mode=OUT_F32,
                         res1=g_out, res1_cs=nf, res1_co=0, beta1=s_o,
                         res2=g_skip if r == 0 else None, res2_cs=nf, res2_co=0,
                         aux=aux, aux_cs=dc, aux_co=4 * gc, aux_scale=0.2 * (0.2 if r == 0 else 1.0))
            self._rdb_wgrad(i, src, dz, n, h, w, ws, acc)
            hook = self.gen._grad_ready_hook
            if hook is not None and r == 0 and blk in self.gen._grad_ready_blocks:
                # every gradient from RRDB_trunk.<blk> on (flat order: trunk blocks, tail convs) is final
                hook(self.gen._block_flat_lo(blk))
        # ---- conv_first: grad wrt fea = trunk path + global skip
        axpby(npx_lr, nf, 1.0, g_fea2, nf, 0, 1.0, G[0], nf, 0)
        act_grad(npx_lr, nf, G[0], nf, 0, None, 0, 0, ACT_NONE, dz64, nf)
        P["conv_first"].wgrad(sv["lr"], self.cin_pad, 0, h, w, dz64, nf, n, ws, acc)


class _GeneratorFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, elev, mask, engine_box, *params):
        engine, keep, via_autograd = engine_box  # grad mode is off inside Function.forward: decided by the caller
        out, saved = engine.forward(x, elev, mask, keep=keep)
        ctx.engine = engine
        ctx.saved = saved
        ctx.via_autograd = via_autograd
        return out

    @staticmethod
    def backward(ctx, gout):
        engine = ctx.engine
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1] or ctx.needs_input_grad[2]:
            raise NotImplementedError("gradient w.r.t. the generator inputs is not implemented (never needed by the task)")
        if ctx.saved is None:
            raise RuntimeError("generator forward ran without saving activations")
        gen = engine.gen
        if ctx.via_autograd:  # torch DDP: the gradients go through AccumulateGrad (and the reducer's hooks)
            buf, prev = gen._begin_autograd_grads()
            engine.bind_grads()
            engine.backward(gout, ctx.saved, accumulate=False)
            ctx.saved = None
            return (None, None, None, None) + gen._end_autograd_grads(buf, prev, ctx.needs_input_grad[4:])
        acc = gen.grads_as_views()
        engine.bind_grads()
        engine.backward(gout, ctx.saved, accumulate=acc)
        ctx.saved = None
        return (None, None, None, None) + tuple(None for _ in range(len(ctx.needs_input_grad) - 4))


class ESRGANGenerator(FlatParamsMixin, nn.Module):
    def __init__(self, in_channels: int = 3, out_channels: int = 3, nf: int = 64, nb: int = 23, gc: int = 32,
                 scaling_factor: int = 4, **kwargs):
        super().__init__()
        self.scale_factor = scaling_factor
        self.in_channels, self.out_channels, self.nf, self.nb, self.gc = in_channels, out_channels, nf, nb, gc
        self.conv_first = nn.Conv2d(in_channels, nf, 3, 1, 1, bias=True)
        self.RRDB_trunk = nn.Sequential(*[ResidualInResidualDenseBlock(nf=nf, gc=gc) for _ in range(nb)])
        self.trunk_conv = nn.Conv2d(nf, nf, 3, 1, 1, bias=True)
        self.upconv1 = nn.Conv2d(nf, nf, 3, 1, 1, bias=True)
        if self.scale_factor == 4:
            self.upconv2 = nn.Conv2d(nf, nf, 3, 1, 1, bias=True)
        self.HRconv = nn.Conv2d(nf, nf, 3, 1, 1, bias=True)
        self.conv_last = nn.Conv2d(nf, out_channels, 3, 1, 1, bias=True)
        self.lrelu = nn.LeakyReLU(negative_slope=0.2, inplace=True)
        self.srcnn = SRCNN(in_channels=3, out_channels=out_channels)
        self._flatten()
        object.__setattr__(self, "_engine", None)
        object.__setattr__(self, "_grad_ready_hook", None)
        object.__setattr__(self, "_grad_ready_blocks", ())

    def set_grad_ready_hook(self, fn, blocks=None) -> None:
        """Call ``fn(lo)`` during backward when every flat-gradient entry at offset >= lo is final: after the
        RRDB blocks in ``blocks`` (default: about every quarter of the trunk).  Used by the overlapped DDP
        all-reduce (core/ddp.OverlappedGradAllReducer); ``fn=None`` removes it."""
        if blocks is None:
            blocks = tuple(sorted({b for b in (3 * self.nb // 4, self.nb // 2, self.nb // 4) if 0 < b < self.nb}, reverse=True))
        object.__setattr__(self, "_grad_ready_hook", fn)
        object.__setattr__(self, "_grad_ready_blocks", tuple(blocks) if fn is not None else ())

    def _block_flat_lo(self, blk: int) -> int:
        p = self.RRDB_trunk[blk].RDB1.conv1.weight
        for q, off, _n in self._flat_index:
            if q is p:
                return off
        raise KeyError(f"RRDB_trunk.{blk} not in the flat parameter index")

    def _on_flat_moved(self):
        object.__setattr__(self, "_engine", None)

    def engine(self) -> _Engine:
        self._ensure_flat()
        if self._engine is None or self._engine.gen is not self:
            object.__setattr__(self, "_engine", _Engine(self))
        return self._engine

    def repack_weights(self) -> None:
        """Refresh the bf16 MFMA weight layouts after an in-place update of the fp32 master weights."""
        self.engine().repack()

    def forward(self, x: Tensor, elev: Tensor, mask: Tensor) -> Tensor:
        if not x.is_cuda:
            raise RuntimeError("climsr_amd.ESRGANGenerator runs on the GPU only (no CPU fallback); move it with .cuda()")
        eng = self.engine()
        params = self._flat_params()
        keep = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        return _GeneratorFn.apply(x, elev, mask, (eng, keep, keep and self._route_grads_through_autograd()), *params)

    def _flat_params(self) -> List[nn.Parameter]:
        return [p for p, _o, _n in self._flat_index]
