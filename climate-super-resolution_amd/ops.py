"""Host-side conv layer plans over the HIP C ABI (all arithmetic in libclimsr_hip.so).

``ConvPlan`` holds one nn.Conv2d's geometry: the packed bf16 weight layouts for the forward
(``wpk``) and for the data gradient (``wpk_t``, transposed + flipped taps), and issues the
forward / dgrad / wgrad launches on torch's current stream.  Activation buffers are NHWC torch
tensors (bf16 or fp32) addressed by (channel stride, channel offset).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch

from . import _lib
from ._lib import ChainDesc, ConvDesc, Epilogue, PackDesc, PullPackDesc, ReduceDesc, check, ptr

ACT_NONE, ACT_LRELU, ACT_RELU = 0, 1, 2
ACT_LRELU_BWD, ACT_RELU_BWD = 3, 4  # epilogue multiplies by act'(res1), res1 = the activation's output
OUT_BF16, OUT_F32, OUT_F32_ADD = 0, 1, 2


def round_up(a: int, b: int) -> int:
    return (a + b - 1) // b * b


# Optional launch observer (bench.py's per-kernel HIP-event timer).  Called as
# PROFILER(kernel_name, algorithmic_flops, launch_fn, tag, algorithmic_bytes); must call launch_fn() exactly
# once.  algorithmic_bytes = every operand read once and every result written once (no halo re-reads).
PROFILER = None


def _kname(d, bias, ep) -> str:
    """The kernel climsr_conv2d_fwd will launch for (d, ep) -- only asked when a profiler is attached."""
    if PROFILER is None:
        return ""
    return _lib.load().climsr_conv2d_fwd_kernel(ctypes.byref(d), bias, ctypes.byref(ep)).decode()


def _run(name, flops, fn, tag="", nbytes=0):
    if PROFILER is None:
        fn()
    else:
        PROFILER(name, flops, fn, tag, nbytes)


def _launch(label: str, call, nbytes: int = 0, flops: int = 0) -> None:
    """Run one C-ABI entry point (``call`` returns its status) under the launch observer, raising on error."""
    if PROFILER is None:
        check(call(), label)
    else:
        PROFILER(label, flops, lambda: check(call(), label), label, nbytes)


def _esize(t: Optional[torch.Tensor]) -> int:
    return 0 if t is None else t.element_size()


class ConvPlan:
    """Geometry + packed weights for one square-kernel conv (``nn.Conv2d``)."""

    def __init__(self, cin_real: int, cout: int, ks: int, stride: int = 1, pad: Optional[int] = None, name: str = ""):
        lib = _lib.load()
        self.name = name
        self.cin_real, self.cout, self.ks, self.stride = cin_real, cout, ks, stride
        self.pad = ks // 2 if pad is None else pad
        self.cin = round_up(cin_real, 8)
        # <= 4 real input channels: taps packed 4 channels apart (climsr_conv_chunk_ex returns 4 for the shapes it
        # has a kernel for); cin_k = the channel count of the packed K layout
        self.cc = lib.climsr_conv_chunk_ex(4 if cin_real <= 4 else self.cin, ks, cout, stride)
        if self.cc == 4 and self.pad != ks // 2:
            self.cc = lib.climsr_conv_chunk_ex(self.cin, ks, cout, stride)
        self.cin_k = 4 if self.cc == 4 else self.cin
        self.kpk = lib.climsr_conv_packed_k(self.cin_k, ks, self.cc)
        self.rows = lib.climsr_conv_packed_rows(cout)
        # transposed conv (data gradient): in = cout (padded to 8), out = cin_real
        self.cin_t = round_up(cout, 8)
        self.cout_t = cin_real
        self.cc_t = lib.climsr_conv_chunk_ex(self.cin_t, ks, self.cout_t, stride)
        self.kpk_t = lib.climsr_conv_packed_k(self.cin_t, ks, self.cc_t)
        self.rows_t = lib.climsr_conv_packed_rows(self.cout_t)
        self.wpk: Optional[torch.Tensor] = None
        self.wpk_t: Optional[torch.Tensor] = None
        self.weight: Optional[torch.Tensor] = None  # fp32 OIHW master (a view of the module's flat buffer)
        self.bias: Optional[torch.Tensor] = None
        self.gw: Optional[torch.Tensor] = None  # fp32 OIHW weight grad (view of the flat grad buffer)
        self.gb: Optional[torch.Tensor] = None

    def flops_per_px(self) -> int:
        return 2 * self.cin_real * self.cout * self.ks * self.ks

    # ---------------------------------------------------------------- packing
    def bind(self, weight: torch.Tensor, bias: Optional[torch.Tensor], need_t: bool = True) -> None:
        self.weight, self.bias = weight, bias
        dev = weight.device
        if self.wpk is None or self.wpk.device != dev:
            self.wpk = torch.empty((self.rows, self.kpk), dtype=torch.bfloat16, device=dev)
            self.wpk_t = torch.empty((self.rows_t, self.kpk_t), dtype=torch.bfloat16, device=dev) if need_t else None

    def pack(self, stream: Optional[int] = None) -> None:
        lib = _lib.load()
        s = _lib.stream_ptr() if stream is None else stream
        w = self.weight
        assert w is not None and w.dtype == torch.float32 and w.is_contiguous()
        _launch(f"pack {self.name}", lambda: lib.climsr_pack_conv_weight(ptr(w), self.cout, self.cin_k, self.cin_real, self.cout, self.ks, self.cc,
                                          0, ptr(self.wpk), s))
        if self.wpk_t is not None:
            _launch(f"pack_t {self.name}", lambda: lib.climsr_pack_conv_weight(ptr(w), self.cout_t, self.cin_t, self.cout, self.cout_t, self.ks, self.cc_t, 1,
                                              ptr(self.wpk_t), s))

    def pack_descs(self):
        out = [PackDesc(ptr(self.weight), ptr(self.wpk), self.cout, self.cin_k, self.cin_real, self.cout, self.ks, self.cc, 0, 0)]
        if self.wpk_t is not None:
            out.append(PackDesc(ptr(self.weight), ptr(self.wpk_t), self.cout_t, self.cin_t, self.cout, self.cout_t, self.ks,
                                self.cc_t, 1, 0))
        return out

    # ---------------------------------------------------------------- launches
    def out_hw(self, in_h: int, in_w: int, up: int = 1):
        h = (in_h * up + 2 * self.pad - self.ks) // self.stride + 1
        w = (in_w * up + 2 * self.pad - self.ks) // self.stride + 1
        return h, w

    def fwd(self, x: torch.Tensor, x_cs: int, x_co: int, in_h: int, in_w: int, y: torch.Tensor, y_cs: int, y_co: int,
            n: int, up: int = 1, act: int = ACT_NONE, slope: float = 0.2, use_bias: bool = True,
            res1: Optional[torch.Tensor] = None, alpha1: float = 1.0, res1_cs: int = 0, res1_co: int = 0,
            res2: Optional[torch.Tensor] = None, alpha2: float = 1.0, res2_cs: int = 0, res2_co: int = 0,
            out_mode: int = OUT_BF16, beta1: float = 1.0, beta2: float = 1.0, aux: Optional[torch.Tensor] = None,
            aux_cs: int = 0, aux_co: int = 0, aux_scale: float = 1.0, bn_part: Optional[torch.Tensor] = None,
            ch_part: Optional[torch.Tensor] = None, pool2: bool = False) -> None:
        """y = epilogue(conv(x)); residuals res1/res2 may be bf16 or fp32 tensors (dtype decides), aux = optional
        second bf16 output aux_scale * y; bn_part (fp64, bn_parts() rows x 2 x cout) = BatchNorm partial sums of y
        for bn_forward_parts; ch_part (fp32, ch_parts() rows x cout) = per-tile channel sums of y (fp32 output);
        pool2: y is the 2x2 max pool of the activated output (half the height and width; pool_ok())."""
        oh, ow = self.out_hw(in_h, in_w, up)
        if (not pool2 and self.cin_real == 1 and self.ks in (3, 5) and self.stride == 1 and self.pad == self.ks // 2 and up == 1
                and self.cout in (32, 64) and out_mode == OUT_BF16 and y.dtype == torch.bfloat16 and res1 is None and res2 is None
                and aux is None and act in (ACT_NONE, ACT_LRELU, ACT_RELU) and (y_cs | y_co) % 8 == 0):
            # one input channel: a 1 -> C stencil (climsr_conv_single_input), not a GEMM with K padded 9 -> 96
            px = n * oh * ow
            b = ptr(self.bias) if (use_bias and self.bias is not None) else None
            kn = "dgrad_ci1_kernel<%d, %d, true>" % (self.ks, self.cout // 8) if PROFILER is not None else ""
            _run(kn, 2 * self.cout * self.ks * self.ks * px, lambda: check(
                _lib.load().climsr_conv_single_input(n, in_h, in_w, self.ks, self.pad, ptr(x), x_cs, x_co, ptr(self.weight), b,
                                                     self.cout, act, slope, ptr(y), y_cs, y_co, _lib.stream_ptr()),
                f"conv fwd {self.name}"), "fwd " + self.name, px * 2 + px * self.cout * 2)
            return
        d = ConvDesc(n, in_h, in_w, self.cin_k, x_cs, x_co, up, self.ks, self.stride, self.pad, oh, ow, self.cout, y_cs, y_co,
                     self.cc)
        rf = (1 if res1 is not None and res1.dtype == torch.float32 else 0) | \
             (2 if res2 is not None and res2.dtype == torch.float32 else 0)
        ep = Epilogue(act, slope, alpha1, ptr(res1), res1_cs, res1_co, alpha2, ptr(res2), res2_cs, res2_co, out_mode, 0,
                      rf, beta1, beta2, aux_cs, ptr(aux), aux_co, aux_scale, ptr(bn_part), ch_part=ptr(ch_part), pool2=int(pool2))
        b = ptr(self.bias) if (use_bias and self.bias is not None) else None
        flops = 2 * self.cin_real * self.cout * self.ks * self.ks * n * oh * ow
        opx = n * oh * ow // (4 if pool2 else 1)
        nbytes = (n * in_h * in_w * self.cin_real * 2 + self.rows * self.kpk * 2 +
                  opx * self.cout * (y.element_size() * (2 if out_mode == OUT_F32_ADD else 1) + _esize(res1) + _esize(res2) +
                                     _esize(aux)))
        _run(_kname(d, b, ep), flops, lambda: check(
            _lib.load().climsr_conv2d_fwd(ctypes.byref(d), ptr(x), ptr(self.wpk), b, ctypes.byref(ep), ptr(y), _lib.stream_ptr()),
            f"conv fwd {self.name}"), "fwd " + self.name, nbytes)

    def pool_ok(self, x_cs: int, in_h: int, in_w: int, n: int, y_cs: int, act: int = ACT_RELU) -> bool:
        """Whether fwd(..., act=act, pool2=True) has a fused conv + 2x2 max-pool kernel (climsr_conv2d_fwd_pool_ok)."""
        oh, ow = self.out_hw(in_h, in_w)
        d = ConvDesc(n, in_h, in_w, self.cin_k, x_cs, 0, 1, self.ks, self.stride, self.pad, oh, ow, self.cout, y_cs, 0, self.cc)
        ep = Epilogue(act, 0.2, 1.0, None, 0, 0, 1.0, None, 0, 0, OUT_BF16, 0, 0, 1.0, 1.0, 0, None, 0, 1.0, None, pool2=1)
        return bool(_lib.load().climsr_conv2d_fwd_pool_ok(ctypes.byref(d), ctypes.byref(ep)))

    def bn_parts(self, x_cs: int, in_h: int, in_w: int, n: int, y_cs: int) -> int:
        """Rows of BatchNorm partials fwd(..., use_bias=False, bn_part=...) writes (plain bf16 output), 0 if its kernel
        cannot (climsr_conv2d_fwd_bn_parts)."""
        oh, ow = self.out_hw(in_h, in_w)
        d = ConvDesc(n, in_h, in_w, self.cin_k, x_cs, 0, 1, self.ks, self.stride, self.pad, oh, ow, self.cout, y_cs, 0, self.cc)
        ep = Epilogue(ACT_NONE, 0.0, 1.0, None, 0, 0, 1.0, None, 0, 0, OUT_BF16, 0, 0, 1.0, 1.0, 0, None, 0, 1.0, 1)
        return int(_lib.load().climsr_conv2d_fwd_bn_parts(ctypes.byref(d), ctypes.byref(ep)))

    def ch_parts(self, x_cs: int, in_h: int, in_w: int, n: int, y_cs: int) -> tuple:
        """(rows, rows per image) of the per-tile channel sums fwd(..., ch_part=...) writes (fp32 or bf16 output), (0, 0)
        if its kernel cannot (climsr_conv2d_fwd_ch_parts)."""
        oh, ow = self.out_hw(in_h, in_w)
        d = ConvDesc(n, in_h, in_w, self.cin_k, x_cs, 0, 1, self.ks, self.stride, self.pad, oh, ow, self.cout, y_cs, 0, self.cc)
        ep = Epilogue(ACT_NONE, 0.0, 1.0, None, 0, 0, 1.0, None, 0, 0, OUT_F32, 0, 0, 1.0, 1.0, 0, None, 0, 1.0, None)
        tpi = ctypes.c_int32(0)
        rows = int(_lib.load().climsr_conv2d_fwd_ch_parts(ctypes.byref(d), ctypes.byref(ep), ctypes.byref(tpi)))
        return rows, int(tpi.value)

    def dgrad(self, dz: torch.Tensor, dz_cs: int, out_h: int, out_w: int, g: torch.Tensor, g_cs: int, g_co: int, n: int,
              accumulate: bool = False, down2: bool = False, cout_t: Optional[int] = None, aux: Optional[torch.Tensor] = None,
              aux_cs: int = 0, aux_co: int = 0, aux_scale: float = 1.0, act: int = ACT_NONE, res1: Optional[torch.Tensor] = None,
              res1_cs: int = 0, res1_co: int = 0, bn_bwd: Optional[tuple] = None, res2: Optional[torch.Tensor] = None,
              res2_cs: int = 0, res2_co: int = 0) -> None:
        """Data gradient: g[:, :, :, g_co:g_co+cin_real] (+)= conv^T(dz); (out_h, out_w) are dz's dims.  g is fp32
        (= or += with accumulate), or bf16: then it is the NEXT layer's conv output gradient directly, with
        act = ACT_LRELU_BWD / ACT_RELU_BWD applied from that layer's stored activation res1.  With down2 the
        result is summed over 2x2 pixel blocks (backward of the nearest x2 upsample feeding this conv).
        Stride-2 convs (pad 1, even input) run as a stride-1 conv over the zero-inserted dz.
        bn_bwd = (part, z, z_cs, mean, rstd, gamma, beta): g (bf16) is dL/da of the previous BatchNorm + LeakyReLU(0.2)
        layer and the epilogue writes that layer's backward statistics partials into part (fp64, dgrad_bn_parts() rows x 2
        x cin) for bn_backward_parts.  With act = ACT_NONE, res1 / res2 (bf16 or fp32, dtype decides) are added to the
        result (g = conv^T(dz) + res1 + res2; the aux copy is of that sum)."""
        ct = self.cout_t if cout_t is None else cout_t
        if (self.cout == 1 and self.stride == 1 and self.ks in (3, 5) and self.pad == self.ks // 2 and g.dtype == torch.bfloat16
                and not down2 and aux is None and act in (ACT_NONE, ACT_LRELU_BWD, ACT_RELU_BWD) and ct == self.cin_real
                and ct in (32, 64) and res2 is None and (res1 is None or act != ACT_NONE)):
            # one output channel: its data gradient is a 1 -> C stencil (climsr_dgrad_single_output), not a GEMM
            hw = n * out_h * out_w
            nbytes = hw * 2 + hw * ct * 2 * (2 if res1 is not None else 1)
            kn = _lib.load().climsr_dgrad_single_output_kernel(self.ks, ct, act).decode() if PROFILER is not None else ""
            _run(kn, 2 * ct * self.ks * self.ks * hw, lambda: check(
                _lib.load().climsr_dgrad_single_output(n, out_h, out_w, self.ks, self.pad, ptr(dz), dz_cs, 0, ptr(self.weight), ct, act,
                                                       0.2, ptr(res1), res1_cs, res1_co, ptr(g), g_cs, g_co, _lib.stream_ptr()),
                f"conv dgrad {self.name}"), "dgrad " + self.name, nbytes)
            return
        assert self.stride == 1 or not down2
        d = self._dgrad_desc(dz_cs, out_h, out_w, g_cs, g_co, n, ct)
        out_h, out_w = d.out_h, d.out_w
        mode = OUT_BF16 if g.dtype == torch.bfloat16 else (OUT_F32_ADD if accumulate else OUT_F32)
        rf = (1 if res1 is not None and res1.dtype == torch.float32 else 0) | \
             (2 if res2 is not None and res2.dtype == torch.float32 else 0)
        ep = Epilogue(act, 0.2 if act == ACT_LRELU_BWD else 0.0, 1.0, ptr(res1), res1_cs, res1_co, 1.0, ptr(res2), res2_cs, res2_co,
                      mode, 1 if down2 else 0, rf, 1.0, 1.0, aux_cs, ptr(aux), aux_co, aux_scale)
        if bn_bwd is not None:
            part, z, z_cs, mean, rstd, gamma, beta = bn_bwd
            ep.bn_part, ep.bn_z, ep.bn_z_cstride, ep.bn_slope = ptr(part), ptr(z), z_cs, 0.2
            ep.bn_mean, ep.bn_rstd, ep.bn_gamma, ep.bn_beta = ptr(mean), ptr(rstd), ptr(gamma), ptr(beta)
        # algorithmic: the forward's FLOPs (stride 2: the zero-inserted taps are not work)
        flops = 2 * self.cout * ct * self.ks * self.ks * n * out_h * out_w // (self.stride * self.stride)
        gpx = n * out_h * out_w // (4 if down2 else 1)  # result pixels (after the 2x2 sum)
        nbytes = (n * d.in_h * d.in_w * self.cout * 2 + self.rows_t * self.kpk_t * 2 +
                  gpx * ct * (g.element_size() * (2 if mode == OUT_F32_ADD else 1) + _esize(res1) + _esize(res2) + _esize(aux)))
        _run(_kname(d, None, ep), flops, lambda: check(
            _lib.load().climsr_conv2d_fwd(ctypes.byref(d), ptr(dz), ptr(self.wpk_t), None, ctypes.byref(ep), ptr(g),
                                          _lib.stream_ptr()), f"conv dgrad {self.name}"), "dgrad " + self.name, nbytes)

    def _dgrad_desc(self, dz_cs, out_h, out_w, g_cs, g_co, n, ct):
        pad_t = self.ks - 1 - self.pad
        if self.stride == 1:  # input size = out + ks - 1 - 2 pad (== out for 'same' convs)
            ih, iw = out_h + 2 * pad_t - self.ks + 1, out_w + 2 * pad_t - self.ks + 1
            return ConvDesc(n, out_h, out_w, self.cin_t, dz_cs, 0, 1, self.ks, 1, pad_t, ih, iw, ct, g_cs, g_co, self.cc_t)
        # stride 2: stride-1 conv over the zero-inserted gradient (logical size 2*out)
        assert self.stride == 2
        ih, iw = 2 * out_h + 2 * pad_t - self.ks + 1, 2 * out_w + 2 * pad_t - self.ks + 1
        return ConvDesc(n, out_h, out_w, self.cin_t, dz_cs, 0, -2, self.ks, 1, pad_t, ih, iw, ct, g_cs, g_co, self.cc_t)

    def dgrad_bn_parts(self, dz_cs: int, out_h: int, out_w: int, g_cs: int, n: int, z_cs: int) -> int:
        """Rows of BatchNorm-backward partials dgrad(..., bn_bwd=...) writes for a bf16 g, 0 if its kernel cannot."""
        d = self._dgrad_desc(dz_cs, out_h, out_w, g_cs, 0, n, self.cout_t)
        ep = Epilogue(ACT_NONE, 0.0, 1.0, None, 0, 0, 1.0, None, 0, 0, OUT_BF16, 0, 0, 1.0, 1.0, 0, None, 0, 1.0, 1)
        ep.bn_z, ep.bn_z_cstride = 1, z_cs
        return int(_lib.load().climsr_conv2d_fwd_bn_parts(ctypes.byref(d), ctypes.byref(ep)))

    @property
    def cin_w(self) -> int:
        """Input channels as seen by the wgrad kernel: 4 selects the <=4-real-channel (tap-packed) variant."""
        return 4 if self.cin_real <= 4 else self.cin

    def wgrad_desc(self, n, in_h, in_w, x_cs, x_co, up):
        oh, ow = self.out_hw(in_h, in_w, up)
        return ConvDesc(n, in_h, in_w, self.cin_w, x_cs, x_co, up, self.ks, self.stride, self.pad, oh, ow, self.cout, 0, 0,
                        self.cc)

    def wgrad(self, x: torch.Tensor, x_cs: int, x_co: int, in_h: int, in_w: int, dz: torch.Tensor, dz_cs: int, n: int,
              workspace: "Workspace", accumulate: bool, up: int = 1) -> None:
        """Weight/bias gradient into self.gw / self.gb (fp32 OIHW)."""
        lib = _lib.load()
        d = self.wgrad_desc(n, in_h, in_w, x_cs, x_co, up)
        ns = lib.climsr_conv2d_wgrad_splits(ctypes.byref(d))
        need = lib.climsr_conv2d_wgrad_workspace(ctypes.byref(d), ns)
        ws = workspace.get(need, x.device)
        cw = self.cin_w
        rows_c = need // (ns * (cw * self.ks * self.ks + 1))  # co_rows
        part = ws
        bpart = ws[ns * rows_c * cw * self.ks * self.ks:]
        s = _lib.stream_ptr()
        has_b = self.bias is not None and self.gb is not None
        flops = 2 * self.cin_real * self.cout * self.ks * self.ks * n * d.out_h * d.out_w
        nbytes = n * in_h * in_w * self.cin_real * 2 + n * d.out_h * d.out_w * self.cout * 2 + self.cout * self.cin_real * self.ks ** 2 * 4
        _run(lib.climsr_conv2d_wgrad_kernel(ctypes.byref(d)).decode() if PROFILER is not None else "", flops,
             lambda: check(
            lib.climsr_conv2d_wgrad(ctypes.byref(d), ptr(x), ptr(dz), dz_cs, ptr(part), ptr(bpart) if has_b else None, ns,
                                    _lib.stream_ptr()), f"conv wgrad {self.name}"), "wgrad " + self.name, nbytes)
        _launch(f"wgrad reduce {self.name}", lambda: lib.climsr_conv2d_wgrad_reduce(ptr(part), ptr(bpart) if has_b else None, ns, self.cout, self.cin_real, cw,
                                             self.ks, ptr(self.gw), ptr(self.gb) if has_b else None,
                                             1 if accumulate else 0, s))


class GroupedWgrad:
    """Weight/bias gradients of several 3x3 convs that read channel prefixes of ONE input buffer and whose
    output gradients sit side by side in ONE buffer (the residual dense block: conv_k reads x..x_{k-1},
    dZ = [dZ1|..|dZ5]): one wgrad GEMM over all output-gradient channels x all input channels, then one
    row-sliced reduction into every conv's OIHW gradient (upper-triangle blocks are computed and dropped)."""

    def __init__(self, plans, in_c: int, name: str = ""):
        self.plans, self.in_c, self.name = plans, in_c, name
        self.out_c = sum(p.cout for p in plans)
        assert self.out_c % 64 == 0 and in_c % 64 == 0 and all(p.ks == 3 and p.stride == 1 for p in plans)
        self.row0 = []
        r = 0
        for p in plans:
            self.row0.append(r)
            r += p.cout
        self.max_elems = max(p.cout * p.cin_real * 9 + p.cout for p in plans)
        self._key = None
        self.table = None

    def _table(self, dev):
        key = tuple((ptr(p.gw), ptr(p.gb)) for p in self.plans)
        if key != self._key:
            descs = [ReduceDesc(ptr(p.gw), ptr(p.gb) if p.bias is not None else None, r0, p.cout, p.cin_real, 0)
                     for p, r0 in zip(self.plans, self.row0)]
            arr = (ReduceDesc * len(descs))(*descs)
            self.table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(dev)
            self._key = key
        return self.table

    def run(self, x: torch.Tensor, x_cs: int, x_co: int, in_h: int, in_w: int, dz: torch.Tensor, dz_cs: int, n: int,
            workspace: "Workspace", accumulate: bool) -> None:
        lib = _lib.load()
        d = ConvDesc(n, in_h, in_w, self.in_c, x_cs, x_co, 1, 3, 1, 1, in_h, in_w, self.out_c, 0, 0, 8)
        ns = lib.climsr_conv2d_wgrad_splits(ctypes.byref(d))
        need = lib.climsr_conv2d_wgrad_workspace(ctypes.byref(d), ns)
        ws = workspace.get(need, x.device)
        part = ws
        bpart = ws[ns * self.out_c * self.in_c * 9:]
        s = _lib.stream_ptr()
        flops = sum(2 * p.cin_real * p.cout * 9 for p in self.plans) * n * in_h * in_w
        nbytes = n * in_h * in_w * (self.in_c + self.out_c) * 2 + sum(p.cout * p.cin_real * 9 * 4 for p in self.plans)
        _run(lib.climsr_conv2d_wgrad_kernel(ctypes.byref(d)).decode() if PROFILER is not None else "", flops, lambda: check(
            lib.climsr_conv2d_wgrad(ctypes.byref(d), ptr(x), ptr(dz), dz_cs, ptr(part), ptr(bpart), ns, _lib.stream_ptr()),
            f"grouped wgrad {self.name}"), "wgrad " + self.name, nbytes)
        tab = self._table(x.device)
        _launch(f"grouped wgrad reduce {self.name}", lambda: lib.climsr_conv2d_wgrad_reduce_rows(ptr(part), ptr(bpart), ns, self.out_c, self.in_c * 9, 3, ptr(tab),
                                                  len(self.plans), self.max_elems, 1 if accumulate else 0, s))


class Workspace:
    """Grow-only fp32 scratch buffer (wgrad split partials)."""

    def __init__(self):
        self.buf: Optional[torch.Tensor] = None

    def get(self, nfloats: int, device) -> torch.Tensor:
        if self.buf is None or self.buf.numel() < nfloats or self.buf.device != device:
            self.buf = torch.empty(max(nfloats, 1 << 20), dtype=torch.float32, device=device)
        return self.buf


def act_grad(npix: int, c_real: int, g: torch.Tensor, g_cs: int, g_co: int, y: Optional[torch.Tensor], y_cs: int, y_co: int,
             act: int, dz: torch.Tensor, dz_cs: int, scale: float = 1.0, slope: float = 0.2) -> None:
    if g.dtype != torch.float32:  # the C ABI reads `const float* g`
        raise TypeError(f"act_grad: the incoming gradient must be float32, got {g.dtype}")
    _launch("act_grad", lambda: _lib.load().climsr_act_grad(npix, c_real, ptr(g), g_cs, g_co, ptr(y), y_cs, y_co, act, slope, scale, ptr(dz), dz_cs,
                                      _lib.stream_ptr()))


def axpby(npix: int, c: int, a: float, x: Optional[torch.Tensor], x_cs: int, x_co: int, b: float, y: torch.Tensor, y_cs: int,
          y_co: int) -> None:
    _launch("axpby", lambda: _lib.load().climsr_axpby_f32(npix, c, a, ptr(x), x_cs, x_co, b, ptr(y), y_cs, y_co, _lib.stream_ptr()))


def nchw_to_nhwc(src: torch.Tensor, dst: torch.Tensor, cs: int, co: int) -> None:
    n, c, h, w = src.shape
    assert src.dtype == torch.float32 and src.is_contiguous()
    _launch("nchw_to_nhwc", lambda: _lib.load().climsr_nchw_to_nhwc_bf16(ptr(src), n, c, h, w, ptr(dst), cs, co, _lib.stream_ptr()))


def pack_planes8(planes, n: int, h: int, w: int, dst: torch.Tensor) -> None:
    """dst [n,h,w,8] bf16 (all 8 channels written): channel k = planes[k] (an fp32 [n,c,h,w] tensor and its channel
    index, or None -> zeros)."""
    assert dst.dtype == torch.bfloat16 and dst.is_contiguous() and dst.shape[-1] == 8 and len(planes) <= 8
    pl = _lib.Planes8()
    for k, spec in enumerate(planes):
        if spec is None:
            continue
        t, ch = spec
        assert t.dtype == torch.float32 and t.is_contiguous() and t.shape[0] == n and t.shape[2:] == (h, w)
        pl.p[k] = t.data_ptr() + ch * h * w * 4
        pl.img_stride[k] = t.shape[1] * h * w
    keep = [spec[0] for spec in planes if spec is not None]  # keep the sources alive until the launch is queued
    _launch("pack_planes8", lambda: _lib.load().climsr_pack_planes_nhwc8_bf16(ctypes.byref(pl), n, h, w, ptr(dst), _lib.stream_ptr()),
            nbytes=n * h * w * (16 + 4 * len(keep)))


def nhwc_to_nchw(src: torch.Tensor, n: int, c: int, h: int, w: int, cs: int, co: int, dst: torch.Tensor) -> None:
    is_bf16 = 1 if src.dtype == torch.bfloat16 else 0
    _launch("nhwc_to_nchw", lambda: _lib.load().climsr_nhwc_to_nchw_f32(ptr(src), is_bf16, n, c, h, w, cs, co, ptr(dst), _lib.stream_ptr()))


def rdb_bwd_init(npix: int, nf: int, dc: int, gx: torch.Tensor, gy: torch.Tensor, gskip: torch.Tensor, dz: torch.Tensor, a_o: float,
                 save_skip: bool, add_skip: bool) -> None:
    _launch("rdb_bwd_init", lambda: _lib.load().climsr_rdb_bwd_init(npix, nf, dc, ptr(gx), ptr(gy), ptr(gskip), ptr(dz), a_o, int(save_skip), int(add_skip),
                                          _lib.stream_ptr()))


class BatchedPacker:
    """All weight packs of a network as ONE launch (descriptor table resident on the device)."""

    def __init__(self, plans, device, extra=()):
        descs = []
        for p in plans:
            descs += p.pack_descs()
        descs += list(extra)
        arr = (PackDesc * len(descs))(*descs)
        raw = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
        self.table = raw.to(device)
        self.n = len(descs)
        self.max_elems = max(d.out_c for d in descs)  # placeholder, replaced below
        self.max_elems = max(p.rows * p.kpk for p in plans)
        for p in plans:
            if p.wpk_t is not None:
                self.max_elems = max(self.max_elems, p.rows_t * p.kpk_t)
        for d in extra:
            self.max_elems = max(self.max_elems, 16 * 9 * d.cc)

    def run(self):
        _launch("pack batched", lambda: _lib.load().climsr_pack_conv_weights_batched(ptr(self.table), self.n, self.max_elems, _lib.stream_ptr()))


class PullPlan(ConvPlan):
    """Data gradient of one channel group of a residual dense block's concatenation, as ONE conv over the
    side-by-side output gradients of every conv that reads the group (climsr_hip.h, ClimsrPullPackDesc).
    ``segs`` = [(weight OIHW fp32, out_c, in_c_real)] of the consuming convs in dZ-channel order."""

    def __init__(self, segs, out_c: int, ci_off: int, ks: int = 3, name: str = ""):
        in_c = sum(oc for _w, oc, _ic in segs)
        super().__init__(in_c, out_c, ks, 1, None, name)
        self.segs, self.ci_off = segs, ci_off
        self.wpk = torch.empty((self.rows, self.kpk), dtype=torch.bfloat16, device=segs[0][0].device)

    def pull_desc(self) -> PullPackDesc:
        d = PullPackDesc()
        d.out = ptr(self.wpk)
        for k, (w, oc, ic) in enumerate(self.segs):
            assert w.dtype == torch.float32 and w.is_contiguous() and tuple(w.shape) == (oc, ic, self.ks, self.ks)
            d.seg_w[k], d.seg_oc[k], d.seg_ic[k] = ptr(w), oc, ic
        d.nseg, d.out_c, d.in_c, d.ks, d.cc, d.ci_off = len(self.segs), self.cout, self.cin, self.ks, self.cc, self.ci_off
        return d


class RdbChain:
    """The four 16-output convs of a residual dense block (esrgan.py:22-37) as ONE row-streaming launch
    (csrc/rdb_chain.hip), forward (conv1..conv4 -> x1..x4) and pull backward (pull4..pull1 -> dZ4..dZ1).
    convs: the block's five ConvPlans (bound).  Needs nf = 64, gc = 16."""

    def __init__(self, convs, name: str = ""):
        lib = _lib.load()
        self.convs, self.name = convs, name
        dev = convs[0].weight.device
        self.kp = [lib.climsr_rdb_chain_kp(L) for L in range(1, 5)]
        self.w_fwd = [torch.empty((16, 9 * kp), dtype=torch.bfloat16, device=dev) for kp in self.kp]
        self.w_pull = [torch.empty((16, 9 * kp), dtype=torch.bfloat16, device=dev) for kp in self.kp]

    def pack_descs(self):
        out = []
        for L in range(1, 5):
            c = self.convs[L - 1]
            out.append(PackDesc(ptr(c.weight), ptr(self.w_fwd[L - 1]), 16, self.kp[L - 1], c.cin_real, 16, 3, self.kp[L - 1], 0, 0))
        return out

    def pull_descs(self):
        out = []
        for L in range(1, 5):
            j = 5 - L  # this level produces dZ_j, the gradient of x_j (channels 64 + 16(j-1) of the block input)
            d = PullPackDesc()
            d.out = ptr(self.w_pull[L - 1])
            order = [5] + list(range(4, j, -1))  # base dZ5, then dZ4, dZ3, ... (chain channel order)
            for si, k in enumerate(order):
                c = self.convs[k - 1]
                d.seg_w[si], d.seg_oc[si], d.seg_ic[si] = ptr(c.weight), c.cout, c.cin_real
            d.nseg, d.out_c, d.in_c, d.ks, d.cc, d.ci_off = len(order), 16, sum(self.convs[k - 1].cout for k in order), 3, \
                self.kp[L - 1], 64 + 16 * (j - 1)
            out.append(d)
        return out

    def _launch(self, d, tag):
        """Forward = ``rdb_chain_kernel<0>`` (reads x: 64 ch, writes x1..x4: 64 ch); pull = ``rdb_chain_kernel<1>``
        (reads dZ5: 64 ch and the stored activations x1..x4: 64 ch, writes dZ4..dZ1: 64 ch); bf16, every operand
        once per pixel (the intermediate levels stay on chip)."""
        npx = d.n * d.h * d.w
        flops = sum(2 * self.convs[L].cin_real * 16 * 9 for L in range(4)) * npx
        pull = tag == "pull"
        nbytes = npx * 2 * ((64 + 64 + 64) if pull else (64 + 64)) + sum(w.numel() * 2 for w in (self.w_pull if pull else self.w_fwd))
        name = _lib.load().climsr_rdb_chain_kernel(ctypes.byref(d)).decode() if PROFILER is not None else ""
        _run(name, flops, lambda: check(
            _lib.load().climsr_rdb_chain(ctypes.byref(d), _lib.stream_ptr()), f"rdb chain {self.name}"), tag + " " + self.name,
            nbytes)

    def forward(self, dense: torch.Tensor, dc: int, n: int, h: int, w: int, slope: float = 0.2) -> None:
        d = ChainDesc()
        d.base, d.bcs, d.boff, d.out, d.ocs = ptr(dense), dc, 0, ptr(dense), dc
        for L in range(4):
            d.ooff[L] = 64 + 16 * L
            d.wt[L] = ptr(self.w_fwd[L])
            d.bias[L] = ptr(self.convs[L].bias)
        d.mask, d.mcs, d.act, d.slope, d.n, d.h, d.w = None, 0, ACT_LRELU, slope, n, h, w
        self._launch(d, "fwd")

    def pull(self, dz: torch.Tensor, dense: torch.Tensor, dc: int, n: int, h: int, w: int, slope: float = 0.2) -> None:
        d = ChainDesc()
        d.base, d.bcs, d.boff, d.out, d.ocs = ptr(dz), dc, 64, ptr(dz), dc
        for L in range(4):
            j = 4 - L  # level L+1 produces dZ_j
            d.ooff[L] = 16 * (j - 1)
            d.wt[L] = ptr(self.w_pull[L])
            d.bias[L] = None
            d.moff[L] = 64 + 16 * (j - 1)
        d.mask, d.mcs, d.act, d.slope, d.n, d.h, d.w = ptr(dense), dc, ACT_LRELU_BWD, slope, n, h, w
        self._launch(d, "pull")


class SrcnnTail:
    """srcnn.conv1 -> ReLU -> conv2 -> ReLU -> conv3 (srcnn.py:9-18) of the generator tail as ONE launch
    (csrc/srcnn.hip): reads the 4-channel bf16 cat[out, elev, mask] input, writes the fp32 output; the 64- / 32-channel
    intermediates never leave the chip (the backward recomputes them).  ``convs``: the three bound ConvPlans."""

    def __init__(self, convs, name: str = "srcnn"):
        self.convs, self.name = convs, name
        c1, c2, c3 = convs
        assert (c1.cin_real <= 4 and c1.cout == 64 and c1.ks == 9 and c2.cout == 32 and c2.ks == 1 and c3.cout == 1
                and c3.ks == 5), "the fused SRCNN tail takes in_c <= 4, 64 / 32 / 1 channels, 9 / 1 / 5 kernels"
        # the kernel hard-codes stride 1 and 'same' padding 4 / 0 / 2 (srcnn.py:9-11) and adds all three biases
        assert all(c.stride == 1 and c.pad == c.ks // 2 for c in convs), "the fused SRCNN tail takes stride 1, padding ks // 2"
        self.wpk = torch.empty((_lib.load().climsr_srcnn_packed_elems(),), dtype=torch.bfloat16, device=c1.weight.device)

    def pack(self) -> None:
        c1, c2, c3 = self.convs
        assert c1.bias is not None and c2.bias is not None and c3.bias is not None, "the fused SRCNN tail adds all three biases"
        _launch("srcnn pack", lambda: _lib.load().climsr_srcnn_pack(ptr(c1.weight), ptr(c2.weight), ptr(c3.weight), c1.cin_real,
                                                                    ptr(self.wpk), _lib.stream_ptr()))

    def fwd(self, x: torch.Tensor, x_cs: int, x_co: int, n: int, h: int, w: int, out: torch.Tensor) -> None:
        c1, c2, c3 = self.convs
        assert out.dtype == torch.float32 and out.is_contiguous() and out.numel() == n * h * w
        assert x.dtype == torch.bfloat16 and x.is_contiguous() and x.numel() == n * h * w * x_cs
        d = _lib.SrcnnDesc()
        d.x, d.x_cs, d.x_co, d.wpk = ptr(x), x_cs, x_co, ptr(self.wpk)
        d.b1, d.b2, d.b3, d.out = ptr(c1.bias), ptr(c2.bias), ptr(c3.bias), ptr(out)
        d.n, d.h, d.w = n, h, w
        npx = n * h * w
        flops = 2 * npx * (c1.cin_real * 81 * 64 + 64 * 32 + 32 * 25)
        _run("srcnn_tail_kernel" if PROFILER is not None else "", flops,
             lambda: check(_lib.load().climsr_srcnn_fwd(ctypes.byref(d), _lib.stream_ptr()), "srcnn tail"), "fwd " + self.name, npx * 12)

    def bwd(self, x: torch.Tensor, x_cs: int, x_co: int, n: int, h: int, w: int, gout: torch.Tensor, dz1: torch.Tensor,
            ws: "Workspace", accumulate: bool) -> None:
        """Backward below conv1 (csrc/srcnn.hip srcnn_bwd_kernel): recomputes relu(conv1) / relu(conv2) from the input
        x, writes dz1 = the conv1 output gradient (bf16 NHWC, 64 ch) and the conv2 / conv3 weight + bias gradients
        (into the plans' bound .gw / .gb, += when accumulate)."""
        c1, c2, c3 = self.convs
        assert gout.dtype == torch.float32 and gout.is_contiguous() and gout.numel() == n * h * w
        assert dz1.dtype == torch.bfloat16 and dz1.is_contiguous() and dz1.numel() == n * h * w * 64
        for c in (c2, c3):
            assert c.gw is not None and c.gb is not None, "bind_grads() first"
        L = _lib.load()
        part = ws.get((L.climsr_srcnn_bwd_workspace(n, h, w) + 3) // 4, x.device)
        d = _lib.SrcnnBwdDesc()
        d.x, d.x_cs, d.x_co, d.gout, d.wpk = ptr(x), x_cs, x_co, ptr(gout), ptr(self.wpk)
        d.b1, d.b2, d.dz1, d.part = ptr(c1.bias), ptr(c2.bias), ptr(dz1), ptr(part)
        d.gw2, d.gb2, d.gw3, d.gb3 = ptr(c2.gw), ptr(c2.gb), ptr(c3.gw), ptr(c3.gb)
        d.accumulate, d.n, d.h, d.w = int(accumulate), n, h, w
        npx = n * h * w
        # recompute conv1 + conv2, dA2, dA1, dW2, dW3 (algorithmic, own pixels once)
        flops = 2 * npx * (c1.cin_real * 81 * 64 + 64 * 32 + 32 * 25 + 32 * 64 + 32 * 64 + 32 * 25)
        nbytes = npx * (8 + 4 + 128)
        _run("srcnn_bwd_kernel" if PROFILER is not None else "", flops,
             lambda: check(L.climsr_srcnn_bwd(ctypes.byref(d), _lib.stream_ptr()), "srcnn tail backward"), "bwd " + self.name, nbytes)


class PullPacker:
    """Every pull weight of a network packed by ONE launch (descriptor table resident on the device)."""

    def __init__(self, pulls, device, extra=()):
        descs = [p.pull_desc() for p in pulls] + list(extra)
        arr = (PullPackDesc * len(descs))(*descs)
        self.table = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(device)
        self.n = len(descs)
        self.max_elems = max([p.rows * p.kpk for p in pulls] + [16 * 9 * d.cc for d in extra])

    def run(self):
        _launch("pack pull batched", lambda: _lib.load().climsr_pack_pull_weights_batched(ptr(self.table), self.n, self.max_elems, _lib.stream_ptr()))


# ------------------------------------------------------------------ discriminator / VGG / GAN-loss ops
def _L():
    return _lib.load()


def bn_workspace(npix: int, c: int, cache: dict, dev) -> torch.Tensor:
    """fp64 partial-sum scratch for bn_forward / bn_backward (grow-only, kept in ``cache``)."""
    need = int(_L().climsr_bn_workspace_doubles(npix, c))
    if need <= 0:
        raise RuntimeError(f"bn: unsupported shape npix={npix} c={c}")
    t = cache.get("bnws")
    if t is None or t.numel() < need or t.device != dev:
        t = torch.empty(max(need, 1 << 16), dtype=torch.float64, device=dev)
        cache["bnws"] = t
    return t


def bn_forward(z, npix, c, gamma, beta, mean, rstd, y, ws, run_mean=None, run_var=None, act=ACT_LRELU, slope=0.2, eps=1e-5,
               momentum=0.1, num_batches_tracked=None):
    _run("bn_forward", 0, lambda: check(
        _L().climsr_bn_forward(ptr(z), npix, c, ptr(gamma), ptr(beta), act, slope, eps, momentum, ptr(ws), ptr(mean), ptr(rstd),
                               ptr(run_mean), ptr(run_var), ptr(num_batches_tracked), ptr(y), _lib.stream_ptr()), "bn_forward"),
         "bn_forward", npix * c * 6)


def bn_forward_parts(parts, nparts, z, npix, c, gamma, beta, mean, rstd, y, run_mean=None, run_var=None, act=ACT_LRELU, slope=0.2,
                     eps=1e-5, momentum=0.1, num_batches_tracked=None):
    """bn_forward with the batch statistics from the producing conv's epilogue partials (ConvPlan.fwd bn_part)."""
    _run("bn_forward", 0, lambda: check(
        _L().climsr_bn_forward_parts(ptr(parts), nparts, ptr(z), npix, c, ptr(gamma), ptr(beta), act, slope, eps, momentum, ptr(mean),
                                     ptr(rstd), ptr(run_mean), ptr(run_var), ptr(num_batches_tracked), ptr(y), _lib.stream_ptr()),
        "bn_forward_parts"), "bn_forward", npix * c * 4)


def bn_inference(z, npix, c, run_mean, run_var, gamma, beta, y, act=ACT_LRELU, slope=0.2, eps=1e-5):
    _run("bn_inference", 0, lambda: check(
        _L().climsr_bn_inference(ptr(z), npix, c, ptr(run_mean), ptr(run_var), eps, ptr(gamma), ptr(beta), act, slope, ptr(y),
                                 _lib.stream_ptr()), "bn_inference"), "bn_inference", npix * c * 4)


def bn_backward(da, a, z, npix, c, mean, rstd, gamma, ws, coef, dgamma, dbeta, accumulate, dz, slope=0.2, out_slope=1.0):
    _run("bn_backward", 0, lambda: check(
        _L().climsr_bn_backward(ptr(da), ptr(a), ptr(z), npix, c, ptr(mean), ptr(rstd), ptr(gamma), slope, out_slope, ptr(ws),
                                ptr(coef), ptr(dgamma), ptr(dbeta), int(accumulate), ptr(dz), _lib.stream_ptr()), "bn_backward"),
         "bn_backward", npix * c * 18)


def bn_backward_parts(parts, nparts, da, z, npix, c, mean, rstd, gamma, beta, coef, dgamma, dbeta, accumulate, dz, slope=0.2):
    """bn_backward_z (bf16 da) with the statistics from the producing data gradient's epilogue (ConvPlan.dgrad bn_bwd)."""
    _run("bn_backward", 0, lambda: check(
        _L().climsr_bn_backward_parts(ptr(parts), nparts, ptr(da), ptr(z), npix, c, ptr(mean), ptr(rstd), ptr(gamma), ptr(beta), slope,
                                      ptr(coef), ptr(dgamma), ptr(dbeta), int(accumulate), ptr(dz), _lib.stream_ptr()),
        "bn_backward_parts"), "bn_backward", npix * c * 6)


def bn_backward_z(da, z, npix, c, mean, rstd, gamma, beta, ws, coef, dgamma, dbeta, accumulate, dz, slope=0.2):
    """Backward of LeakyReLU(BN(z)) from da (bf16 or fp32) and z alone (lrelu' recomputed from z)."""
    bf = 1 if da.dtype == torch.bfloat16 else 0
    _run("bn_backward", 0, lambda: check(
        _L().climsr_bn_backward_z(ptr(da), bf, ptr(z), npix, c, ptr(mean), ptr(rstd), ptr(gamma), ptr(beta), slope, ptr(ws),
                                  ptr(coef), ptr(dgamma), ptr(dbeta), int(accumulate), ptr(dz), _lib.stream_ptr()), "bn_backward_z"),
         "bn_backward", npix * c * (3 * da.element_size() + 6))


def reflect_pad1(x, n, h, w, cs, y):
    _launch("reflect_pad1", lambda: _L().climsr_reflect_pad1_bf16(ptr(x), n, h, w, cs, ptr(y), _lib.stream_ptr()))


def reflect_pad1_bwd(gp, n, h, w, c, g):
    _launch("reflect_pad1_bwd", lambda: _L().climsr_reflect_pad1_bwd_f32(ptr(gp), n, h, w, c, ptr(g), _lib.stream_ptr()))


def adaptive_pool_fwd(x, n, h, w, c, oh, ow, out, out_t=None, n_pad=0):
    _launch("adaptive_pool_fwd", lambda: _L().climsr_adaptive_pool_fwd(ptr(x), n, h, w, c, oh, ow, ptr(out), ptr(out_t), n_pad, _lib.stream_ptr()))


def adaptive_pool_bwd(dp, n, h, w, c, oh, ow, dx):
    _launch("adaptive_pool_bwd", lambda: _L().climsr_adaptive_pool_bwd(ptr(dp), n, h, w, c, oh, ow, ptr(dx), _lib.stream_ptr()))


def linear_fwd(x, w, bias, n, k, o, y, ws, act=ACT_NONE, slope=0.2):
    # label = the kernel climsr_linear_fwd dispatches (o % 256 == 0: 64 weight rows per wave) + its split-K reduce
    _run("linear_fwd_wide_kernel" if o % 256 == 0 else "linear_fwd_kernel", 2 * n * k * o, lambda: check(
        _L().climsr_linear_fwd(ptr(x), ptr(w), ptr(bias), n, k, o, act, slope, ptr(ws), ws.numel(), ptr(y), _lib.stream_ptr()),
        "linear_fwd"), "fwd fc.0")


def linear_dgrad(dy, w, n, k, o, dx, accumulate=False):
    _run("linear_dgrad_wide_kernel" if k % 128 == 0 else "linear_dgrad_kernel", 2 * n * k * o, lambda: check(
        _L().climsr_linear_dgrad(ptr(dy), ptr(w), n, k, o, ptr(dx), int(accumulate), _lib.stream_ptr()), "linear_dgrad"),
        "dgrad fc.0")


def linear_wgrad(dy_t, x_t, n_pad, k, o, dw, accumulate):
    _run("linear_wgrad_kernel", 2 * n_pad * k * o, lambda: check(
        _L().climsr_linear_wgrad(ptr(dy_t), ptr(x_t), n_pad, k, o, ptr(dw), int(accumulate), _lib.stream_ptr()), "linear_wgrad"),
        "wgrad fc.0")


def linear_wgrad2(dy_t, x_t, n_pad, dy_t2, x_t2, n_pad2, k, o, dw, accumulate):
    """linear_wgrad over two batches in one launch: dw (+)= dy_t . x_t^T + dy_t2 . x_t2^T."""
    _run("linear_wgrad_kernel", 2 * (n_pad + n_pad2) * k * o, lambda: check(
        _L().climsr_linear_wgrad2(ptr(dy_t), ptr(x_t), n_pad, ptr(dy_t2), ptr(x_t2), n_pad2, k, o, ptr(dw), int(accumulate),
                                  _lib.stream_ptr()), "linear_wgrad2"), "wgrad fc.0")


def d_head_fwd(h, w2, b2, n, o, s, sigmoid=True):
    _launch("d_head_fwd", lambda: _L().climsr_d_head_fwd(ptr(h), ptr(w2), ptr(b2), n, o, int(sigmoid), ptr(s), _lib.stream_ptr()))


def d_head_bwd(h, s, ds, w2, n, o, n_pad, dw2, db2, db0, accumulate, du0, du0_t, slope=0.2, sigmoid=True):
    _launch("d_head_bwd", lambda: _L().climsr_d_head_bwd(ptr(h), ptr(s), ptr(ds), ptr(w2), n, o, n_pad, slope, int(sigmoid), ptr(dw2), ptr(db2), ptr(db0),
                                 int(accumulate), ptr(du0), ptr(du0_t), _lib.stream_ptr()))


def relativistic_bce(s_real, s_fake, n, t_rf, t_fr, loss=None, gscale=None, g_real=None, g_fake=None):
    _launch("relativistic_bce", lambda: _L().climsr_relativistic_bce(ptr(s_real), ptr(s_fake), n, t_rf, t_fr, ptr(loss), ptr(gscale), ptr(g_real), ptr(g_fake),
                                       _lib.stream_ptr()))


def d_stem_s2(x, x_cs, w0, plan2, a0, z2, bn_part, n, h, w, slope=0.2):
    """The RFB discriminator's features.0 (1 -> 64 + LeakyReLU, recomputed on chip) and features.2 (64 -> 64 / stride 2,
    pre-BatchNorm z2 + the BatchNorm partial sums of its 16x16 tiles) in one launch (csrc/stem.hip,
    rfb_esrgan.py:28-31); a0 (features.0's output for the backward) is written only when given."""
    assert x.dtype == torch.bfloat16 and z2.dtype == torch.bfloat16 and w0.dtype == torch.float32 and w0.is_contiguous()
    assert tuple(w0.shape) == (64, 1, 3, 3) and plan2.cin_real == 64 and plan2.cout == 64 and plan2.stride == 2 and plan2.kpk == 576
    assert a0 is None or (a0.dtype == torch.bfloat16 and a0.numel() == n * h * w * 64)
    oh, ow = (h + 1) // 2, (w + 1) // 2
    assert z2.numel() == n * oh * ow * 64
    d = _lib.StemDesc()
    d.x, d.x_cs, d.w0, d.w2, d.kpk2 = ptr(x), x_cs, ptr(w0), ptr(plan2.wpk), plan2.kpk
    d.a0, d.z2, d.bn_part = ptr(a0) if a0 is not None else None, ptr(z2), ptr(bn_part) if bn_part is not None else None
    d.slope, d.n, d.h, d.w = slope, n, h, w
    flops = 2 * n * h * w * 64 * 9 + 2 * n * oh * ow * 64 * 576
    _run("stem_s2_kernel" if PROFILER is not None else "", flops,
         lambda: check(_L().climsr_d_stem_s2(ctypes.byref(d), _lib.stream_ptr()), "d_stem_s2"), "features.0+2",
         n * h * w * 2 + n * oh * ow * 128 + (n * h * w * 128 if a0 is not None else 0))


def vgg_conv1_1(xa, xb, n_half, h, w, weight, bias, y):
    """VGG19 conv1_1 + ReLU on the 1 -> 3 channel repeat of two fp32 image batches (perceptual.py:16,26-31) as one
    1-channel conv (csrc/stem.hip): y bf16 NHWC [2 n_half, h, w, 64], images of xa first."""
    assert xa.dtype == torch.float32 and xb.dtype == torch.float32 and xa.is_contiguous() and xb.is_contiguous()
    assert xa.numel() == n_half * h * w and xb.numel() == n_half * h * w
    assert tuple(weight.shape) == (64, 3, 3, 3) and weight.dtype == torch.float32 and weight.is_contiguous()
    assert bias.numel() == 64 and bias.dtype == torch.float32 and y.dtype == torch.bfloat16 and y.numel() == 2 * n_half * h * w * 64
    _run("vgg_conv1_1_kernel", 2 * 2 * n_half * h * w * 64 * 27,
         lambda: check(_L().climsr_vgg_conv1_1(ptr(xa), ptr(xb), n_half, h, w, ptr(weight), ptr(bias), ptr(y), _lib.stream_ptr()),
                       "vgg_conv1_1"), "vgg conv1_1", 2 * n_half * h * w * (4 + 128))


def d_stem_s2_bn_parts(n, h, w):
    return int(_L().climsr_d_stem_s2_bn_parts(n, h, w))


def maxpool2(x, n, h, w, c, y):
    _launch("maxpool2", lambda: _L().climsr_maxpool2_bf16(ptr(x), n, h, w, c, ptr(y), _lib.stream_ptr()))


def l1_bf16(a, b, n, ws, out):
    _launch("l1_bf16", lambda: _L().climsr_l1_loss_bf16(ptr(a), ptr(b), n, ptr(ws), ptr(out), _lib.stream_ptr()))


def f32_to_bf16(x, y):
    _launch("f32_to_bf16", lambda: _L().climsr_f32_to_bf16(ptr(x), x.numel(), ptr(y), _lib.stream_ptr()))


def increment_i64(t):
    _launch("increment_i64", lambda: _L().climsr_increment_i64(ptr(t), _lib.stream_ptr()))
