"""ctypes binding of libclimsr_hip.so (the C ABI declared in include/climsr_hip.h).

The product path has no CPU fallback: if the library is missing or a call fails, this module
raises.  torch is imported first so the process has exactly one HIP runtime (torch's bundled
libamdhip64 has the same SONAME, libamdhip64.so.7, that the library links against).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional

import torch  # noqa: F401  (must be loaded before the HIP library, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("CLIMSR_HIP_LIB", os.path.join(_HERE, "csrc", "libclimsr_hip.so"))

c_int, c_float, c_double, c_void_p, c_int64, c_size_t = (ctypes.c_int, ctypes.c_float, ctypes.c_double, ctypes.c_void_p,
                                                         ctypes.c_int64, ctypes.c_size_t)


class ConvDesc(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int32) for n in (
        "n", "in_h", "in_w", "in_c", "in_cstride", "in_coff", "up", "ks", "stride", "pad", "out_h", "out_w", "out_c",
        "out_cstride", "out_coff", "cc")]


class Epilogue(ctypes.Structure):
    _fields_ = [("act", ctypes.c_int32), ("slope", c_float), ("alpha1", c_float), ("res1", c_void_p),
                ("res1_cstride", ctypes.c_int32), ("res1_coff", ctypes.c_int32), ("alpha2", c_float), ("res2", c_void_p),
                ("res2_cstride", ctypes.c_int32), ("res2_coff", ctypes.c_int32), ("out_mode", ctypes.c_int32),
                ("down2", ctypes.c_int32), ("res_f32", ctypes.c_int32), ("beta1", c_float), ("beta2", c_float),
                ("aux_cstride", ctypes.c_int32), ("aux", c_void_p), ("aux_coff", ctypes.c_int32), ("aux_scale", c_float),
                ("bn_part", c_void_p), ("bn_z", c_void_p), ("bn_z_cstride", ctypes.c_int32), ("bn_slope", c_float),
                ("bn_mean", c_void_p), ("bn_rstd", c_void_p), ("bn_gamma", c_void_p), ("bn_beta", c_void_p),
                ("ch_part", c_void_p), ("pool2", ctypes.c_int32)]

    def __init__(self, *args, **kw):
        # plain residual adds unless a caller scales them (beta1 / beta2 are positional fields 13 / 14)
        if len(args) <= 13:
            kw.setdefault("beta1", 1.0)
        if len(args) <= 14:
            kw.setdefault("beta2", 1.0)
        super().__init__(*args, **kw)


class StemDesc(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("x_cs", ctypes.c_int32), ("w0", c_void_p), ("w2", c_void_p), ("kpk2", ctypes.c_int32),
                ("a0", c_void_p), ("z2", c_void_p), ("bn_part", c_void_p), ("slope", c_float), ("n", ctypes.c_int32),
                ("h", ctypes.c_int32), ("w", ctypes.c_int32)]


class Planes8(ctypes.Structure):
    _fields_ = [("p", c_void_p * 8), ("img_stride", ctypes.c_int64 * 8)]


class PackDesc(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("out", c_void_p)] + [(n, ctypes.c_int32) for n in (
        "out_c", "in_c", "in_c_real", "out_c_real", "ks", "cc", "tflip", "reserved")]


class ReduceDesc(ctypes.Structure):
    _fields_ = [("wgrad", c_void_p), ("bias_grad", c_void_p), ("row0", ctypes.c_int32), ("out_c", ctypes.c_int32),
                ("in_c_real", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class ChainDesc(ctypes.Structure):
    _fields_ = [("base", c_void_p), ("bcs", ctypes.c_int32), ("boff", ctypes.c_int32), ("out", c_void_p), ("ocs", ctypes.c_int32),
                ("ooff", ctypes.c_int32 * 4), ("wt", c_void_p * 4), ("bias", c_void_p * 4), ("mask", c_void_p),
                ("mcs", ctypes.c_int32), ("moff", ctypes.c_int32 * 4), ("act", ctypes.c_int32), ("slope", c_float),
                ("n", ctypes.c_int32), ("h", ctypes.c_int32), ("w", ctypes.c_int32)]


class PullPackDesc(ctypes.Structure):
    _fields_ = [("out", c_void_p), ("seg_w", c_void_p * 5), ("seg_oc", ctypes.c_int32 * 5), ("seg_ic", ctypes.c_int32 * 5)] + [
        (n, ctypes.c_int32) for n in ("nseg", "out_c", "in_c", "ks", "cc", "ci_off")]


class SrcnnDesc(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("x_cs", ctypes.c_int32), ("x_co", ctypes.c_int32), ("wpk", c_void_p), ("b1", c_void_p),
                ("b2", c_void_p), ("b3", c_void_p), ("out", c_void_p), ("n", ctypes.c_int32), ("h", ctypes.c_int32),
                ("w", ctypes.c_int32)]


class SrcnnBwdDesc(ctypes.Structure):
    _fields_ = [("x", c_void_p), ("x_cs", ctypes.c_int32), ("x_co", ctypes.c_int32), ("gout", c_void_p), ("wpk", c_void_p),
                ("b1", c_void_p), ("b2", c_void_p), ("dz1", c_void_p), ("part", c_void_p), ("gw2", c_void_p), ("gb2", c_void_p),
                ("gw3", c_void_p), ("gb3", c_void_p), ("accumulate", ctypes.c_int32), ("n", ctypes.c_int32),
                ("h", ctypes.c_int32), ("w", ctypes.c_int32)]


class TileDesc(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("hr_raw", "elev_raw", "hr_min", "hr_max", "elev_minmax", "xform", "lr", "hr", "elev",
                                        "mask", "nearest", "elev_lr", "hr_lr")] + [
        (n, c_double) for n in ("range_a", "range_b", "eps", "nan_sub", "zs_hr_mean", "zs_hr_std", "zs_hr_nan_sub",
                                "zs_elev_mean", "zs_elev_std", "zs_elev_nan_sub")] + [("elev_missing", c_float)] + [
        (n, ctypes.c_int32) for n in ("method", "n", "h", "w", "scale", "lr_c", "srcnn", "use_elev", "use_mask")]


SR_METRICS = 17


class MetricsDesc(ctypes.Structure):
    _fields_ = [(n, c_void_p) for n in ("sr", "hr", "original", "mask", "min", "max", "workspace", "out")] + [
        (n, c_double) for n in ("range_a", "range_b", "eps", "zs_mean", "zs_std")] + [("acc_eps", c_float * 8)] + [
        (n, ctypes.c_int32) for n in ("n", "h", "w", "method")]


P = ctypes.POINTER
# name -> (restype, argtypes); must match include/climsr_hip.h exactly (tests/test_abi.py checks the symbols)
SIGNATURES = {
    "climsr_last_error": (ctypes.c_char_p, []),
    "climsr_version": (c_int, []),
    "climsr_conv_chunk": (c_int, [c_int, c_int, c_int]),
    "climsr_conv_chunk_ex": (c_int, [c_int, c_int, c_int, c_int]),
    "climsr_conv_packed_k": (c_int, [c_int, c_int, c_int]),
    "climsr_conv_packed_rows": (c_int, [c_int]),
    "climsr_pack_conv_weight": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "climsr_pack_conv_weights_batched": (c_int, [c_void_p, c_int, c_int64, c_void_p]),
    "climsr_pack_pull_weights_batched": (c_int, [c_void_p, c_int, c_int64, c_void_p]),
    "climsr_rdb_chain": (c_int, [P(ChainDesc), c_void_p]),
    "climsr_rdb_chain_kernel": (ctypes.c_char_p, [P(ChainDesc)]),
    "climsr_rdb_chain_kp": (c_int, [c_int]),
    "climsr_srcnn_fwd": (c_int, [P(SrcnnDesc), c_void_p]),
    "climsr_srcnn_pack": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "climsr_srcnn_packed_elems": (c_int64, []),
    "climsr_srcnn_bwd": (c_int, [P(SrcnnBwdDesc), c_void_p]),
    "climsr_srcnn_bwd_workspace": (c_int64, [c_int, c_int, c_int]),
    "climsr_conv2d_fwd": (c_int, [P(ConvDesc), c_void_p, c_void_p, c_void_p, P(Epilogue), c_void_p, c_void_p]),
    "climsr_conv2d_fwd_bn_parts": (ctypes.c_int64, [P(ConvDesc), P(Epilogue)]),
    "climsr_bn_forward_parts": (c_int, [c_void_p, ctypes.c_int64, c_void_p, ctypes.c_int64, c_int, c_void_p, c_void_p, c_int, c_float,
                                        c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "climsr_conv2d_fwd_kernel": (ctypes.c_char_p, [P(ConvDesc), c_void_p, P(Epilogue)]),
    "climsr_conv2d_wgrad_kernel": (ctypes.c_char_p, [P(ConvDesc)]),
    "climsr_dgrad_single_output_kernel": (ctypes.c_char_p, [c_int, c_int, c_int]),
    "climsr_conv_single_input": (c_int, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int,
                                         c_int, c_float, c_void_p, c_int, c_int, c_void_p]),
    "climsr_dgrad_single_output": (c_int, [c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int,
                                           c_float, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_void_p]),
    "climsr_conv2d_wgrad": (c_int, [P(ConvDesc), c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p]),
    "climsr_conv2d_wgrad_reduce": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                                           c_void_p]),
    "climsr_conv2d_wgrad_splits": (c_int, [P(ConvDesc)]),
    "climsr_conv2d_wgrad_reduce_rows": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int64, c_int,
                                                c_void_p]),
    "climsr_conv2d_wgrad_workspace": (c_size_t, [P(ConvDesc), c_int]),
    "climsr_act_grad": (c_int, [c_int64, c_int, c_void_p, c_int, c_int, c_void_p, c_int, c_int, c_int, c_float, c_float,
                                c_void_p, c_int, c_void_p]),
    "climsr_nchw_to_nhwc_bf16": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p]),
    "climsr_pack_planes_nhwc8_bf16": (c_int, [ctypes.POINTER(Planes8), c_int, c_int, c_int, c_void_p, c_void_p]),
    "climsr_nhwc_to_nchw_f32": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "climsr_axpby_f32": (c_int, [c_int64, c_int, c_float, c_void_p, c_int, c_int, c_float, c_void_p, c_int, c_int, c_void_p]),
    "climsr_rdb_bwd_init": (c_int, [c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_float, c_int, c_int,
                                    c_void_p]),
    "climsr_l1_loss": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "climsr_l1_loss_grad": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "climsr_adamw_hparams": (c_int, [c_void_p, c_int, c_double, c_double, c_double, c_double, c_double, c_double, c_double,
                                     c_void_p, c_void_p]),
    "climsr_adamw_step": (c_int, [c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "climsr_adamw_step_mirror": (c_int, [c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_void_p,
                                         c_void_p]),
    "climsr_bn_workspace_doubles": (c_int64, [c_int64, c_int]),
    "climsr_bn_forward": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_int, c_float, c_float, c_float, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p]),
    "climsr_bn_backward": (c_int, [c_void_p, c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_float, c_float,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "climsr_bn_backward_z": (c_int, [c_void_p, c_int, c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_float,
                                     c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "climsr_bn_backward_parts": (c_int, [c_void_p, ctypes.c_int64, c_void_p, c_void_p, c_int64, c_int, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_float, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    "climsr_reflect_pad1_bf16": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "climsr_reflect_pad1_bwd_f32": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "climsr_adaptive_pool_fwd": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p, c_int,
                                         c_void_p]),
    "climsr_adaptive_pool_bwd": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "climsr_linear_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_float, c_void_p, c_int64,
                                  c_void_p, c_void_p]),
    "climsr_linear_dgrad": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "climsr_linear_wgrad": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "climsr_linear_wgrad2": (c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "climsr_d_head_fwd": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p]),
    "climsr_d_stem_s2": (c_int, [c_void_p, c_void_p]),
    "climsr_conv2d_fwd_pool_ok": (c_int, [c_void_p, c_void_p]),
    "climsr_d_stem_s2_bn_parts": (c_int64, [ctypes.c_int32, ctypes.c_int32, ctypes.c_int32]),
    "climsr_d_head_bwd": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int, c_float, c_int, c_void_p, c_void_p,
                                  c_void_p, c_int, c_void_p, c_void_p, c_void_p]),
    "climsr_relativistic_bce": (c_int, [c_void_p, c_void_p, c_int, c_float, c_float, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p]),
    "climsr_maxpool2_bf16": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    "climsr_l1_loss_bf16": (c_int, [c_void_p, c_void_p, c_int64, c_void_p, c_void_p, c_void_p]),
    "climsr_f32_to_bf16": (c_int, [c_void_p, c_int64, c_void_p, c_void_p]),
    "climsr_bn_inference": (c_int, [c_void_p, c_int64, c_int, c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_int, c_float,
                                    c_void_p, c_void_p]),
    "climsr_increment_i64": (c_int, [c_void_p, c_void_p]),
    "climsr_tile_minmax_f32": (c_int, [c_void_p, c_int, c_int64, c_float, c_int, c_void_p, c_void_p]),
    "climsr_tile_prepare": (c_int, [P(TileDesc), c_void_p]),
    "climsr_resize_cubic_f32": (c_int, [c_void_p, c_int, c_int, c_int, c_void_p, c_int, c_int, c_void_p]),
    "climsr_sr_metrics_workspace": (c_size_t, []),
    "climsr_sr_metrics": (c_int, [P(MetricsDesc), c_void_p]),
    "climsr_regression_accuracy_update": (c_int, [c_void_p, c_void_p, c_int64, c_float, c_void_p, c_void_p]),
    "climsr_denormalize_mask": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_double, c_double, c_int, c_int64, c_void_p,
                                        c_void_p]),
    "climsr_channel_attention_workspace": (c_size_t, [c_int, c_int]),
    "climsr_channel_attention": (c_int, [c_void_p, c_int, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                         c_void_p, c_void_p, c_void_p]),
    "climsr_channel_attention_parts": (c_int, [c_void_p, c_int, c_int, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                               c_int, c_void_p, c_void_p, c_void_p]),
    "climsr_conv2d_fwd_ch_parts": (ctypes.c_int64, [P(ConvDesc), P(Epilogue), c_void_p]),
    "climsr_ca_scale_add": (c_int, [c_void_p, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int, c_int, c_int64, c_int, c_void_p]),
    "climsr_pixel_shuffle_bf16": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "climsr_pixel_unshuffle_bf16": (c_int, [c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_int, c_void_p]),
    "climsr_channel_attention_mean": (c_int, [c_void_p, c_int, c_int64, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int,
                                              c_void_p, c_void_p, c_void_p, c_void_p]),
    "climsr_channel_attention_parts_mean": (c_int, [c_void_p, c_int, c_int, c_int64, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                                    c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "climsr_vgg_conv1_1": (c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_void_p]),
    "climsr_ca_backward_workspace": (c_size_t, [c_int, c_int64, c_int, c_int]),
    "climsr_ca_backward": (c_int, [c_void_p, c_int, c_void_p, c_int, c_int, c_void_p, c_void_p, c_int, c_int64, c_int, c_void_p,
                                   c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int,
                                   c_void_p]),
}

_lib: Optional[ctypes.CDLL] = None


class ClimsrError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load (once) and type the HIP library.  Raises if it is not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ClimsrError(f"libclimsr_hip.so not found at {LIB_PATH}: build it with `python -c 'import __graft_entry__ as g; "
                          f"g.build()'` (the product path has no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    # an A/B build named by CLIMSR_HIP_LIB (tools/perf_*.py) may predate later entry points: those stay unbound and
    # fail when called; the in-tree library must export every one
    ab = "CLIMSR_HIP_LIB" in os.environ
    for name, (res, args) in SIGNATURES.items():
        if ab and not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        msg = load().climsr_last_error().decode(errors="replace")
        raise ClimsrError(f"{what} failed (rc={rc}): {msg}")


def stream_ptr(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t) -> Optional[int]:
    return None if t is None else t.data_ptr()
