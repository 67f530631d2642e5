"""CPU checks of the C ABI boundary (no GPU compute): the library loads, exports every symbol
include/climsr_hip.h declares, the ctypes signatures cover them, host-side geometry helpers and
argument validation behave."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "climsr_hip.h")
CSRC = os.path.join(ROOT, "climate-super-resolution_amd", "csrc")


@pytest.fixture(scope="module")
def lib():
    so = os.path.join(CSRC, "libclimsr_hip.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", CSRC, "-j8"], check=True, capture_output=True)
    import climsr_amd  # noqa: F401
    from climsr_amd import _lib

    return _lib.load()


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(climsr_[a-z0-9_]+)\s*\(", txt)))


def test_header_declares_the_hot_path():
    fns = header_functions()
    for need in ("climsr_conv2d_fwd", "climsr_conv2d_wgrad", "climsr_conv2d_wgrad_reduce", "climsr_pack_conv_weight",
                 "climsr_act_grad", "climsr_l1_loss", "climsr_adamw_step", "climsr_last_error"):
        assert need in fns


def test_every_declared_symbol_is_exported_and_bound(lib):
    from climsr_amd import _lib

    for name in header_functions():
        assert hasattr(lib, name), f"{name} declared in climsr_hip.h but not exported"
        assert name in _lib.SIGNATURES, f"{name} has no ctypes signature in _lib.py"
    assert set(_lib.SIGNATURES) <= set(header_functions())


def test_struct_layouts_match_header(lib):
    from climsr_amd import _lib

    assert ctypes.sizeof(_lib.ConvDesc) == 16 * 4
    # ClimsrEpilogue: int, float, float, ptr, int, int, float, ptr, int, int, int, int, int, float, float, int, ptr,
    # int, float, ptr (bn_part), ptr (bn_z), int, float, 4 ptrs (natural alignment)
    assert ctypes.sizeof(_lib.Epilogue) == 168  # ... bn_beta, ch_part (pointer), pool2 (int, padded)
    assert _lib.Epilogue.aux.offset == 80 and _lib.Epilogue.aux_scale.offset == 92
    assert _lib.Epilogue().beta1 == 1.0 and _lib.Epilogue().beta2 == 1.0
    # ClimsrPullPackDesc: ptr, ptr[5], int[5], int[5], 6 ints
    assert ctypes.sizeof(_lib.PullPackDesc) == 8 + 40 + 20 + 20 + 24
    assert ctypes.sizeof(_lib.PackDesc) == 2 * 8 + 8 * 4


STRUCTS = {"ConvDesc": "ClimsrConvDesc", "Epilogue": "ClimsrEpilogue", "PackDesc": "ClimsrPackDesc",
           "ReduceDesc": "ClimsrReduceDesc", "ChainDesc": "ClimsrChainDesc", "PullPackDesc": "ClimsrPullPackDesc",
           "TileDesc": "ClimsrTileDesc", "MetricsDesc": "ClimsrMetricsDesc", "Planes8": "ClimsrPlanes8"}


def test_struct_offsets_match_gcc(lib, tmp_path):
    """Every ctypes mirror has the size and field offsets gcc gives the header's C struct."""
    from climsr_amd import _lib

    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "climsr_hip.h"', "int main(void) {"]
    for py, c in STRUCTS.items():
        lines.append(f'printf("{py} size %zu\\n", sizeof({c}));')
        for f in getattr(_lib, py)._fields_:
            lines.append(f'printf("{py} {f[0]} %zu\\n", offsetof({c}, {f[0]}));')
    lines += ["return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    for row in filter(None, out):
        py, field, val = row.split()
        cls = getattr(_lib, py)
        got = ctypes.sizeof(cls) if field == "size" else getattr(cls, field).offset
        assert got == int(val), f"{py}.{field}: ctypes {got} != C {val}"


def test_geometry_helpers(lib):
    assert lib.climsr_version() >= 1
    # chunking keeps the staged LDS tile within budget; packed K is a multiple of 32 per chunk
    for cin, ks, cout in [(64, 3, 16), (128, 3, 64), (112, 3, 16), (8, 9, 64), (512, 3, 512)]:
        cc = lib.climsr_conv_chunk(cin, ks, cout)
        if cout <= 16 and ks == 3 and cin <= 128:  # n16 kernel: one chunk, channels padded to 32/64/128
            assert cc == (32 if cin <= 32 else 64 if cin <= 64 else 128)
        else:
            assert cc % 8 == 0 and 8 <= cc <= cin
        k = lib.climsr_conv_packed_k(cin, ks, cc)
        assert k % 32 == 0 and k >= ks * ks * cin
    assert lib.climsr_conv_chunk_ex(112, 3, 16, 2) != 128  # stride 2: generic chunk
    assert lib.climsr_conv_packed_rows(1) == 16
    assert lib.climsr_conv_packed_rows(48) == 64
    assert lib.climsr_conv_packed_rows(512) == 512


def test_argument_validation_does_not_touch_the_gpu(lib):
    from climsr_amd import _lib

    d = _lib.ConvDesc(2, 16, 16, 7, 8, 0, 1, 3, 1, 1, 16, 16, 16, 16, 0, 8)  # in_c not a multiple of 8
    ep = _lib.Epilogue()
    assert lib.climsr_conv2d_fwd(ctypes.byref(d), 1, 1, None, ctypes.byref(ep), 1, None) == -1
    assert b"unsupported geometry" in lib.climsr_last_error()
    assert lib.climsr_conv2d_fwd(None, None, None, None, None, None, None) == -1
    d = _lib.ConvDesc(2, 16, 16, 8, 8, 0, 1, 3, 1, 1, 16, 16, 16, 16, 0, 8)
    ep = _lib.Epilogue(act=3)  # activation backward needs res1 (the activation output) as its mask source
    assert lib.climsr_conv2d_fwd(ctypes.byref(d), 1, 1, None, ctypes.byref(ep), 1, None) == -1
    assert b"act 3" in lib.climsr_last_error()
    assert lib.climsr_pack_pull_weights_batched(None, 0, 0, None) == -1
    assert lib.climsr_adamw_step(0, None, None, None, None, None, None) == -1
    assert lib.climsr_l1_loss(None, None, 0, None, None, None) == -1


def test_product_has_no_cpu_fallback():
    """The native modules refuse CPU tensors instead of silently computing elsewhere."""
    import torch

    from climsr_amd.models.esrgan import ESRGANGenerator

    g = ESRGANGenerator(3, 1, nf=64, nb=1, gc=16)
    x = torch.zeros(1, 3, 8, 8)
    e = torch.zeros(1, 1, 32, 32)
    with pytest.raises(RuntimeError, match="GPU only"):
        g(x, e, e)


def test_plain_discriminator_drop_in_keys():
    """climsr_amd.models.discriminator.Discriminator has the reference's state_dict (discriminator.py:6-40)."""
    import torch

    from climsr_amd.models.discriminator import Discriminator
    from oracle import climsr_ref as ref

    d = Discriminator()
    sd = d.state_dict()
    shapes = ref.plain_discriminator_shapes()
    assert set(sd) == set(shapes)
    assert all(tuple(sd[k].shape) == tuple(shapes[k]) for k in sd)
    with pytest.raises(RuntimeError, match="GPU only"):
        d(torch.zeros(1, 1, 128, 128))
