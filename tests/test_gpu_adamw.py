"""The native AdamW update (climsr_adamw_step / climsr_adamw_step_mirror, elementwise.hip; torch.optim.AdamW
single-tensor semantics, conf/optimizers/adamw.yaml) on flat buffers of ragged lengths -- whole blocks, a partial last
block, fewer elements than one vector group -- against the same update in fp64 (rel 1e-6), and the bf16 mirror of
the updated parameters (the discriminator's fc.0 operand) bit-exact against torch's round-to-nearest-even over an
arbitrary sub-range, nothing written outside it."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _hp(lr=3e-4, b1=0.9, b2=0.999, eps=1e-8, wd=1e-2, t=3):
    bc1, bc2 = 1 - b1 ** t, 1 - b2 ** t
    return torch.tensor([lr, b1, b2, eps, wd, lr / bc1, bc2 ** 0.5, 0.0], dtype=torch.float32, device=DEV)


def _want(p, g, m, v, hp):
    lr, b1, b2, eps, wd, ss, bc2s = (float(x) for x in hp[:7].cpu())
    p, g, m, v = (t.double().cpu() for t in (p, g, m, v))
    p = p * (1 - lr * wd)
    m = m + (g - m) * (1 - b1)
    v = v * b2 + g * g * (1 - b2)
    return p - ss * (m / (v.sqrt() / bc2s + eps)), m, v


@pytest.mark.parametrize("n", [1, 3, 4, 1027, 2048, 2049, 4099, 100003])
@pytest.mark.parametrize("mirror", [False, True])
def test_adamw_step_vs_fp64(n, mirror):
    from climsr_amd import _lib
    from climsr_amd._lib import check, ptr

    gen = torch.Generator().manual_seed(n)
    p = torch.randn(n, generator=gen).to(DEV)
    g = (torch.randn(n, generator=gen) * 0.1).to(DEV)
    m = (torch.randn(n, generator=gen) * 0.01).to(DEV)
    v = (torch.rand(n, generator=gen) * 1e-3).to(DEV)
    hp = _hp()
    wp, wm, wv = _want(p, g, m, v, hp)
    L = _lib.load()
    if mirror:
        lo, mn = n // 3, max(1, n - n // 3 - 1)  # (an odd start: not 4-aligned to the vector groups)
        buf = torch.full((mn + 2,), 0x7FC1, dtype=torch.int16, device=DEV)
        check(L.climsr_adamw_step_mirror(n, ptr(p), ptr(g), ptr(m), ptr(v), ptr(hp), lo, mn, buf[1:].data_ptr(), _lib.stream_ptr()),
              "adamw mirror")
    else:
        check(L.climsr_adamw_step(n, ptr(p), ptr(g), ptr(m), ptr(v), ptr(hp), _lib.stream_ptr()), "adamw")
    torch.cuda.synchronize()
    for name, got, want in (("p", p, wp), ("m", m, wm), ("v", v, wv)):
        err = (got.double().cpu() - want).abs().max().item()
        assert err <= 1e-6 * max(want.abs().max().item(), 1e-30), f"{name}: {err}"
    if mirror:
        b = buf.cpu()
        assert b[0].item() == 0x7FC1 and b[-1].item() == 0x7FC1, "mirror written outside its range"
        assert torch.equal(b[1:-1].view(torch.bfloat16), p[lo:lo + mn].cpu().to(torch.bfloat16))
