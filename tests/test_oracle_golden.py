"""Pin the oracle (oracle/climsr_ref.py) against fixtures produced by the REFERENCE's own model files
(tests/golden/make_golden.py) and torch's AdamW/OneCycleLR.  CPU only."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import climsr_ref as ref
from tests.helpers import gen_params, plain_d_params, rfb_d_params, vgg_params


def _load(golden_dir, name):
    return np.load(os.path.join(golden_dir, name))


@pytest.mark.parametrize("tag,nb,b,hr", [("g_nb1_16to64", 1, 2, 64), ("g_nb1_32to128", 1, 2, 128), ("g_nb11_16to64", 11, 1, 64)])
def test_generator_matches_reference(golden_dir, tag, nb, b, hr):
    p = gen_params(nb)
    bt = ref.synthetic_batch(b, hr, dtype=torch.float64)
    with torch.no_grad():
        sr = ref.generator_forward(p, bt["lr"], bt["elevation"], bt["mask"], nb)
    want = _load(golden_dir, tag + ".npz")["sr"]
    assert sr.shape == want.shape
    np.testing.assert_allclose(sr.numpy(), want, rtol=0, atol=1e-12)


def test_generator_state_dict_keys_match_reference(golden_dir):
    man = json.load(open(os.path.join(golden_dir, "manifest.json")))
    for tag, nb in [("g_nb1_16to64", 1), ("g_nb11_16to64", 11)]:
        shapes = ref.generator_shapes(nb=nb)
        assert len(shapes) == man["files"][tag]["n_tensors"]
        assert sum(int(np.prod(s)) for s in shapes.values()) == man["files"][tag]["n_params"]
    # production config nb=11, gc=16: 4,278,530 params, 174 convs
    shapes = ref.generator_shapes(nb=11)
    assert sum(int(np.prod(s)) for s in shapes.values()) == 4278530
    assert sum(1 for k in shapes if k.endswith(".weight")) == 174


@pytest.mark.parametrize("hr", [64, 128])
def test_rfb_discriminator_matches_reference(golden_dir, hr):
    g = _load(golden_dir, "rfb_d.npz")
    p = rfb_d_params()
    x = ref.synthetic_batch(2, hr, seed=7, dtype=torch.float64)["hr"]
    with torch.no_grad():
        s = ref.rfb_discriminator_forward(p, x, training=True)
    np.testing.assert_allclose(s.numpy(), g[f"score_train_{hr}"], rtol=0, atol=1e-12)
    rm = np.concatenate([p[pre + ".running_mean"].numpy() for pre in ref.rfb_bn_prefixes()])
    rv = np.concatenate([p[pre + ".running_var"].numpy() for pre in ref.rfb_bn_prefixes()])
    np.testing.assert_allclose(rm, g[f"running_mean_{hr}"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(rv, g[f"running_var_{hr}"], rtol=1e-12, atol=1e-12)
    with torch.no_grad():
        se = ref.rfb_discriminator_forward(p, x, training=False)
    np.testing.assert_allclose(se.numpy(), g[f"score_eval_after_{hr}"], rtol=0, atol=1e-12)
    assert len(ref.rfb_discriminator_shapes()) == 47


def test_plain_discriminator_matches_reference(golden_dir):
    p = plain_d_params()
    x = ref.synthetic_batch(2, 128, seed=9, dtype=torch.float64)["hr"]
    with torch.no_grad():
        s = ref.plain_discriminator_forward(p, x)
    np.testing.assert_allclose(s.numpy(), _load(golden_dir, "plain_d.npz")["score_train_128"], rtol=0, atol=1e-12)


def test_one_cycle_matches_torch():
    total = 37
    w = torch.zeros(3, requires_grad=True)
    opt = torch.optim.AdamW([w], lr=1e-4)
    sch = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=1e-4, total_steps=total, pct_start=0.05, div_factor=2,
                                              final_div_factor=100)
    for s in range(total):
        lr, b1 = ref.one_cycle(s, total, 1e-4)
        assert abs(lr - opt.param_groups[0]["lr"]) < 1e-18
        assert abs(b1 - opt.param_groups[0]["betas"][0]) < 1e-15
        opt.step()
        sch.step()


def _checks(p, keys):
    return {k: [float(p[k].double().sum()), float(p[k].double().norm())] for k in keys}


def test_pretrain_steps_match_reference(golden_dir):
    want = json.load(open(os.path.join(golden_dir, "pretrain_steps.json")))
    p = gen_params(1)
    keys = list(p.keys())
    opt = ref.AdamWState(p, keys, lr=1e-4, total_steps=10)
    for s in range(3):
        bt = ref.synthetic_batch(2, 64, seed=100 + s, dtype=torch.float64)
        lr, b1 = opt.hparams()
        assert abs(lr - want["lr"][s]) < 1e-18 and abs(b1 - want["beta1"][s]) < 1e-15
        if s == 0:
            for k in keys:
                p[k].requires_grad_(True)
            sr = ref.generator_forward(p, bt["lr"], bt["elevation"], bt["mask"], 1)
            g = torch.autograd.grad(ref.l1_loss(sr, bt["hr"]), [p[k] for k in keys])
            for k in keys:
                p[k].requires_grad_(False)
            for k, gk in zip(keys, g):
                np.testing.assert_allclose([float(gk.sum()), float(gk.norm())], want["grads0"][k], rtol=1e-9, atol=1e-13)
        loss = ref.pretrain_step(p, opt, bt, nb=1)
        assert abs(float(loss) - want["loss"][s]) < 1e-12
    got = _checks(p, keys)
    for k in keys:
        np.testing.assert_allclose(got[k], want["params_after"][k], rtol=1e-10, atol=1e-12)


def test_gan_step_matches_reference(golden_dir):
    want = json.load(open(os.path.join(golden_dir, "gan_step.json")))
    gp, dp, vp = gen_params(1), rfb_d_params(), vgg_params()
    gk = list(gp.keys())
    dk = ref.trainable_keys(dp)
    og = ref.AdamWState(gp, gk, 1e-4, 10)
    od = ref.AdamWState(dp, dk, 1e-4, 10)
    bt = ref.synthetic_batch(2, 128, seed=5, dtype=torch.float64)
    out = ref.gan_step(gp, dp, vp, og, od, bt, nb=1)
    for k in ("loss_G", "adversarial_loss", "perceptual_loss", "pixel_level_loss", "loss_D"):
        assert abs(float(out[k]) - want[k]) <= 1e-10 * max(1.0, abs(want[k])), k
    got = _checks(gp, gk)
    for k in gk:
        np.testing.assert_allclose(got[k], want["g_params_after"][k], rtol=1e-9, atol=1e-12)
    got = _checks(dp, dk)
    for k in dk:
        np.testing.assert_allclose(got[k], want["d_params_after"][k], rtol=1e-9, atol=1e-12)
    bufs = {k: [float(dp[k].sum()), float(dp[k].norm())] for k in dp if k.endswith(("running_mean", "running_var"))}
    for k, v in bufs.items():
        np.testing.assert_allclose(v, want["d_buffers_after"][k], rtol=1e-10, atol=1e-12)


def test_nearest_upsample_index_map_bit_exact():
    x = torch.arange(2 * 3 * 5 * 7, dtype=torch.int64).reshape(2, 3, 5, 7)
    u = ref.upsample_nearest2x(x)
    yy, xx = torch.meshgrid(torch.arange(10), torch.arange(14), indexing="ij")
    assert torch.equal(u, x[:, :, yy >> 1, xx >> 1])
    assert torch.equal(u.double(), torch.nn.functional.interpolate(x.double(), scale_factor=2, mode="nearest"))


def test_adaptive_pool_windows():
    w = ref.adaptive_avg_pool_windows(16, 14)
    assert w[0] == (0, 2) and w[-1] == (14, 16) and len(w) == 14
    x = torch.randn(1, 1, 16, 16, dtype=torch.float64)
    man = torch.stack([torch.stack([x[0, 0, a:b, c:d].mean() for c, d in w]) for a, b in w])
    assert torch.allclose(man, ref.adaptive_avg_pool2d(x, (14, 14))[0, 0])


def test_perceptual_loss_properties():
    """Reference property tests tests/losses/test_pertceptual.py:12-35 (0 for identical, >0 otherwise)."""
    vp = vgg_params(torch.float32)
    g = torch.Generator().manual_seed(0)
    hr = torch.rand(2, 1, 32, 32, generator=g)
    assert float(ref.perceptual_loss(vp, hr.clone(), hr)) == 0.0
    assert float(ref.perceptual_loss(vp, torch.rand(2, 1, 32, 32, generator=g), hr)) != 0.0


@pytest.mark.parametrize("name,ng,nb,sf,b,lr_size", [("rcan_g2b2_x4", 2, 2, 4, 2, 16), ("rcan_g2b2_x2", 2, 2, 2, 1, 24),
                                                     ("rcan_g10b20_x4", 10, 20, 4, 1, 16)])
def test_rcan_oracle_matches_reference(golden_dir, name, ng, nb, sf, b, lr_size):
    """oracle.rcan_forward vs the reference's climsr/models/rcan.py output (tests/golden/make_rcan_golden.py), fp64."""
    import torch

    from climsr_amd.core.init import init_state, spec_from_shapes
    from climsr_amd.models.rcan import RCAN

    shapes = {k: tuple(v.shape) for k, v in RCAN(n_resgroups=ng, n_resblocks=nb, scaling_factor=sf).state_dict().items()}
    p = {k: torch.from_numpy(np.asarray(v)).double() for k, v in init_state(spec_from_shapes(shapes)).items()}
    g = torch.Generator().manual_seed(42)
    hr = lr_size * sf
    t = torch.rand((b, 1, hr, hr), generator=g) * 2 - 1
    e = torch.rand((b, 1, hr, hr), generator=g) * 2 - 1
    m = (torch.rand((b, 1, hr, hr), generator=g) < 0.7).float()
    lr = torch.cat([t, e, m], 1)[:, :, ::sf, ::sf].contiguous()
    got = ref.rcan_forward(p, lr.double(), e.double(), m.double(), ng, nb, sf)
    want = torch.from_numpy(np.load(os.path.join(golden_dir, "rcan.npz"))[name])
    assert (got - want).abs().max().item() <= 1e-10


def test_pixel_shuffle_index_map_bit_exact():
    import torch

    x = torch.arange(2 * 36 * 3 * 5, dtype=torch.float64).reshape(2, 36, 3, 5)
    for r in (2, 3):
        assert torch.equal(ref.pixel_shuffle(x, r), torch.nn.functional.pixel_shuffle(x, r))


@pytest.mark.parametrize("name", ["rcan_g2b2_x4", "rcan_g1b2_x2", "rcan_g1b1_x3"])
def test_rcan_oracle_training_grads_match_reference(golden_dir, name):
    """oracle.rcan_forward + L1 (task.py:141) autograd gradients vs the reference module's own (make_rcan_golden.py,
    tests/golden/rcan_train.json), fp64: loss and every parameter's (sum, norm)."""
    import torch

    from tests.helpers import RCAN_TRAIN, rcan_params, rcan_train_batch

    ng, nb, sf, b, lr_size = RCAN_TRAIN[name]
    want = json.load(open(os.path.join(golden_dir, "rcan_train.json")))[name]
    p = {k: v.requires_grad_(True) for k, v in rcan_params(ng, nb, sf).items()}
    bt = rcan_train_batch(b, lr_size, sf)
    loss = ref.l1_loss(ref.rcan_forward(p, bt["lr"], bt["elevation"], bt["mask"], ng, nb, sf), bt["hr"])
    keys = list(p)
    gs = torch.autograd.grad(loss, [p[k] for k in keys])
    assert abs(float(loss) - want["loss"]) <= 1e-12
    assert set(keys) == set(want["grads"])
    for k, gk in zip(keys, gs):
        np.testing.assert_allclose([float(gk.sum()), float(gk.norm())], want["grads"][k], rtol=1e-9, atol=1e-13, err_msg=k)
