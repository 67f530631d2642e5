"""Generate the committed golden fixtures by running the REFERENCE's own model files.

Run in the build container (needs /root/reference; never on the GPU box):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports ``climsr.models.{esrgan,rfb_esrgan,discriminator,srcnn}`` read-only from
/root/reference, loads the deterministic weights of ``climsr_amd.core.init`` by state_dict key,
and records outputs (fp64), loss scalars, per-tensor gradient checksums and post-optimizer-step
parameter checksums.  The optimizer/schedule are torch's own ``AdamW`` and ``OneCycleLR`` (the
reference's dependency, wired as in ``climsr/core/instantiator.py:48-64``); the Lightning step order
is restated from ``climsr/task/pl_gan.py:63-97`` (Lightning itself is not importable here).
VGG19[:35] is rebuilt from torchvision's cfg "E" (torchvision is absent; ImageNet weights cannot be
fetched) with deterministic random weights — numerics of that piece are parity-unpinned.
Outputs: tests/golden/*.npz + manifest.json.
"""
import json
import os
import sys
import time

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, "/root/reference")

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

from climsr.models.discriminator import Discriminator  # noqa: E402  (reference)
from climsr.models.esrgan import ESRGANGenerator  # noqa: E402  (reference)
from climsr.models.rfb_esrgan import RFBESRGANDiscriminator  # noqa: E402  (reference)

from climsr_amd.core.init import spec_from_shapes, init_state  # noqa: E402

torch.set_num_threads(8)


def det_state(module, bn_prefixes=(), gain=1.0):
    shapes = {k: tuple(v.shape) for k, v in module.state_dict().items()}
    return init_state(spec_from_shapes(shapes, bn_prefixes), gain=gain)


def load(module, st):
    module.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    return module


def batch(b, hr, seed=42):
    g = torch.Generator().manual_seed(seed)
    t = torch.rand((b, 1, hr, hr), generator=g) * 2 - 1
    e = torch.rand((b, 1, hr, hr), generator=g) * 2 - 1
    m = (torch.rand((b, 1, hr, hr), generator=g) < 0.7).float()
    lr = torch.cat([t, e, m], 1)[:, :, ::4, ::4].contiguous()
    return {"lr": lr, "hr": t, "elevation": e, "mask": m}


def to64(bt):
    return {k: v.double() for k, v in bt.items()}


def bn_prefixes_of(module):
    return [n for n, m in module.named_modules() if isinstance(m, nn.BatchNorm2d)]


def vgg_seq():
    cfg = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]
    layers, cin = [], 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2d(2, 2))
        else:
            layers += [nn.Conv2d(cin, v, 3, padding=1), nn.ReLU(inplace=True)]
            cin = v
    return nn.Sequential(*layers[:35])


def checks(named):
    return {k: [float(v.double().sum()), float(v.double().norm())] for k, v in named}


def main():
    out = {}
    manifest = {"torch": torch.__version__, "seed": 42, "reference": "/root/reference (xultaeculcis/climate-super-resolution @ v1)",
                "files": {}}
    t0 = time.time()

    # ---------------- generator forward fixtures ----------------
    for tag, nb, b, hr in [("g_nb1_16to64", 1, 2, 64), ("g_nb1_32to128", 1, 2, 128), ("g_nb11_16to64", 11, 1, 64)]:
        g = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=nb, gc=16, scale_factor=4)
        st = det_state(g)
        load(g, st)
        g = g.double().eval()
        bt = to64(batch(b, hr))
        with torch.no_grad():
            sr = g(bt["lr"], bt["elevation"], bt["mask"])
        g32 = load(ESRGANGenerator(3, 1, nf=64, nb=nb, gc=16), st).eval()
        with torch.no_grad():
            sr32 = g32(*(v.float() for v in (bt["lr"], bt["elevation"], bt["mask"])))
        np.savez_compressed(os.path.join(HERE, tag + ".npz"), sr=sr.numpy(), sr_fp32=sr32.numpy())
        manifest["files"][tag] = {"nb": nb, "batch": b, "hr": hr, "keys": list(st.keys())[:3] + ["..."],
                                  "n_tensors": len(st), "n_params": int(sum(v.size for v in st.values())),
                                  "fp32_vs_fp64_maxabs": float((sr32.double() - sr).abs().max())}
        print(tag, "done", time.time() - t0, flush=True)

    # ---------------- discriminators ----------------
    d = RFBESRGANDiscriminator(in_channels=1)
    bnp = bn_prefixes_of(d)
    dst = det_state(d, bnp)
    load(d, dst)
    d = d.double().train()
    res = {}
    for hr in (64, 128):
        x = batch(2, hr, seed=7)["hr"].double()
        dd = load(RFBESRGANDiscriminator(1), dst).double().train()
        with torch.no_grad():
            res[f"score_train_{hr}"] = dd(x).numpy()
        res[f"running_mean_{hr}"] = np.concatenate([dd.state_dict()[p + ".running_mean"].numpy() for p in bnp])
        res[f"running_var_{hr}"] = np.concatenate([dd.state_dict()[p + ".running_var"].numpy() for p in bnp])
        dd.eval()
        with torch.no_grad():
            res[f"score_eval_after_{hr}"] = dd(x).numpy()
    np.savez_compressed(os.path.join(HERE, "rfb_d.npz"), **res)
    manifest["files"]["rfb_d"] = {"n_tensors": len(dst), "bn": bnp}
    print("rfb_d done", time.time() - t0, flush=True)

    pd_ = Discriminator(in_channels=1, out_channels=64, num_conv_block=4)
    pbn = bn_prefixes_of(pd_)
    pst = det_state(pd_, pbn)
    load(pd_, pst)
    pd_ = pd_.double().train()
    x = batch(2, 128, seed=9)["hr"].double()
    with torch.no_grad():
        ps = pd_(x).numpy()
    np.savez_compressed(os.path.join(HERE, "plain_d.npz"), score_train_128=ps)
    manifest["files"]["plain_d"] = {"n_tensors": len(pst), "bn": pbn}

    # ---------------- L1 pretrain steps (nb=1, B=2, 16->64), 3 steps ----------------
    g = load(ESRGANGenerator(3, 1, nf=64, nb=1, gc=16), det_state(ESRGANGenerator(3, 1, nf=64, nb=1, gc=16))).double().train()
    opt = torch.optim.AdamW(g.parameters(), lr=1e-4, weight_decay=1e-4)
    sch = torch.optim.lr_scheduler.OneCycleLR(opt, max_lr=1e-4, total_steps=10, epochs=1, pct_start=0.05, div_factor=2,
                                              final_div_factor=100)
    crit = nn.L1Loss()
    rec = {}
    for s in range(3):
        bt = to64(batch(2, 64, seed=100 + s))
        opt.zero_grad()
        sr = g(bt["lr"], bt["elevation"], bt["mask"])
        loss = crit(sr, bt["hr"])
        loss.backward()
        if s == 0:
            rec["grads0"] = checks((k, p.grad) for k, p in g.named_parameters())
        rec.setdefault("loss", []).append(float(loss))
        rec.setdefault("lr", []).append(opt.param_groups[0]["lr"])
        rec.setdefault("beta1", []).append(opt.param_groups[0]["betas"][0])
        opt.step()
        sch.step()
    rec["params_after"] = checks(g.named_parameters())
    with open(os.path.join(HERE, "pretrain_steps.json"), "w") as f:
        json.dump(rec, f)
    print("pretrain done", time.time() - t0, flush=True)

    # ---------------- one full GAN step (nb=1, B=2, 32->128, RFB-D) ----------------
    g = load(ESRGANGenerator(3, 1, nf=64, nb=1, gc=16), det_state(ESRGANGenerator(3, 1, nf=64, nb=1, gc=16))).double()
    d = load(RFBESRGANDiscriminator(1), dst).double().train()
    holder = nn.Module()
    holder.loss_network = vgg_seq()  # same state_dict keys as PerceptualLoss (perceptual.py:17-19)
    vst = det_state(holder, gain=float(np.sqrt(6.0)))
    load(holder, vst)
    vgg = holder.loss_network.double().eval()
    for p_ in vgg.parameters():
        p_.requires_grad_(False)
    bce, l1 = nn.BCEWithLogitsLoss(), nn.L1Loss()

    def perceptual(a, b):
        with torch.no_grad():
            return l1(vgg(torch.cat([a, a, a], 1)), vgg(torch.cat([b, b, b], 1)))

    og = torch.optim.AdamW(g.parameters(), lr=1e-4, weight_decay=1e-4)
    od = torch.optim.AdamW(d.parameters(), lr=1e-4, weight_decay=1e-4)
    sg = torch.optim.lr_scheduler.OneCycleLR(og, max_lr=1e-4, total_steps=10, pct_start=0.05, div_factor=2, final_div_factor=100)
    sd = torch.optim.lr_scheduler.OneCycleLR(od, max_lr=1e-4, total_steps=10, pct_start=0.05, div_factor=2, final_div_factor=100)
    bt = to64(batch(2, 128, seed=5))
    hr = bt["hr"]
    real, fake = torch.ones((2, 1), dtype=torch.float64), torch.zeros((2, 1), dtype=torch.float64)
    # optimizer_idx 0 (Lightning toggles D params off)
    for p_ in d.parameters():
        p_.requires_grad_(False)
    og.zero_grad()
    sr = g(bt["lr"], bt["elevation"], bt["mask"])
    s_r, s_f = d(hr), d(sr)
    adv = (bce(s_f - s_r.mean(), real) + bce(s_r - s_f.mean(), fake)) / 2
    perc = perceptual(hr, sr)
    pix = l1(sr, hr)
    lg = 0.01 * pix + 1.0 * perc + 0.005 * adv
    lg.backward()
    gan = {"loss_G": float(lg), "adversarial_loss": float(adv), "perceptual_loss": float(perc), "pixel_level_loss": float(pix),
           "grads_g": checks((k, p_.grad) for k, p_ in g.named_parameters()), "sr": sr.detach().double().flatten()[:64].tolist()}
    og.step()
    for p_ in d.parameters():
        p_.requires_grad_(True)
    # optimizer_idx 1 (G toggled off; common_step runs G again with updated weights)
    for p_ in g.parameters():
        p_.requires_grad_(False)
    od.zero_grad()
    with torch.no_grad():
        sr2 = g(bt["lr"], bt["elevation"], bt["mask"])
    s_r, s_f = d(hr), d(sr2.detach())
    ld = (bce(s_f - s_r.mean(), fake) + bce(s_r - s_f.mean(), real)) / 2
    ld.backward()
    gan["loss_D"] = float(ld)
    gan["grads_d"] = checks((k, p_.grad) for k, p_ in d.named_parameters())
    od.step()
    sg.step()
    sd.step()
    gan["g_params_after"] = checks(g.named_parameters())
    gan["d_params_after"] = checks(d.named_parameters())
    gan["d_buffers_after"] = checks((k, v) for k, v in d.named_buffers() if v.is_floating_point())
    with open(os.path.join(HERE, "gan_step.json"), "w") as f:
        json.dump(gan, f)
    manifest["files"]["gan_step"] = {"batch": 2, "hr": 128, "nb": 1, "vgg_init_gain": "sqrt(6)"}
    print("gan done", time.time() - t0, flush=True)

    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
