"""ORACLE — test infrastructure only.  CPU restatement of the reference hot path.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
this module, and only as the checker / the timed CPU baseline.  The product package
(``climsr_amd``) never imports it; the product fails loudly when its HIP library is missing.

This is a functional, PyTorch-CPU (fp32 or fp64) restatement of
xultaeculcis/climate-super-resolution @ v1 (``/root/reference``), written from the reference's
behaviour, not copied from it.  Parameters are plain ``{state_dict key: tensor}`` dicts whose keys
equal the reference modules' ``state_dict`` keys, so the same weights drive the reference (golden
fixture generation, ``tests/golden/make_golden.py``), this oracle and the HIP product.

Pinning: ``tests/test_oracle_golden.py`` checks every function here against fixtures produced by
importing the reference's own ``climsr/models/*.py`` read-only (generator, both discriminators,
SRCNN) and against torch's own ``AdamW`` / ``OneCycleLR`` / ``BCEWithLogitsLoss`` (the reference's
pinned dependency for those, ``environment.yml:78``).  VGG19 (``perceptual.py``) and the Lightning
step orchestration (``pl_gan.py``) cannot be imported here (torchvision / pytorch_lightning absent);
they are restated from the reference source and torchvision's published cfg "E"; their numerics are
"parity unpinned" beyond the reference's own property tests (``tests/losses/test_pertceptual.py``).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn.functional as F

Params = Dict[str, torch.Tensor]

# --------------------------------------------------------------------------------------------
# Shapes (state_dict key -> shape).  Mirrors the reference constructors.
# --------------------------------------------------------------------------------------------


def generator_shapes(in_channels: int = 3, out_channels: int = 1, nf: int = 64, nb: int = 11, gc: int = 16,
                     scaling_factor: int = 4) -> Dict[str, Tuple[int, ...]]:
    """``climsr/models/esrgan.py:58-87`` (+ SRCNN tail ``srcnn.py:7-11`` with in_channels=3)."""
    s: Dict[str, Tuple[int, ...]] = {}

    def conv(name, cin, cout, k):
        s[name + ".weight"] = (cout, cin, k, k)
        s[name + ".bias"] = (cout,)

    conv("conv_first", in_channels, nf, 3)
    for i in range(nb):
        for r in (1, 2, 3):
            p = f"RRDB_trunk.{i}.RDB{r}"
            for c in range(1, 5):
                conv(f"{p}.conv{c}", nf + (c - 1) * gc, gc, 3)
            conv(f"{p}.conv5", nf + 4 * gc, nf, 3)
    conv("trunk_conv", nf, nf, 3)
    conv("upconv1", nf, nf, 3)
    if scaling_factor == 4:
        conv("upconv2", nf, nf, 3)
    conv("HRconv", nf, nf, 3)
    conv("conv_last", nf, out_channels, 3)
    conv("srcnn.conv1", 3, 64, 9)
    conv("srcnn.conv2", 64, 32, 1)
    conv("srcnn.conv3", 32, out_channels, 5)
    return s


# RFB-ESRGAN discriminator layer table (rfb_esrgan.py:28-52): (features idx of conv, cin, cout, stride, bn idx or None)
def rfb_d_layers(in_channels: int = 1):
    return [
        (0, in_channels, 64, 1, None),
        (2, 64, 64, 2, 3),
        (5, 64, 128, 1, 6),
        (8, 128, 128, 2, 9),
        (11, 128, 256, 1, 12),
        (14, 256, 256, 2, 15),
        (17, 256, 512, 1, 18),
        (20, 512, 512, 2, 21),
    ]


def rfb_discriminator_shapes(in_channels: int = 1) -> Dict[str, Tuple[int, ...]]:
    """``climsr/models/rfb_esrgan.py:26-61``."""
    s: Dict[str, Tuple[int, ...]] = {}
    for ci, cin, cout, _st, bn in rfb_d_layers(in_channels):
        s[f"features.{ci}.weight"] = (cout, cin, 3, 3)
        if bn is not None:
            s[f"features.{bn}.weight"] = (cout,)
            s[f"features.{bn}.bias"] = (cout,)
            s[f"features.{bn}.running_mean"] = (cout,)
            s[f"features.{bn}.running_var"] = (cout,)
            s[f"features.{bn}.num_batches_tracked"] = ()
    s["fc.0.weight"] = (1024, 512 * 14 * 14)
    s["fc.0.bias"] = (1024,)
    s["fc.2.weight"] = (1, 1024)
    s["fc.2.bias"] = (1,)
    return s


def rfb_bn_prefixes(in_channels: int = 1) -> List[str]:
    return [f"features.{bn}" for _c, _i, _o, _s, bn in rfb_d_layers(in_channels) if bn is not None]


def plain_d_layers(in_channels: int = 1, out_channels: int = 64, num_conv_block: int = 4):
    """``climsr/models/discriminator.py:6-34``: (seq idx of conv, cin, cout, stride, reflect-pad, lrelu slope after,
    bn idx after the lrelu or None)."""
    layers = []
    idx = 0
    cin, cout = in_channels, out_channels
    for _ in range(num_conv_block):
        layers.append((idx + 1, cin, cout, 1, True, 0.01, idx + 3))
        cin = cout
        layers.append((idx + 5, cin, cout, 2, True, 0.01, None))
        idx += 7
        cout *= 2
    cout //= 2
    cin = cout
    layers.append((idx + 0, cin, cout, 1, False, 0.2, None))
    layers.append((idx + 2, cout, cout, 1, False, None, None))
    return layers


def plain_discriminator_shapes(in_channels: int = 1, out_channels: int = 64, num_conv_block: int = 4):
    s: Dict[str, Tuple[int, ...]] = {}
    for ci, cin, cout, _st, _rp, _sl, bn in plain_d_layers(in_channels, out_channels, num_conv_block):
        s[f"feature_extraction.{ci}.weight"] = (cout, cin, 3, 3)
        s[f"feature_extraction.{ci}.bias"] = (cout,)
        if bn is not None:
            for leaf in ("weight", "bias", "running_mean", "running_var"):
                s[f"feature_extraction.{bn}.{leaf}"] = (cout,)
            s[f"feature_extraction.{bn}.num_batches_tracked"] = ()
    s["classification.0.weight"] = (100, 8192)
    s["classification.0.bias"] = (100,)
    s["classification.1.weight"] = (1, 100)
    s["classification.1.bias"] = (1,)
    return s


def plain_bn_prefixes(in_channels: int = 1, out_channels: int = 64, num_conv_block: int = 4) -> List[str]:
    return [f"feature_extraction.{bn}" for *_x, bn in plain_d_layers(in_channels, out_channels, num_conv_block) if bn is not None]


# torchvision VGG19 cfg "E" truncated at features[:35] (perceptual.py:16): conv indices and widths; 'M' = maxpool.
VGG19_E = [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512]


def vgg19_layers():
    """(features idx, cin, cout, relu_after, pool_after) for features[:35]; conv5_4 (idx 34) has no ReLU."""
    out = []
    idx, cin = 0, 3
    for j, v in enumerate(VGG19_E):
        if v == "M":
            idx += 1
            continue
        pool_after = j + 1 < len(VGG19_E) and VGG19_E[j + 1] == "M"
        relu = idx + 1 < 35
        out.append((idx, cin, v, relu, pool_after))
        cin = v
        idx += 2
    return out


def vgg19_shapes() -> Dict[str, Tuple[int, ...]]:
    s = {}
    for idx, cin, cout, _r, _p in vgg19_layers():
        s[f"loss_network.{idx}.weight"] = (cout, cin, 3, 3)
        s[f"loss_network.{idx}.bias"] = (cout,)
    return s


# --------------------------------------------------------------------------------------------
# Forward functions
# --------------------------------------------------------------------------------------------


def _conv(p: Params, name: str, x: torch.Tensor, stride: int = 1, padding: Optional[int] = None) -> torch.Tensor:
    w = p[name + ".weight"]
    b = p.get(name + ".bias")
    if padding is None:
        padding = w.shape[-1] // 2
    return F.conv2d(x, w, b, stride=stride, padding=padding)


def lrelu(x: torch.Tensor, slope: float = 0.2) -> torch.Tensor:
    return F.leaky_relu(x, slope)


def upsample_nearest2x(x: torch.Tensor) -> torch.Tensor:
    """``F.interpolate(scale_factor=2, mode="nearest")`` (esrgan.py:94,97): out[y, x] = in[y >> 1, x >> 1]."""
    return x.repeat_interleave(2, dim=-2).repeat_interleave(2, dim=-1)


def rdb_forward(p: Params, pre: str, x: torch.Tensor) -> torch.Tensor:
    """``ResidualDenseBlock.forward`` (esrgan.py:32-38)."""
    x1 = lrelu(_conv(p, pre + ".conv1", x))
    x2 = lrelu(_conv(p, pre + ".conv2", torch.cat((x, x1), 1)))
    x3 = lrelu(_conv(p, pre + ".conv3", torch.cat((x, x1, x2), 1)))
    x4 = lrelu(_conv(p, pre + ".conv4", torch.cat((x, x1, x2, x3), 1)))
    x5 = _conv(p, pre + ".conv5", torch.cat((x, x1, x2, x3, x4), 1))
    return x5 * 0.2 + x


def rrdb_forward(p: Params, pre: str, x: torch.Tensor) -> torch.Tensor:
    """``ResidualInResidualDenseBlock.forward`` (esrgan.py:50-54)."""
    out = rdb_forward(p, pre + ".RDB1", x)
    out = rdb_forward(p, pre + ".RDB2", out)
    out = rdb_forward(p, pre + ".RDB3", out)
    return out * 0.2 + x


def srcnn_forward(p: Params, x: torch.Tensor, pre: str = "srcnn") -> torch.Tensor:
    """``SRCNN.forward`` (srcnn.py:13-18)."""
    out = F.relu(_conv(p, pre + ".conv1", x))
    out = F.relu(_conv(p, pre + ".conv2", out))
    return _conv(p, pre + ".conv3", out)


def generator_forward(p: Params, x: torch.Tensor, elev: torch.Tensor, mask: torch.Tensor, nb: int,
                      scaling_factor: int = 4) -> torch.Tensor:
    """``ESRGANGenerator.forward`` (esrgan.py:89-102)."""
    fea = _conv(p, "conv_first", x)
    t = fea
    for i in range(nb):
        t = rrdb_forward(p, f"RRDB_trunk.{i}", t)
    fea = fea + _conv(p, "trunk_conv", t)
    fea = lrelu(_conv(p, "upconv1", upsample_nearest2x(fea)))
    if scaling_factor == 4:
        fea = lrelu(_conv(p, "upconv2", upsample_nearest2x(fea)))
    out = _conv(p, "conv_last", lrelu(_conv(p, "HRconv", fea)))
    return srcnn_forward(p, torch.cat([out, elev, mask], 1))


def pixel_shuffle(x: torch.Tensor, r: int) -> torch.Tensor:
    """``nn.PixelShuffle(r)`` (rcan.py:33,40) as an explicit index map: out[c][y*r+i][x*r+j] = in[c*r*r+i*r+j][y][x]."""
    n, c4, h, w = x.shape
    c = c4 // (r * r)
    return x.reshape(n, c, r, r, h, w).permute(0, 1, 4, 2, 5, 3).reshape(n, c, h * r, w * r)


def rcan_forward(p: Params, x: torch.Tensor, elev: torch.Tensor, mask: torch.Tensor, n_resgroups: int, n_resblocks: int,
                 scaling_factor: int = 4) -> torch.Tensor:
    """``RCAN.forward`` (rcan.py:181-192): head, residual groups of RCABs with channel attention (rcan.py:50-107),
    body skip, Upsampler (conv + PixelShuffle per x2 stage, or one x3 stage), last conv, SRCNN."""
    h = _conv(p, "head.0", x)
    t = h
    for g in range(n_resgroups):
        gin = t
        for b in range(n_resblocks):
            pre = f"body.{g}.body.{b}.body"
            u = _conv(p, pre + ".2", F.relu(_conv(p, pre + ".0", t)))
            y = u.mean(dim=(2, 3), keepdim=True)                                   # AdaptiveAvgPool2d(1)
            y = torch.sigmoid(_conv(p, pre + ".3.conv_du.2", F.relu(_conv(p, pre + ".3.conv_du.0", y))))
            t = u * y + t
        t = _conv(p, f"body.{g}.body.{n_resblocks}", t) + gin
    t = _conv(p, f"body.{n_resgroups}", t) + h
    if scaling_factor in (2, 4):
        for k in range(int(math.log2(scaling_factor))):
            t = pixel_shuffle(_conv(p, f"tail.0.{2 * k}", t), 2)
    else:
        t = pixel_shuffle(_conv(p, "tail.0.0", t), 3)
    out = _conv(p, "tail.1", t)
    return srcnn_forward(p, torch.cat([out, elev, mask], 1))


def batch_norm_train(x: torch.Tensor, p: Params, pre: str, training: bool, momentum: float = 0.1,
                     eps: float = 1e-5, update: bool = True) -> torch.Tensor:
    """``nn.BatchNorm2d`` (train: batch stats over N,H,W with biased var for normalisation, unbiased var
    for the running estimate; eval: running stats)."""
    w, b = p[pre + ".weight"], p[pre + ".bias"]
    rm, rv = p[pre + ".running_mean"], p[pre + ".running_var"]
    if training:
        mean = x.mean(dim=(0, 2, 3))
        var = x.var(dim=(0, 2, 3), unbiased=False)
        if update:
            n = x.numel() / x.shape[1]
            with torch.no_grad():
                rm.mul_(1 - momentum).add_(momentum * mean.detach().to(rm.dtype))
                rv.mul_(1 - momentum).add_(momentum * (var.detach() * n / max(n - 1, 1)).to(rv.dtype))
                nbt = pre + ".num_batches_tracked"
                if nbt in p:
                    p[nbt].add_(1)
    else:
        mean, var = rm, rv
    xh = (x - mean[None, :, None, None]) / torch.sqrt(var[None, :, None, None] + eps)
    return xh * w[None, :, None, None] + b[None, :, None, None]


def adaptive_avg_pool_windows(inp: int, out: int) -> List[Tuple[int, int]]:
    """``nn.AdaptiveAvgPool2d`` window i = [floor(i*in/out), ceil((i+1)*in/out))."""
    return [((i * inp) // out, -((-(i + 1) * inp) // out)) for i in range(out)]


def adaptive_avg_pool2d(x: torch.Tensor, out_hw: Tuple[int, int]) -> torch.Tensor:
    return F.adaptive_avg_pool2d(x, out_hw)


def rfb_discriminator_forward(p: Params, x: torch.Tensor, training: bool = True, update_stats: bool = True,
                              in_channels: int = 1) -> torch.Tensor:
    """``RFBESRGANDiscriminator.forward`` (rfb_esrgan.py:63-69)."""
    out = x
    for ci, _cin, _cout, st, bn in rfb_d_layers(in_channels):
        out = _conv(p, f"features.{ci}", out, stride=st, padding=1)
        if bn is not None:
            out = batch_norm_train(out, p, f"features.{bn}", training, update=update_stats)
        out = lrelu(out, 0.2)
    out = adaptive_avg_pool2d(out, (14, 14))
    out = torch.flatten(out, 1)
    out = lrelu(F.linear(out, p["fc.0.weight"], p["fc.0.bias"]), 0.2)
    out = F.linear(out, p["fc.2.weight"], p["fc.2.bias"])
    return torch.sigmoid(out)


def plain_discriminator_forward(p: Params, x: torch.Tensor, training: bool = True, update_stats: bool = True) -> torch.Tensor:
    """``Discriminator.forward`` (discriminator.py:42-46); only valid at 128x128 input (F6)."""
    out = x
    for ci, _cin, _cout, st, rpad, slope, bn in plain_d_layers():
        if rpad:
            out = F.pad(out, (1, 1, 1, 1), mode="reflect")
        out = _conv(p, f"feature_extraction.{ci}", out, stride=st, padding=0)
        if slope is not None:
            out = lrelu(out, slope)
        if bn is not None:
            out = batch_norm_train(out, p, f"feature_extraction.{bn}", training, update=update_stats)
    out = out.reshape(out.shape[0], -1)
    out = F.linear(out, p["classification.0.weight"], p["classification.0.bias"])
    return F.linear(out, p["classification.1.weight"], p["classification.1.bias"])


def vgg19_features(p: Params, x: torch.Tensor) -> torch.Tensor:
    """torchvision ``vgg19().features[:35]`` (perceptual.py:16)."""
    out = x
    for idx, _cin, _cout, relu, pool in vgg19_layers():
        out = _conv(p, f"loss_network.{idx}", out, padding=1)
        if relu:
            out = F.relu(out)
        if pool:
            out = F.max_pool2d(out, 2, 2)
    return out


def perceptual_loss(p: Params, a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """``PerceptualLoss.forward`` (perceptual.py:22-36): L1 of VGG features on 1->3 channel repeats, no grad."""
    with torch.no_grad():
        fa = vgg19_features(p, torch.cat([a, a, a], 1))
        fb = vgg19_features(p, torch.cat([b, b, b], 1))
        return (fa - fb).abs().mean()


def l1_loss(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    return (a - b).abs().mean()


def bce_with_logits(x: torch.Tensor, y: torch.Tensor) -> torch.Tensor:
    """``nn.BCEWithLogitsLoss`` (mean): max(x,0) - x*y + log1p(exp(-|x|))."""
    return (torch.clamp(x, min=0) - x * y + torch.log1p(torch.exp(-x.abs()))).mean()


# --------------------------------------------------------------------------------------------
# Losses of the GAN task (pl_gan.py:28-61)
# --------------------------------------------------------------------------------------------

LOSS_FACTORS = {"pixel_level_loss_factor": 0.01, "perceptual_loss_factor": 1.0, "adversarial_loss_factor": 0.005}


def loss_g(d_fn, vgg_p: Params, hr, sr, factors=LOSS_FACTORS):
    """``GANLightningModule.loss_g`` (pl_gan.py:28-49).  ``d_fn`` is the discriminator callable; it is
    called separately on hr and sr (F8: per-call BN statistics)."""
    n = hr.shape[0]
    real = torch.ones((n, 1), dtype=hr.dtype, device=hr.device)
    fake = torch.zeros((n, 1), dtype=hr.dtype, device=hr.device)
    score_real = d_fn(hr)
    score_fake = d_fn(sr)
    rf = score_real - score_fake.mean()
    fr = score_fake - score_real.mean()
    adv = (bce_with_logits(fr, real) + bce_with_logits(rf, fake)) / 2
    perc = perceptual_loss(vgg_p, hr, sr)
    pix = l1_loss(sr, hr)
    total = (factors["pixel_level_loss_factor"] * pix + factors["perceptual_loss_factor"] * perc
             + factors["adversarial_loss_factor"] * adv)
    return perc, adv, pix, total


def loss_d(d_fn, hr, sr):
    """``GANLightningModule.loss_d`` (pl_gan.py:51-61)."""
    n = hr.shape[0]
    real = torch.ones((n, 1), dtype=hr.dtype, device=hr.device)
    fake = torch.zeros((n, 1), dtype=hr.dtype, device=hr.device)
    score_real = d_fn(hr)
    score_fake = d_fn(sr.detach())
    rf = score_real - score_fake.mean()
    fr = score_fake - score_real.mean()
    return (bce_with_logits(fr, fake) + bce_with_logits(rf, real)) / 2


# --------------------------------------------------------------------------------------------
# Optimiser + schedule (conf/optimizers/adamw.yaml, conf/schedulers/one_cycle_schedule.yaml)
# --------------------------------------------------------------------------------------------


def one_cycle(step: int, total_steps: int, max_lr: float, pct_start: float = 0.05, div_factor: float = 2.0,
              final_div_factor: float = 100.0, base_momentum: float = 0.85, max_momentum: float = 0.95):
    """torch ``OneCycleLR`` (cos annealing, two phases, cycle_momentum on Adam beta1) at ``last_epoch=step``.
    Returns (lr, beta1).  Wired by ``climsr/core/instantiator.py:51-64`` with total_steps=num_training_steps."""
    initial_lr = max_lr / div_factor
    min_lr = initial_lr / final_div_factor

    def cos_anneal(start, end, pct):
        return end + (start - end) / 2.0 * (math.cos(math.pi * pct) + 1)

    phases = [
        (float(pct_start * total_steps) - 1, initial_lr, max_lr, max_momentum, base_momentum),
        (total_steps - 1, max_lr, min_lr, base_momentum, max_momentum),
    ]
    start = 0.0
    lr = mom = None
    for i, (end, lr0, lr1, m0, m1) in enumerate(phases):
        if step <= end or i == len(phases) - 1:
            pct = (step - start) / (end - start)
            lr = cos_anneal(lr0, lr1, pct)
            mom = cos_anneal(m0, m1, pct)
            break
        start = end
    return lr, mom


def adamw_update(param: torch.Tensor, grad: torch.Tensor, exp_avg: torch.Tensor, exp_avg_sq: torch.Tensor, step: int,
                 lr: float, beta1: float, beta2: float = 0.999, eps: float = 1e-8, weight_decay: float = 1e-4) -> None:
    """torch ``AdamW`` (amsgrad=False): decoupled decay, bias-corrected moments; in place."""
    param.mul_(1 - lr * weight_decay)
    exp_avg.mul_(beta1).add_(grad, alpha=1 - beta1)
    exp_avg_sq.mul_(beta2).addcmul_(grad, grad, value=1 - beta2)
    bc1 = 1 - beta1 ** step
    bc2 = 1 - beta2 ** step
    denom = (exp_avg_sq.sqrt() / math.sqrt(bc2)).add_(eps)
    param.addcdiv_(exp_avg, denom, value=-lr / bc1)


class AdamWState:
    """Per-network optimiser state for the oracle step."""

    def __init__(self, params: Params, keys: List[str], lr: float, total_steps: int, weight_decay: float = 1e-4):
        self.keys = keys
        self.max_lr = lr
        self.total_steps = total_steps
        self.wd = weight_decay
        self.m = {k: torch.zeros_like(params[k]) for k in keys}
        self.v = {k: torch.zeros_like(params[k]) for k in keys}
        self.step_count = 0      # optimizer steps taken
        self.sched_step = 0      # scheduler last_epoch

    def hparams(self):
        return one_cycle(self.sched_step, self.total_steps, self.max_lr)

    def step(self, params: Params, grads: Params):
        self.step_count += 1
        lr, beta1 = self.hparams()
        with torch.no_grad():
            for k in self.keys:
                adamw_update(params[k], grads[k], self.m[k], self.v[k], self.step_count, lr, beta1, weight_decay=self.wd)

    def sched(self):
        self.sched_step += 1


# --------------------------------------------------------------------------------------------
# Task steps (Lightning-1.x automatic optimisation semantics)
# --------------------------------------------------------------------------------------------


def _grads(loss, params: Params, keys: List[str]) -> Params:
    ts = [params[k] for k in keys]
    gs = torch.autograd.grad(loss, ts, allow_unused=True)
    return {k: (g if g is not None else torch.zeros_like(t)) for k, t, g in zip(keys, ts, gs)}


def trainable_keys(p: Params) -> List[str]:
    return [k for k, v in p.items() if v.is_floating_point() and not k.endswith(("running_mean", "running_var"))]


def pretrain_step(g_p: Params, opt: AdamWState, batch: Dict[str, torch.Tensor], nb: int) -> torch.Tensor:
    """``SuperResolutionLightningModule.training_step`` (pl_generator_pre_training.py:18-33) with
    ``L1Loss`` (task.py:141), then AdamW + OneCycleLR(interval=step)."""
    for k in opt.keys:
        g_p[k].requires_grad_(True)
    sr = generator_forward(g_p, batch["lr"], batch["elevation"], batch["mask"], nb)
    loss = l1_loss(sr, batch["hr"])
    grads = _grads(loss, g_p, opt.keys)
    for k in opt.keys:
        g_p[k].requires_grad_(False)
    opt.step(g_p, grads)
    opt.sched()
    return loss.detach()


def gan_step(g_p: Params, d_p: Params, vgg_p: Params, opt_g: AdamWState, opt_d: AdamWState,
             batch: Dict[str, torch.Tensor], nb: int, d_forward=rfb_discriminator_forward, factors=LOSS_FACTORS):
    """``GANLightningModule.training_step`` for optimizer_idx 0 then 1 (pl_gan.py:63-97), PL-1.x order:
    G pass (D frozen) -> AdamW_G; D pass with a fresh G forward (updated weights) -> AdamW_D; then both
    OneCycleLR schedulers step."""
    hr = batch["hr"]
    # ---- optimizer_idx = 0 (generator)
    for k in opt_g.keys:
        g_p[k].requires_grad_(True)
    sr = generator_forward(g_p, batch["lr"], batch["elevation"], batch["mask"], nb)
    d_fn = lambda t: d_forward(d_p, t, training=True)  # noqa: E731
    perc, adv, pix, lg = loss_g(d_fn, vgg_p, hr, sr, factors)
    grads_g = _grads(lg, g_p, opt_g.keys)
    for k in opt_g.keys:
        g_p[k].requires_grad_(False)
    opt_g.step(g_p, grads_g)
    # ---- optimizer_idx = 1 (discriminator)
    with torch.no_grad():
        sr2 = generator_forward(g_p, batch["lr"], batch["elevation"], batch["mask"], nb)
    for k in opt_d.keys:
        d_p[k].requires_grad_(True)
    ld = loss_d(d_fn, hr, sr2)
    grads_d = _grads(ld, d_p, opt_d.keys)
    for k in opt_d.keys:
        d_p[k].requires_grad_(False)
    opt_d.step(d_p, grads_d)
    opt_g.sched()
    opt_d.sched()
    return {"perceptual_loss": perc.detach(), "adversarial_loss": adv.detach(), "pixel_level_loss": pix.detach(),
            "loss_G": lg.detach(), "loss_D": ld.detach()}


# --------------------------------------------------------------------------------------------
# Synthetic batch: seed 42 (+rank), HR temp/elev U(-1,1), mask Bernoulli(0.7),
# LR = cat([temp, elev, mask])[:, :, ::4, ::4]  (cv2 INTER_NEAREST 1/4 decimation, climate_dataset.py:84-90)
# --------------------------------------------------------------------------------------------


def synthetic_batch(batch: int, hr_size: int, seed: int = 42, scale: int = 4, dtype=torch.float32) -> Dict[str, torch.Tensor]:
    g = torch.Generator().manual_seed(seed)
    hr = torch.rand((batch, 1, hr_size, hr_size), generator=g) * 2 - 1
    elev = torch.rand((batch, 1, hr_size, hr_size), generator=g) * 2 - 1
    mask = (torch.rand((batch, 1, hr_size, hr_size), generator=g) < 0.7).float()
    lr = torch.cat([hr, elev, mask], 1)[:, :, ::scale, ::scale].contiguous()
    return {k: v.to(dtype) for k, v in {"lr": lr, "hr": hr, "elevation": elev, "mask": mask}.items()}
