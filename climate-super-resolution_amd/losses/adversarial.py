"""Relativistic-average adversarial loss of the GAN task as one native autograd node.

``GANLightningModule.loss_g`` (pl_gan.py:31-38): BCEWithLogits(s_f - mean(s_r), 1) and
BCEWithLogits(s_r - mean(s_f), 0), averaged; ``loss_d`` (pl_gan.py:52-59) swaps the labels.  The
scores are the discriminator's sigmoid outputs, fed to BCE-with-logits exactly as the reference
does (the double sigmoid, F6, is kept).
"""
import torch

from .. import ops


class _RelBCE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, s_real, s_fake, t_rf, t_fr):
        s_real = s_real.contiguous().float()
        s_fake = s_fake.contiguous().float()
        n = s_real.numel()
        loss = torch.empty((), dtype=torch.float32, device=s_real.device)
        ops.relativistic_bce(s_real, s_fake, n, t_rf, t_fr, loss=loss)
        ctx.save_for_backward(s_real, s_fake)
        ctx.t = (t_rf, t_fr)
        return loss

    @staticmethod
    def backward(ctx, g):
        s_real, s_fake = ctx.saved_tensors
        gr = torch.empty_like(s_real)
        gf = torch.empty_like(s_fake)
        ops.relativistic_bce(s_real, s_fake, s_real.numel(), ctx.t[0], ctx.t[1], gscale=g.contiguous().float(), g_real=gr, g_fake=gf)
        return gr, gf, None, None


def relativistic_adversarial_loss(score_real, score_fake, generator_step: bool):
    """generator_step=True: loss_g's adversarial term; False: loss_d."""
    if generator_step:
        return _RelBCE.apply(score_real, score_fake, 0.0, 1.0)
    return _RelBCE.apply(score_real, score_fake, 1.0, 0.0)
