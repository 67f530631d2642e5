"""GAN task (mirror of climsr/task/pl_gan.py:12-97) on the native G, D, VGG and losses."""
from typing import Any, Dict, Optional, Tuple

import torch
from torch import Tensor

from ..core.task import TaskSuperResolutionModule
from ..losses.adversarial import relativistic_adversarial_loss
from ..losses.l1 import L1Loss
from ..losses.perceptual import PerceptualLoss


class GANLightningModule(TaskSuperResolutionModule):
    def __init__(self, *args, **kwargs):
        kwargs.setdefault("pixel_level_loss_factor", 0.01)       # conf/task/gan_training.yaml:6-8
        kwargs.setdefault("perceptual_loss_factor", 1.0)
        kwargs.setdefault("adversarial_loss_factor", 0.005)
        super().__init__(*args, **kwargs)
        self.perceptual_criterion = PerceptualLoss()
        self.pixel_level_criterion = L1Loss()

    def _real_fake(self, size: int) -> Tuple[Tensor, Tensor]:
        dev = next(self.generator.parameters()).device
        return torch.ones((size, 1), device=dev), torch.zeros((size, 1), device=dev)

    def loss_g(self, hr: Tensor, sr: Tensor, real_labels: Tensor = None, fake_labels: Tensor = None):
        """pl_gan.py:28-49 (labels implied: BCE(fr, 1), BCE(rf, 0))."""
        score_real = self.discriminator(hr)
        score_fake = self.discriminator(sr)
        adversarial_loss = relativistic_adversarial_loss(score_real, score_fake, generator_step=True)
        perceptual_loss = self.perceptual_criterion(hr, sr)
        pixel_level_loss = self.pixel_level_criterion(sr, hr)
        hp = self.hparams
        loss_g = (hp.pixel_level_loss_factor * pixel_level_loss + hp.perceptual_loss_factor * perceptual_loss
                  + hp.adversarial_loss_factor * adversarial_loss)
        return perceptual_loss, adversarial_loss, pixel_level_loss, loss_g

    def loss_d(self, hr: Tensor, sr: Tensor, real_labels: Tensor = None, fake_labels: Tensor = None):
        """pl_gan.py:51-61 (labels implied: BCE(fr, 0), BCE(rf, 1))."""
        score_real = self.discriminator(hr)
        score_fake = self.discriminator(sr.detach())
        return relativistic_adversarial_loss(score_real, score_fake, generator_step=False)

    def training_step(self, batch: Any, batch_idx: int, optimizer_idx: int) -> Dict[str, Any]:
        hr, sr = self.common_step(batch)
        if optimizer_idx == 0:
            perceptual_loss, adversarial_loss, pixel_level_loss, loss_g = self.loss_g(hr, sr)
            log_dict = {"train/perceptual_loss": perceptual_loss, "train/adversarial_loss": adversarial_loss,
                        "train/pixel_level_loss": pixel_level_loss, "train/loss_G": loss_g}
            self.log_dict(log_dict, prog_bar=True, on_step=True, on_epoch=False)
            return {"loss": loss_g, "log": log_dict}
        if optimizer_idx == 1:
            loss_d = self.loss_d(hr, sr)
            self.log("train/loss_D", loss_d, prog_bar=True, on_step=True, on_epoch=False)
            return {"loss": loss_d, "log": {"train/loss_D": loss_d}}

    def validation_step(self, batch: Any, batch_idx: int, dataloader_idx: Optional[int] = None) -> Dict[str, Any]:
        """pl_gan.py:99-130: metrics, then loss_g on the (mask-zeroed) hr and the unmasked sr."""
        hr = batch["hr"]
        metric_dict = self.common_val_test_step(batch)
        with torch.no_grad():
            perceptual_loss, adversarial_loss, _, loss_g = self.loss_g(hr, metric_dict["sr"])
        metric_dict.pop("sr", None)
        metric_dict.update({"val/perceptual_loss": perceptual_loss, "val/adversarial_loss": adversarial_loss,
                            "val/loss_G": loss_g})
        self.log_dict(metric_dict, on_step=False, on_epoch=True)
        return metric_dict
