"""Generator pre-training task (mirror of climsr/task/pl_generator_pre_training.py:10-33).

``GeneratorPreTrainingLightningModule`` is provided as an alias: conf/task/generator_pre_training.yaml:4
targets that name, which the reference never defines, so with climsr_amd the shipped config
instantiates.
"""
from typing import Any

from ..core.task import TaskSuperResolutionModule


class SuperResolutionLightningModule(TaskSuperResolutionModule):
    def training_step(self, batch: Any, batch_idx: int) -> Any:
        hr, sr = self.common_step(batch)
        loss = self.loss(sr, hr)
        self.log("train/loss", loss, on_step=True, on_epoch=False)
        return loss


GeneratorPreTrainingLightningModule = SuperResolutionLightningModule
