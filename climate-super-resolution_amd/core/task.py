"""Task base (mirror of ``climsr.core.task.TaskSuperResolutionModule``, task.py:109-260).

Keeps the reference's step API: ``forward(x, elevation, mask)`` (task.py:235-239),
``common_step(batch) -> (hr, sr)`` (task.py:241-260) with batch keys ``lr, hr, elevation, mask``
(climsr/consts/batch_items.py:2-5), and ``configure_optimizers`` returning one AdamW +
OneCycleLR(interval="step") per network (task.py:173-226, 53-59).  Subclasses a
``pytorch_lightning.LightningModule`` when Lightning is importable, otherwise a plain
``nn.Module`` with the few Lightning attributes the step uses (``hparams``, ``log``, ``log_dict``),
driven by ``climsr_amd.core.trainer.Trainer``.

Divergences (documented in DESIGN.md): the statistics feather read of task.py:146-171 is skipped
when ``data_path`` has no statistics (synthetic benchmarking); the stand-alone SRCNN
generator with MSE loss (task.py:141) is outside this build's scope.
"""
from __future__ import annotations

from types import SimpleNamespace
from typing import Any, Dict, List, Optional, Tuple

import torch
from torch import Tensor

from ..losses.l1 import L1Loss
from ..metrics.sr_metrics import SRMetrics
from .checkpoint import load_from_checkpoint as _load_from_checkpoint
from .checkpoint import save_checkpoint as _save_checkpoint
from .instantiator import HydraInstantiator

try:  # pragma: no cover - not installed in the build image
    import pytorch_lightning as pl

    _Base = pl.LightningModule
except ImportError:  # the built-in trainer drives the same API
    _Base = torch.nn.Module

BATCH_KEYS = ("lr", "hr", "elevation", "mask")


def _cfg_dict(cfg):
    """A Hydra/OmegaConf node or mapping as a plain dict (None stays None)."""
    if cfg is None:
        return None
    try:  # pragma: no cover - omegaconf is not installed in the build image
        from omegaconf import OmegaConf

        if OmegaConf.is_config(cfg):
            return OmegaConf.to_container(cfg, resolve=True)
    except ImportError:
        pass
    return dict(cfg)
default_instantiator = HydraInstantiator()


class TaskSuperResolutionModule(_Base):
    def __init__(self, generator, optimizers: Optional[Dict[str, Any]] = None, schedulers: Optional[Dict[str, Any]] = None,
                 discriminator=None, instantiator=default_instantiator, **kwargs):
        super().__init__()
        self._init_cfgs = dict(generator=generator, discriminator=discriminator, optimizers=optimizers, schedulers=schedulers)
        self.instantiator = instantiator
        self.optimizer_cfgs = optimizers or {}
        self.scheduler_cfgs = schedulers or {}
        self.generator = instantiator.instantiate(generator)
        self.discriminator = instantiator.instantiate(discriminator) if discriminator is not None else None
        hp = dict(generator_type="esrgan")
        hp.update(kwargs)
        if _Base is torch.nn.Module:
            self.hparams = SimpleNamespace(**hp)
        else:  # pragma: no cover
            self.save_hyperparameters(*kwargs.keys())
        if getattr(self.hparams, "generator_type", "esrgan") == "srcnn":
            raise NotImplementedError("stand-alone SRCNN + MSE task is outside this build's scope (SURVEY §2)")
        self.loss = L1Loss()  # task.py:141
        self.logged: Dict[str, Tensor] = {}
        zs = dict(getattr(self.hparams, "standardization_stats", None) or {})
        self.metrics = SRMetrics(normalization_method=getattr(self.hparams, "normalization_method", "minmax"),
                                 normalization_range=tuple(getattr(self.hparams, "normalization_range", (-1.0, 1.0))),
                                 zscore_mean=zs.get("mean", 0.0), zscore_std=zs.get("std", 1.0))

    # -- Lightning-compat helpers (no host sync: values are kept as device tensors)
    if _Base is torch.nn.Module:
        def log(self, name, value, **kwargs):
            self.logged[name] = value.detach() if isinstance(value, Tensor) else value

        def log_dict(self, d, **kwargs):
            for k, v in d.items():
                self.log(k, v)

    def forward(self, x: Tensor, elevation: Tensor = None, mask: Tensor = None) -> Tensor:
        return self.generator(x, elevation, mask)

    def common_step(self, batch: Dict[str, Tensor]) -> Tuple[Tensor, Tensor]:
        lr, hr, elev, mask = (batch[k] for k in BATCH_KEYS)
        sr = self(lr, elev, mask)
        return hr, sr

    # -- optimisers / schedulers (task.py:173-226 + LitSuperResolutionModule.configure_optimizers / num_training_steps /
    #    compute_warmup, task.py:53-92)
    DEFAULT_OPTIMIZER = {"_target_": "torch.optim.AdamW", "lr": 1e-4, "weight_decay": 1e-4}          # conf/optimizers/adamw.yaml
    DEFAULT_SCHEDULER = {"_target_": "torch.optim.lr_scheduler.OneCycleLR", "max_lr": 1e-4,           # one_cycle_schedule.yaml
                         "num_training_steps": -1, "pct_start": 0.05, "div_factor": 2, "final_div_factor": 100}

    @property
    def num_training_steps(self) -> int:
        """Total training steps inferred from the trainer and its datamodule (task.py:61-83)."""
        t = getattr(self, "trainer", None)
        if t is None:
            raise RuntimeError("num_training_steps: no trainer attached; set the scheduler cfg's num_training_steps")
        ltb = t.limit_train_batches
        if isinstance(ltb, int) and ltb != 0:
            dataset_size = ltb
        else:
            if getattr(t, "datamodule", None) is None:
                raise ValueError("cannot infer the number of training steps: the trainer has no datamodule and "
                                 f"limit_train_batches={ltb!r} is not a batch count; pass Trainer(num_training_steps=N), "
                                 "Trainer(datamodule=...), an int limit_train_batches, or set the scheduler cfg's "
                                 "num_training_steps")
            n_batches = len(t.datamodule.train_dataloader())
            dataset_size = int(n_batches * ltb) if isinstance(ltb, float) else n_batches  # float: a fraction
        num_devices = max(1, getattr(t, "num_gpus", 0) or 0, getattr(t, "num_processes", 0) or 0)
        if getattr(t, "tpu_cores", None):
            num_devices = max(num_devices, t.tpu_cores)
        effective_batch_size = t.accumulate_grad_batches * num_devices
        max_estimated_steps = (dataset_size // effective_batch_size) * t.max_epochs
        if t.max_steps and -1 < t.max_steps < max_estimated_steps:
            return t.max_steps
        return max_estimated_steps

    def compute_warmup(self, num_training_steps: int, num_warmup_steps):
        """task.py:85-92: < 0 = infer from the trainer; a float < 1 warm-up is a fraction of the steps."""
        if num_training_steps < 0:
            num_training_steps = self.num_training_steps
        if isinstance(num_warmup_steps, float) and num_warmup_steps < 1.0:
            num_warmup_steps *= num_training_steps
        return num_training_steps, num_warmup_steps

    def configure_optimizers(self):
        """The Lightning hook (task.py:173-226): infer the step count from the generator scheduler cfg's
        ``num_training_steps`` (-1 = from the trainer / datamodule), write it and the warm-up into every scheduler
        cfg, then build one optimizer + scheduler per network through the instantiator
        (``HydraInstantiator.optimizer`` / ``.scheduler``, instantiator.py:48-64); schedulers step per batch.
        Missing cfgs default to conf/optimizers/adamw.yaml + conf/schedulers/one_cycle_schedule.yaml (the
        reference has no default and would fail)."""
        if self.instantiator is None:
            raise RuntimeError("To train you must provide an instantiator to instantiate the optimizer and scheduler "
                               "or override `configure_optimizers` in the `LightningModule`.")
        nets = [("generator", self.generator)]
        if self.discriminator is not None:
            nets.append(("discriminator", self.discriminator))
        ocfgs = {n: _cfg_dict(self.optimizer_cfgs.get(f"{n}_optimizer")) for n, _ in nets}
        scfgs = {n: _cfg_dict(self.scheduler_cfgs.get(f"{n}_scheduler")) for n, _ in nets}
        for n, _ in nets:
            if ocfgs[n] is None:
                ocfgs[n] = dict(self.DEFAULT_OPTIMIZER)
            if scfgs[n] is None:
                scfgs[n] = dict(self.DEFAULT_SCHEDULER, max_lr=ocfgs[n].get("lr", 1e-4))
        g = scfgs["generator"]
        num_training_steps, num_warmup_steps = self.compute_warmup(num_training_steps=g.get("num_training_steps", -1),
                                                                   num_warmup_steps=g.get("num_warmup_steps", None))
        for n, _ in nets:
            scfgs[n]["num_training_steps"] = num_training_steps
            scfgs[n]["num_warmup_steps"] = num_warmup_steps
        self.inferred_training_steps = num_training_steps
        self._optimizers, self._schedulers = [], []
        for n, net in nets:
            opt = self.instantiator.optimizer(net, ocfgs[n])
            self._optimizers.append(opt)
            self._schedulers.append(self.instantiator.scheduler(scfgs[n], opt))
        return self._optimizers, [{"scheduler": s, "interval": "step"} for s in self._schedulers]

    # -- validation / test (task.py:262-294, 336-391): metrics fused on device (climsr_amd.metrics)
    def common_val_test_step(self, batch: Any, prefix: str = "val") -> Dict[str, Tensor]:
        original, mask = batch["original_data"], batch["mask"]
        hr, sr = self.common_step(batch)
        sr_copy = sr.detach().clone()
        metric_dict = self.metrics(sr.detach(), hr, original, mask, batch.get("min"), batch.get("max"), prefix=prefix)
        land = mask.bool()
        hr.masked_fill_(~land, 0.0)  # the reference masks the batch's hr in place (task.py:289-290)
        original.masked_fill_(~land, 0.0)
        metric_dict["sr"] = sr_copy
        return metric_dict

    def validation_step(self, batch: Any, batch_idx: int, dataloader_idx: Optional[int] = None) -> Dict[str, Tensor]:
        """pl_generator_pre_training.py:35-50."""
        metric_dict = self.common_val_test_step(batch, prefix="val")
        metric_dict.pop("sr", None)
        self.log_dict(metric_dict, prog_bar=False, on_step=False, on_epoch=True)
        return metric_dict

    def test_step(self, batch: Any, batch_idx: int, dataloader_idx: Optional[int] = None) -> Dict[str, Tensor]:
        """pl_generator_pre_training.py:52-64."""
        return self.common_val_test_step(batch, prefix="test")

    def validation_epoch_end(self, outputs: List[Any]) -> None:
        """hp_metric = mean of the epoch's val/rmse (task.py:387-391)."""
        hp_metric = torch.stack([o["val/rmse"] for o in outputs]).mean()
        self.log("hp_metric", hp_metric)

    # -- checkpoints (Lightning layout; climsr_amd.core.checkpoint)
    def hyper_parameters(self) -> Dict[str, Any]:
        hp = dict(vars(self.hparams)) if hasattr(self.hparams, "__dict__") else dict(self.hparams)
        for k, v in self._init_cfgs.items():
            if isinstance(v, dict):  # Hydra configs (plain dicts); instantiated modules are not re-creatable
                hp[k] = v
        return hp

    def save_checkpoint(self, path: str, epoch: int = 0, global_step: int = 0, optimizers=(), schedulers=()):
        return _save_checkpoint(self, path, epoch, global_step, optimizers, schedulers, self.hyper_parameters())

    if _Base is torch.nn.Module:
        @classmethod
        def load_from_checkpoint(cls, checkpoint_path: str, strict: bool = False, trusted: bool = False, map_location="cpu",
                                 **kwargs):
            """Lightning's ``load_from_checkpoint`` (inference.py:143, cli/train.py:92,115): hyper-parameters from the
            file (overridable by kwargs), then the ``generator.`` / ``discriminator.`` weights."""
            return _load_from_checkpoint(cls, checkpoint_path, strict=strict, trusted=trusted, map_location=map_location,
                                         **kwargs)
