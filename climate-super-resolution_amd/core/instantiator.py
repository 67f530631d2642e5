"""Minimal ``_target_`` instantiation (the reference's HydraInstantiator, climsr/core/instantiator.py:37-82).

Uses ``hydra.utils.instantiate`` when Hydra is importable; otherwise resolves ``_target_`` dotted
paths itself (dicts/OmegaConf-like mappings with ``_target_`` and kwargs), which is all the hot-path
configs (conf/generator/*.yaml, conf/discriminator/*.yaml, conf/optimizers/adamw.yaml,
conf/schedulers/one_cycle_schedule.yaml) need.
"""
from __future__ import annotations

import importlib
from typing import Any, Mapping

import torch


def _locate(path: str):
    mod, _, name = path.rpartition(".")
    return getattr(importlib.import_module(mod), name)


def instantiate(cfg: Any, *args, **kwargs):
    if cfg is None:
        return None
    if isinstance(cfg, torch.nn.Module):
        return cfg
    try:  # pragma: no cover - hydra is not installed in the build image
        import hydra  # noqa: F401

        return hydra.utils.instantiate(cfg, *args, **kwargs)
    except ImportError:
        pass
    if not isinstance(cfg, Mapping) or "_target_" not in cfg:
        raise TypeError(f"cannot instantiate {cfg!r}: expected a mapping with _target_")
    params = {k: v for k, v in dict(cfg).items() if not k.startswith("_")}
    params.update(kwargs)
    return _locate(cfg["_target_"])(*args, **params)


class HydraInstantiator:
    """Same methods as the reference's HydraInstantiator (instantiator.py:37-82)."""

    def model(self, cfg, model_data_kwargs=None):
        return self.instantiate(cfg, instantiator=self, **(model_data_kwargs or {}))

    def optimizer(self, model: torch.nn.Module, cfg):
        return self.instantiate(cfg, model.parameters())

    def scheduler(self, cfg, optimizer):
        cfg = dict(cfg)
        if cfg.get("_target_", "").startswith("torch.optim"):
            if cfg.get("_target_").endswith("OneCycleLR"):
                cfg["total_steps"] = cfg.get("num_training_steps")
            cfg.pop("num_training_steps", None)
            cfg.pop("num_warmup_steps", None)
        return self.instantiate(cfg, optimizer=optimizer)

    def instantiate(self, *args, **kwargs):
        return instantiate(*args, **kwargs)
