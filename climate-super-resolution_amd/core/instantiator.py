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
        """instantiator.py:48-49.  For a native (flat-parameter) network ``torch.optim.AdamW`` resolves to the fused
        ``climsr_amd.core.optim.AdamW`` (same hyper-parameters and param_groups, so OneCycleLR drives it unchanged);
        any other optimizer is instantiated as configured and re-packs the network's bf16 MFMA weights after each
        step (the kernels read those, not the fp32 masters)."""
        cfg = dict(cfg)
        native = hasattr(model, "_flat") and hasattr(model, "repack_weights")
        if native and cfg.get("_target_") in ("torch.optim.AdamW", "climsr_amd.core.optim.AdamW"):
            from .optim import AdamW

            params = {k: v for k, v in cfg.items() if not k.startswith("_")}
            unsupported = dict(AdamW._UNSUPPORTED, amsgrad=False)
            odd = {k: v for k, v in params.items() if k in unsupported and v != unsupported[k]}
            if not odd:
                return AdamW(model.parameters(), owner=model, **params)
            # options the fused update does not implement (amsgrad, maximize, foreach, ...): torch's own AdamW + repack
            opt = torch.optim.AdamW(model.parameters(), **params)
        else:
            opt = self.instantiate(cfg, model.parameters())
        if native:
            step = opt.step

            def step_and_repack(*a, **kw):
                out = step(*a, **kw)
                model.repack_weights()
                return out

            opt.step = step_and_repack
        return opt

    def scheduler(self, cfg, optimizer):
        """instantiator.py:51-64: torch.optim schedulers get OneCycleLR's total_steps from num_training_steps and lose
        the two step keys; only torch.optim and transformers schedulers are accepted."""
        cfg = dict(cfg)
        target = cfg.get("_target_", "")
        if target.startswith("torch.optim"):
            if target.endswith("OneCycleLR"):
                cfg["total_steps"] = cfg.get("num_training_steps")
            cfg.pop("num_training_steps")
            cfg.pop("num_warmup_steps")
        elif not target.startswith("transformers"):
            raise ValueError("Only LR schedulers from `torch.optim` and `transformers` library are supported. "
                             f"If you want to support {target}, you must add your own instantiation logic here.")
        return self.instantiate(cfg, optimizer=optimizer)

    def instantiate(self, *args, **kwargs):
        return instantiate(*args, **kwargs)
