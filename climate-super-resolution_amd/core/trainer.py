"""Built-in trainer loop with Lightning-1.x automatic-optimisation semantics (used when
pytorch_lightning is absent, and by bench.py).  Per batch and per optimizer i:
toggle (only optimizer i's params require grad), zero_grad, training_step(batch, idx[, i]),
backward, optimizer i step; then every scheduler steps (interval "step", task.py:58-59).

It carries the ``pytorch_lightning.Trainer`` attributes the task's ``num_training_steps`` reads
(task.py:61-83: limit_train_batches, datamodule, max_epochs, max_steps, accumulate_grad_batches,
num_gpus / num_processes) and calls the zero-argument ``configure_optimizers()`` hook.  The one extension is
``num_training_steps=N``: a run of exactly N batches (limit_train_batches=N, max_epochs=1).
"""
from __future__ import annotations

from typing import Any, Dict, Iterable, List, Optional


class Trainer:
    def __init__(self, module, num_training_steps: Optional[int] = None, max_epochs: int = 1, max_steps: Optional[int] = None,
                 limit_train_batches=1.0, accumulate_grad_batches: int = 1, datamodule=None, num_gpus: int = 0,
                 num_processes: int = 1):
        if num_training_steps is not None:
            limit_train_batches, max_epochs = int(num_training_steps), 1
        self.module = module
        self.max_epochs, self.max_steps = max_epochs, max_steps
        self.limit_train_batches, self.accumulate_grad_batches = limit_train_batches, accumulate_grad_batches
        self.datamodule, self.num_gpus, self.num_processes, self.tpu_cores = datamodule, num_gpus, num_processes, None
        module.trainer = self
        self.optimizers, self.schedulers = module.configure_optimizers()
        self.nets = [module.generator] + ([module.discriminator] if module.discriminator is not None else [])

    def _toggle(self, i: int) -> None:
        for j, net in enumerate(self.nets):
            for p in net.parameters():
                p.requires_grad_(j == i)

    def training_batch(self, batch: Dict[str, Any], batch_idx: int) -> List[Any]:
        outs = []
        nopt = len(self.optimizers)
        for i, opt in enumerate(self.optimizers):
            if nopt > 1:
                self._toggle(i)
            opt.zero_grad(set_to_none=True)
            out = self.module.training_step(batch, batch_idx, i) if nopt > 1 else self.module.training_step(batch, batch_idx)
            loss = out["loss"] if isinstance(out, dict) else out
            loss.backward()
            opt.step()
            outs.append(out)
        if nopt > 1:
            for net in self.nets:
                for p in net.parameters():
                    p.requires_grad_(True)
        for s in self.schedulers:
            s["scheduler"].step()
        return outs

    def fit(self, batches: Iterable[Dict[str, Any]]):
        outs = []
        for idx, b in enumerate(batches):
            outs.append(self.training_batch(b, idx))
        return outs
