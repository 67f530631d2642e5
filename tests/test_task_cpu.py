"""CPU tests of the task's Lightning hooks: the zero-argument ``configure_optimizers()`` (reference
climsr/core/task.py:173-226 + LitSuperResolutionModule.num_training_steps / compute_warmup, task.py:53-92) and
``HydraInstantiator.optimizer / scheduler`` (instantiator.py:48-64), driven by the reference's own config contents:
conf/optimizers/adamw.yaml and conf/schedulers/one_cycle_schedule.yaml (``${training.lr}`` = 1e-4 from
conf/training/default.yaml, ``${trainer.max_epochs}`` resolved per case)."""
from types import SimpleNamespace

import pytest
import torch

ADAMW_YAML = {"_target_": "torch.optim.AdamW", "lr": 1e-4, "weight_decay": 1e-4}
ONE_CYCLE_YAML = {"_target_": "torch.optim.lr_scheduler.OneCycleLR", "max_lr": 1e-4, "num_training_steps": -1, "epochs": 1,
                  "pct_start": 0.05, "div_factor": 2, "final_div_factor": 100}


class _DM:
    def __init__(self, n):
        self.n = n

    def train_dataloader(self):
        return range(self.n)


def _trainer(**kw):
    base = dict(limit_train_batches=1.0, datamodule=_DM(40), max_epochs=3, max_steps=None, accumulate_grad_batches=2,
                num_gpus=0, num_processes=1, tpu_cores=None)
    base.update(kw)
    return SimpleNamespace(**base)


def _gan(sched_steps=-1):
    from climsr_amd.task.pl_gan import GANLightningModule

    sch = dict(ONE_CYCLE_YAML, num_training_steps=sched_steps)
    return GANLightningModule(
        generator={"_target_": "climsr_amd.models.esrgan.ESRGANGenerator", "in_channels": 3, "out_channels": 1, "nf": 64, "nb": 1,
                   "gc": 16, "scaling_factor": 4},
        discriminator={"_target_": "climsr_amd.models.rfb_esrgan.RFBESRGANDiscriminator", "in_channels": 1},
        optimizers={"generator_optimizer": dict(ADAMW_YAML), "discriminator_optimizer": dict(ADAMW_YAML)},
        schedulers={"generator_scheduler": dict(sch), "discriminator_scheduler": dict(sch)})


def test_configure_optimizers_infers_steps_from_trainer():
    from climsr_amd.core.optim import AdamW

    m = _gan()
    m.trainer = _trainer()
    opts, scheds = m.configure_optimizers()
    assert len(opts) == 2 and len(scheds) == 2
    assert all(isinstance(o, AdamW) for o in opts)  # torch.optim.AdamW -> the fused native AdamW for flat-param nets
    assert opts[0].owner is m.generator and opts[1].owner is m.discriminator
    # (40 batches // (accumulate 2 * 1 device)) * 3 epochs = 60 (task.py:61-83)
    assert m.inferred_training_steps == 60
    for s, o in zip(scheds, opts):
        assert s["interval"] == "step"
        sch = s["scheduler"]
        assert isinstance(sch, torch.optim.lr_scheduler.OneCycleLR) and sch.total_steps == 60
        g = o.param_groups[0]
        assert g["lr"] == pytest.approx(1e-4 / 2) and g["betas"][0] == pytest.approx(0.95)  # OneCycle start, beta1 cycled
        assert g["weight_decay"] == pytest.approx(1e-4)


@pytest.mark.parametrize("kw,want", [(dict(max_steps=50), 50), (dict(max_steps=500), 60), (dict(limit_train_batches=7), 9),
                                     (dict(limit_train_batches=0.5), 30), (dict(num_gpus=2), 30)])
def test_num_training_steps_rules(kw, want):
    m = _gan()
    m.trainer = _trainer(**kw)
    assert m.num_training_steps == want


def test_scheduler_cfg_steps_win_over_trainer():
    m = _gan(sched_steps=123)
    m.trainer = _trainer()
    _opts, scheds = m.configure_optimizers()
    assert all(s["scheduler"].total_steps == 123 for s in scheds)


def test_no_trainer_and_no_steps_raises():
    m = _gan()
    with pytest.raises(RuntimeError):
        m.configure_optimizers()


def test_builtin_trainer_explicit_steps_and_pretrain_defaults():
    """conf/task/generator_pre_training.yaml: no optimizer / scheduler cfgs -> adamw.yaml + one_cycle_schedule.yaml
    defaults; the built-in Trainer's num_training_steps=N is a run of N batches."""
    from climsr_amd.core.trainer import Trainer
    from climsr_amd.task.pl_generator_pre_training import GeneratorPreTrainingLightningModule

    m = GeneratorPreTrainingLightningModule(generator={"_target_": "climsr_amd.models.esrgan.ESRGANGenerator", "nb": 1})
    tr = Trainer(m, num_training_steps=17)
    assert m.trainer is tr and len(tr.optimizers) == 1
    assert tr.schedulers[0]["scheduler"].total_steps == 17


def test_non_adamw_optimizer_repacks_after_step():
    """Any other torch optimizer on a native net still refreshes the bf16 MFMA weights after its step."""
    from climsr_amd.core.instantiator import HydraInstantiator

    calls = []

    class Net(torch.nn.Module):
        def __init__(self):
            super().__init__()
            self.w = torch.nn.Parameter(torch.ones(3))
            self._flat = self.w

        def repack_weights(self):
            calls.append(1)

    net = Net()
    opt = HydraInstantiator().optimizer(net, {"_target_": "torch.optim.SGD", "lr": 0.1})
    net.w.grad = torch.ones(3)
    opt.step()
    assert calls == [1] and torch.allclose(net.w.detach(), torch.full((3,), 0.9))


def test_scheduler_rejects_other_libraries():
    from climsr_amd.core.instantiator import HydraInstantiator

    opt = torch.optim.SGD([torch.nn.Parameter(torch.ones(1))], lr=0.1)
    with pytest.raises(ValueError):
        HydraInstantiator().scheduler({"_target_": "mylib.Sched", "num_training_steps": 1, "num_warmup_steps": 0}, opt)


def test_builtin_trainer_without_steps_or_datamodule_explains():
    """Trainer(module) with neither num_training_steps, a datamodule nor an int limit_train_batches: a clear error
    naming the missing configuration (not an AttributeError on None)."""
    from climsr_amd.core.trainer import Trainer

    with pytest.raises(ValueError, match="num_training_steps"):
        Trainer(_gan())


def test_adamw_rejects_options_it_does_not_implement():
    from climsr_amd.core.instantiator import HydraInstantiator
    from climsr_amd.core.optim import AdamW
    from climsr_amd.models.esrgan import ESRGANGenerator

    g = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=1, gc=16)
    with pytest.raises(ValueError, match="maximize"):
        AdamW(g.parameters(), lr=1e-4, maximize=True)
    with pytest.raises(TypeError, match="bogus"):
        AdamW(g.parameters(), lr=1e-4, bogus=1)
    assert isinstance(AdamW(g.parameters(), lr=1e-4, maximize=False, foreach=None), AdamW)  # defaults are fine
    # through the instantiator a torch.optim.AdamW cfg with such an option falls back to torch's AdamW (+ repack)
    opt = HydraInstantiator().optimizer(g, dict(ADAMW_YAML, maximize=True))
    assert type(opt) is torch.optim.AdamW and opt.param_groups[0]["maximize"] is True
    assert isinstance(HydraInstantiator().optimizer(g, dict(ADAMW_YAML)), AdamW)
    # amsgrad too, also when _target_ names the fused class itself
    for target in ("torch.optim.AdamW", "climsr_amd.core.optim.AdamW"):
        opt = HydraInstantiator().optimizer(g, dict(ADAMW_YAML, _target_=target, amsgrad=True))
        assert type(opt) is torch.optim.AdamW and opt.param_groups[0]["amsgrad"] is True


def test_autograd_grad_route_refuses_a_flat_reducer_hook():
    from climsr_amd.models.esrgan import ESRGANGenerator

    g = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=2, gc=16)
    g._begin_autograd_grads()  # no hook: fine
    g.set_grad_ready_hook(lambda lo: None)
    with pytest.raises(RuntimeError, match="grad-ready hook"):
        g._begin_autograd_grads()
