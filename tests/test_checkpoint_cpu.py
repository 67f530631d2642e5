"""Lightning-layout checkpoint interop, CPU: save -> load round trip through the task's
``load_from_checkpoint``, generator-only loading (the GAN fine-tuning path), a reference-layout file written by
hand, and the refusal of pickled objects under weights_only loading."""
import collections

import pytest
import torch

GEN = {"_target_": "climsr_amd.models.esrgan.ESRGANGenerator", "nb": 1, "gc": 16, "in_channels": 3, "out_channels": 1}


def make_task(seed=0):
    from climsr_amd.task.pl_generator_pre_training import SuperResolutionLightningModule

    torch.manual_seed(seed)
    return SuperResolutionLightningModule(generator=dict(GEN), pixel_level_loss_factor=1.0)


def test_round_trip_restores_weights_and_hparams(tmp_path):
    from climsr_amd.task.pl_generator_pre_training import SuperResolutionLightningModule

    t = make_task(0)
    with torch.no_grad():
        for p in t.parameters():
            p.uniform_(-1, 1)
    path = str(tmp_path / "m.ckpt")
    ck = t.save_checkpoint(path, epoch=3, global_step=120)
    assert ck["state_dict"].keys() == t.state_dict().keys() and all(k.startswith("generator.") for k in ck["state_dict"])
    u = SuperResolutionLightningModule.load_from_checkpoint(path)
    for k, v in t.state_dict().items():
        assert torch.equal(v, u.state_dict()[k]), k
    assert u.hparams.pixel_level_loss_factor == 1.0
    raw = torch.load(path, weights_only=True)
    assert raw["epoch"] == 3 and raw["global_step"] == 120 and raw["hyper_parameters"]["generator"]["nb"] == 1


def test_generator_weights_from_a_reference_layout_checkpoint(tmp_path):
    from climsr_amd.core.checkpoint import load_generator_weights
    from climsr_amd.models.esrgan import ESRGANGenerator

    src = make_task(1)
    sd = collections.OrderedDict((k, torch.randn_like(v)) for k, v in src.state_dict().items())
    sd["discriminator.features.0.weight"] = torch.zeros(64, 1, 3, 3)  # GAN checkpoints carry the D too
    ckpt = {"epoch": 29, "global_step": 2639, "pytorch-lightning_version": "1.5.10", "state_dict": sd,
            "hyper_parameters": {"generator_type": "esrgan"}}
    path = str(tmp_path / "ref.ckpt")
    torch.save(ckpt, path)
    g = ESRGANGenerator(in_channels=3, out_channels=1, nf=64, nb=1, gc=16)
    load_generator_weights(g, path)
    for k, v in g.state_dict().items():
        assert torch.equal(v, sd["generator." + k]), k


class _Opaque:  # stands for the reference's pickled Hydra instantiator (task.py:228-230)
    pass


def test_pickled_objects_are_refused_unless_trusted(tmp_path):
    from climsr_amd.core.checkpoint import load_checkpoint

    path = str(tmp_path / "p.ckpt")
    torch.save({"state_dict": {"generator.x": torch.ones(1)}, "instantiator": _Opaque()}, path)
    with pytest.raises(RuntimeError, match="weights_only"):
        load_checkpoint(path)
    assert "instantiator" in load_checkpoint(path, trusted=True)
