"""climsr_amd — MI355X-native (gfx950) hot path for xultaeculcis/climate-super-resolution.

Drop-in modules for the reference's Hydra ``_target_`` surface:
``climsr_amd.models.esrgan.ESRGANGenerator``, ``climsr_amd.models.rfb_esrgan.RFBESRGANDiscriminator``,
``climsr_amd.models.discriminator.Discriminator``, ``climsr_amd.losses.perceptual.PerceptualLoss``,
``climsr_amd.task.pl_gan.GANLightningModule``, ``climsr_amd.task.pl_generator_pre_training.*``.
All device arithmetic runs in hand-written HIP kernels in ``csrc/`` (``libclimsr_hip.so``).
"""
__version__ = "0.1.0"
