"""SRCNN tail of the ESRGAN generator (``climsr/models/srcnn.py:6-18``).

Inside ``ESRGANGenerator`` the three convs run natively (fused ReLUs, the ``torch.cat`` of
esrgan.py:100 is a channel-packed NHWC buffer).  The stand-alone SRCNN generator (MSE task,
``task.py:141``) is outside this build's scope; this class keeps the reference's
parameter names so ``srcnn.conv{1,2,3}`` state_dict keys match.
"""
import torch.nn as nn


class SRCNN(nn.Module):
    def __init__(self, in_channels=1, out_channels=1, **kwargs):
        super().__init__()
        self.conv1 = nn.Conv2d(in_channels=in_channels, out_channels=64, kernel_size=9, padding=4)
        self.conv2 = nn.Conv2d(in_channels=64, out_channels=32, kernel_size=1, padding=0)
        self.conv3 = nn.Conv2d(in_channels=32, out_channels=out_channels, kernel_size=5, padding=2)

    def forward(self, x):  # pragma: no cover
        raise RuntimeError("SRCNN runs natively only as the ESRGANGenerator tail in this build")
