"""Space-to-depth squeeze (mirror of extenddim.py:17-37).  A pure index map:
on the model path it runs as idf_squeeze / idf_unsqueeze on pixel-major
buffers.  Patching (extenddim.py:40-67) serves configs 4-5."""
import torch

import moduleregister
from invertible import InvertibleModule
from idfcodec._lib import require_device


class NNExtendDim(moduleregister.Register):
    def __init__(self):
        super().__init__()


@NNExtendDim.register
class ExtendDim(InvertibleModule):
    def __init__(self, scale=2):
        super().__init__()
        self.scale = scale

    def forward(self, x, logv):
        require_device(x, "ExtendDim input")
        B, C, H, W = x.shape
        s = self.scale
        x = x.view(B, C, H // s, s, W // s, s).permute(0, 1, 3, 5, 2, 4).contiguous()
        return x.view(B, C * s * s, H // s, W // s), logv

    def backward(self, x):
        require_device(x, "ExtendDim input")
        B, C, H, W = x.shape
        s = self.scale
        x = x.view(B, C // s // s, s, s, H, W).permute(0, 1, 4, 2, 5, 3).contiguous()
        return x.view(B, C // s // s, H * s, W * s)
