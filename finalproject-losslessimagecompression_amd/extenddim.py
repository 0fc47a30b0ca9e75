"""Space-to-depth squeeze (mirror of extenddim.py:17-37).  A pure index map:
on the model path it runs as idf_squeeze / idf_unsqueeze on pixel-major
buffers.  Patching (extenddim.py:40-67), the residual configs' image <-> patch
batch map, runs as idf_patch."""
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


@moduleregister.Register.register
class Patching(InvertibleModule):
    """extenddim.py:40-67: [B, C, H, W] <-> [B*(H/h)*(W/w), C, h, w] (patches row-major)."""

    def __init__(self, H, W, h, w):
        assert H % h == 0 and W % w == 0
        super().__init__()
        self.H, self.W, self.h, self.w = H, W, h, w

    def _run(self, x, inverse, out_shape):
        from idfcodec import _lib
        from idfcodec._lib import check, lib, ptr
        require_device(x, "Patching input")
        x = x.float().contiguous()
        out = torch.empty(out_shape, dtype=torch.float32, device=x.device)
        B = out_shape[0] if inverse else x.shape[0]
        C = x.shape[1]
        check(lib().idf_patch(_lib.stream_ptr(x.device), B, C, self.H, self.W, self.h, self.w,
                              int(inverse), ptr(x), ptr(out)), "patch")
        return out

    def forward(self, x, logv):
        B, C = x.shape[0], x.shape[1]
        n = (self.H // self.h) * (self.W // self.w)
        return self._run(x, False, (B * n, C, self.h, self.w)), logv

    def backward(self, x):
        n = (self.H // self.h) * (self.W // self.w)
        return self._run(x, True, (x.shape[0] // n, x.shape[1], self.H, self.W))
