"""Rounding to the 2^-nbits grid (mirror of roundlib.py:18-38).

On the hot path the rounding is fused into the coupling head epilogue of the
HIP GEMM (flow_kernels.hip round8, rint = torch.round ties-to-even).  The
module form below serves API users; it requires device tensors like every
product op.  VectorQuantizer (roundlib.py:41-89) keeps the reference's codebook
(nn.Embedding, uniform(-1, 1) init) and buffers; its nearest-code search runs as
the fused MFMA argmin kernel idf_vq_argmin (csrc/vq_kernels.hip).
"""
import torch
from torch import nn

import moduleregister
from idfcodec._lib import require_device


class NNRound(moduleregister.Register):
    def __init__(self):
        super().__init__()


class BaseRound(nn.Module):
    """straight-through round: forward value rint(x)"""

    def forward(self, x):
        require_device(x, "Round input")
        y = torch.round(x)
        return x + (y - x).detach()


@NNRound.register
class Round(nn.Module):
    def __init__(self, nbits=None):
        super().__init__()
        self.nbits = nbits
        self.round = BaseRound()

    def forward(self, x, nbits=None):
        bins = 2 ** (nbits or self.nbits or 8)
        return self.round(x * bins) / bins


@NNRound.register
class VectorQuantizer(nn.Module):
    """roundlib.py:41-89.  forward(x [N, D]) -> embed[argmin_k |x - e_k|^2] (value; the
    straight-through form and the training-time codebook re-init are training-only)."""

    def __init__(self, num=4096, dim=512, init="normal", reinit_interval=None, threshold=None):
        super().__init__()
        self.num = num
        self.dim = dim
        self.embed = nn.Embedding(num, dim, padding_idx=0)
        if init == "normal":
            nn.init.uniform_(self.embed.weight.data, -1.0, 1.0)
        else:
            raise Exception(f"Unknown initialization method {init}")
        self.register_buffer("count", torch.zeros(num))
        self.register_buffer("iter_count", torch.zeros(()))
        self.reinit_interval = reinit_interval
        self.threshold = min(threshold, 1.0) if threshold else 0.1

    def indices(self, x):
        """argmin indices of rows x [N, D] (device), int32."""
        from idfcodec import _lib
        from idfcodec._lib import check, lib, ptr
        require_device(x, "VectorQuantizer input")
        x = x.float().contiguous()
        e = self.embed.weight.detach().float().contiguous()
        s = _lib.stream_ptr(x.device)
        en = torch.empty(self.num, dtype=torch.float32, device=x.device)
        check(lib().idf_vq_norms(s, self.num, self.dim, ptr(e), self.dim, ptr(en)), "vq norms")
        idx = torch.empty(x.shape[0], dtype=torch.int32, device=x.device)
        nws = int(lib().idf_vq_argmin_workspace_bytes(x.shape[0], self.num))
        ws = torch.empty(max(nws, 1), dtype=torch.uint8, device=x.device)
        check(lib().idf_vq_argmin_ws(s, x.shape[0], self.dim, ptr(x), self.dim, ptr(e), self.dim,
                                     self.num, ptr(en), ptr(idx), ptr(ws), nws), "vq argmin")
        return idx

    def forward(self, x, beta=0.25, gamma=1.0, require_loss=True):
        idx = self.indices(x)
        vq_x = self.embed.weight.detach()[idx.long()]
        if require_loss:
            loss = torch.mean((x - vq_x) ** 2) * (beta + gamma)
            return vq_x, loss
        return vq_x
