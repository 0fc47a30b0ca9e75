"""Rounding to the 2^-nbits grid (mirror of roundlib.py:18-38).

On the hot path the rounding is fused into the coupling head epilogue of the
HIP GEMM (flow_kernels.hip round8, rint = torch.round ties-to-even).  The
module form below serves API users; it requires device tensors like every
product op.  VectorQuantizer (roundlib.py:41-89) belongs to the VQ-VAE configs
 and is not part of this round.
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
