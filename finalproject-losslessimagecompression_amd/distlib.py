"""Discretised logistic (mirror of distlib.py:34-70).  log_prob gives the
theoretical bpd the reference logs next to the real one (flows.py:154-169);
it is not on the coding path (the coder uses the bit-exact CDF of
idfcodec/csrc/idf_cdf.h).  BinomialDistribution / UnitGaussianDistribution are
VQ-VAE training losses (distlib.py:73-101); they are registered so the residual
configs construct, and compute with torch.distributions (not a coding path)."""
import torch
from torch import nn

import moduleregister
from roundlib import NNRound, Round
from idfcodec._lib import require_device


class NNDistribution(moduleregister.Register):
    def __init__(self):
        super().__init__()


class Distribution(nn.Module):
    def __init__(self, *args, **kargs):
        super().__init__()


def dlogistic_log_prob(x, mean, logscale, nbits=8, eps=1e-8, groups=1, logp=None):
    """idf_log_prob over contiguous fp32 device tensors split into `groups` equal groups:
    fills `logp` (if given) and returns the per-group f64 sums (fixed-order reduction)."""
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    x, mean, logscale = (t.contiguous().float() for t in (x, mean, logscale))
    n = x.numel()
    if n % max(groups, 1):
        raise ValueError("log_prob groups must divide the element count")
    sums = torch.empty(groups, dtype=torch.float64, device=x.device)
    check(lib().idf_log_prob(_lib.stream_ptr(x.device), groups, n // max(groups, 1), ptr(x),
                             ptr(mean), ptr(logscale), int(nbits), float(eps),
                             ptr(logp) if logp is not None else None, ptr(sums)), "log_prob")
    return sums


@NNDistribution.register
class DLogistic(Distribution):
    def __init__(self, round=None):
        super().__init__()
        if round:
            round = dict(round)
            self.round = NNRound.get(round.pop("name"))(**round)
        else:
            self.round = Round()

    def log_prob(self, x, mean, logscale, nbits=8, eps=1e-8):
        """distlib.py:40-55 on the device (idf_log_prob): elementwise, broadcasting as the
        reference's torch ops do."""
        require_device(x, "DLogistic input")
        x, mean, logscale = torch.broadcast_tensors(x, mean, logscale)
        out = torch.empty(x.shape, dtype=torch.float32, device=x.device)
        dlogistic_log_prob(x, mean, logscale, nbits, eps, logp=out)
        return out

    def sample(self, mean, logscale, nbits=8):
        u = torch.rand_like(mean)
        s = torch.log(u / (1 - u)) * torch.exp(logscale) + mean
        return self.round(s, nbits=nbits)


@NNDistribution.register
class BinomialDistribution(nn.Module):
    """distlib.py:73-90 (VQ-VAE training loss only)."""

    def log_prob(self, x, y):
        return torch.distributions.Binomial(255, y).log_prob(torch.round(x * 255))

    def sample(self, y):
        pass


@NNDistribution.register
class UnitGaussianDistribution(nn.Module):
    """distlib.py:93-101 (VQ-VAE training loss only)."""

    def log_prob(self, x, y):
        return torch.distributions.Normal(y, torch.ones_like(y)).log_prob(x)

    def sample(self, y):
        pass
