"""Discretised logistic (mirror of distlib.py:34-70).  log_prob gives the
theoretical bpd the reference logs next to the real one (flows.py:154-169);
it is not on the coding path (the coder uses the bit-exact CDF of
idfcodec/csrc/idf_cdf.h).  BinomialDistribution / UnitGaussianDistribution are
VQ-VAE training losses (distlib.py:73-101); they are registered so the residual
configs construct, and compute with torch.distributions (not a coding path)."""
import torch
import torch.nn.functional as F
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
        require_device(x, "DLogistic input")
        scale = torch.exp(logscale)
        bins = 2 ** nbits
        x_pos = (x + 0.5 / bins - mean) / scale
        x_neg = (x - 0.5 / bins - mean) / scale
        lp, ln = F.logsigmoid(x_pos), F.logsigmoid(x_neg)
        return lp + torch.log(1 - torch.exp(ln - lp) + eps)

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
