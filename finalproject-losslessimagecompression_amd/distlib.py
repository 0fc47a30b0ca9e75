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


def dlogistic_log_prob(x, mean, logscale, nbits=8, eps=1e-8, groups=1, logp=None, sums=True):
    """idf_log_prob over device tensors of x's element count, split into `groups` equal groups:
    fills `logp` (if given) and returns the per-group f64 sums (fixed-order reduction), or None
    with sums=False (then one grid-stride elementwise launch fills logp).  mean / logscale are
    moved to x's device as contiguous fp32 and must have exactly x.numel() elements (broadcast
    them first); logp must be a contiguous fp32 device tensor of that size."""
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    require_device(x, "log_prob input")
    n = x.numel()
    x = x.contiguous().float()
    mean, logscale = (t.to(device=x.device, dtype=torch.float32).contiguous()
                      if isinstance(t, torch.Tensor) else
                      torch.as_tensor(t, dtype=torch.float32, device=x.device)
                      for t in (mean, logscale))
    for name, t in (("mean", mean), ("logscale", logscale)):
        if t.numel() != n:
            raise ValueError(f"log_prob {name} has {t.numel()} elements, x has {n}: "
                             "broadcast the parameters to x's shape first")
    if logp is not None:
        if (logp.device != x.device or logp.dtype != torch.float32 or not logp.is_contiguous()
                or logp.numel() != n):
            raise ValueError("log_prob output must be a contiguous fp32 tensor on x's device "
                             "with x.numel() elements")
    groups = max(int(groups), 1)
    if n % groups:
        raise ValueError("log_prob groups must divide the element count")
    if not sums and logp is None:
        raise ValueError("log_prob with sums=False needs an output tensor")
    out = torch.empty(groups, dtype=torch.float64, device=x.device) if sums else None
    check(lib().idf_log_prob(_lib.stream_ptr(x.device), groups, n // groups, ptr(x),
                             ptr(mean), ptr(logscale), int(nbits), float(eps),
                             ptr(logp) if logp is not None else None,
                             ptr(out) if out is not None else None), "log_prob")
    return out


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
        mean, logscale = (t.to(x.device) if isinstance(t, torch.Tensor) else
                          torch.as_tensor(t, dtype=torch.float32, device=x.device)
                          for t in (mean, logscale))
        x, mean, logscale = torch.broadcast_tensors(x, mean, logscale)
        out = torch.empty(x.shape, dtype=torch.float32, device=x.device)
        dlogistic_log_prob(x, mean, logscale, nbits, eps, logp=out, sums=False)
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
