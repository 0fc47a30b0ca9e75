"""Invertible base modules (mirror of invertible.py:7-76).

Permute keeps the reference's 0/1 matrix parameters P / inv_P (state_dict
compatibility, invertible.py:29-36, drawn with `random.shuffle` in the same
order so seeded models match).  On the device the permutation is a channel
gather (`y[:, i] = x[:, ids[i]]`, ids = argmax of P's rows), fused by the
FlowEngine with the coupling's input copy; no matmul is run."""
import random

import torch
from torch import nn
from torch.nn.parameter import Parameter

from idfcodec._lib import require_device


class InvertibleModule(nn.Module):
    def __init__(self, *args, **kwargs):
        super().__init__()

    def build(self):
        pass

    def forward(self, *args, **kwargs):
        raise NotImplementedError

    def backward(self, *args, **kwargs):
        raise NotImplementedError

    def inverse(self, *args, **kwargs):
        pass


class Permute(InvertibleModule):
    def __init__(self, dim):
        super().__init__()
        ids = list(range(dim))
        random.shuffle(ids)
        p = torch.zeros((dim, dim))
        p[torch.arange(dim), torch.tensor(ids)] = 1
        self.P = Parameter(p, requires_grad=False)
        self.inv_P = Parameter(p.t(), requires_grad=False)

    def ids(self):
        return torch.argmax(self.P, dim=1)

    def forward(self, x, logv):
        require_device(x, "Permute input")
        return x[:, self.ids().to(x.device)], logv

    def backward(self, x):
        require_device(x, "Permute input")
        return x[:, torch.argmax(self.inv_P, dim=1).to(x.device)]


class InvertibleModuleList(InvertibleModule, nn.ModuleList):
    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)

    def inverse(self):
        for m in self:
            if isinstance(m, InvertibleModule):
                m.inverse()

    def forward(self, x, logv, *args, **kwargs):
        for m in self:
            x, logv = m.forward(x, logv, *args, **kwargs)
        return x, logv

    def backward(self, x, *args, **kwargs):
        for m in reversed(list(self)):
            x = m.backward(x, *args, **kwargs)
        return x


class LULinear(InvertibleModule):
    """stub in the reference too (invertible.py:74-76)"""
