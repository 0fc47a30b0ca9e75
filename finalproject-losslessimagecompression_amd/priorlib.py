"""Prior network (mirror of priorlib.py:17-47): mean/logscale of the factored-out
latents from a DenseBlock over the kept half (or over zeros when the prior has
no condition, priorlib.py:42-46 -- data independent, so the FlowEngine computes
it once per model).  On the device the split into mean / logscale, and
scale = exp(logscale) for the coder, are the head GEMM's epilogue."""
import moduleregister
from nnblock import NNBlock
from roundlib import NNRound
from torch import nn as tnn


class NNPrior(moduleregister.Register):
    def __init__(self):
        super().__init__()


@NNPrior.register
class Prior(tnn.Module):
    def __init__(self, out_channel, cond_channel, round=None, nn=None):
        super().__init__()
        self.out_channel = out_channel
        self.cond_channel = cond_channel
        round = dict(round)
        nn = dict(nn)
        self.round = NNRound.get(round.pop("name"))(**round)
        self.nn_type = NNBlock.get(nn.pop("name"))
        if cond_channel > 0:
            self.NN = self.nn_type(cond_channel, out_channel * 2, **nn)
        else:
            self.NN = self.nn_type(out_channel, out_channel * 2, **nn)

    def forward(self, cond):
        from idfcodec.modules import run_prior
        return run_prior(self, cond)
