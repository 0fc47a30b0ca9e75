"""Additive coupling (mirror of couplelib.py:23-61): zb = xb + Round(NN(xa)).
On the device the Round and the add are the epilogue of the DenseBlock's head
GEMM (IDF_EPI_COUPLE_ADD / _SUB), so the NN output never round-trips HBM."""
import moduleregister
from invertible import InvertibleModule
from nnblock import NNBlock
from roundlib import NNRound


class NNCouple(moduleregister.Register):
    def __init__(self):
        super().__init__()


@NNCouple.register
class AdditiveCouple(InvertibleModule):
    def __init__(self, channel, split=0.75, nn=None, round=None):
        super().__init__()
        self.channel = channel
        self.split = split
        self.a_ch = int(channel * split)
        self.b_ch = channel - self.a_ch
        nn = dict(nn)
        round = dict(round)
        self.nn_type = NNBlock.get(nn.pop("name"))
        self.dense = self.nn_type(i_channel=self.a_ch, o_channel=self.b_ch, **nn)
        self.round_type = NNRound.get(round.pop("name"))
        self.round = self.round_type(**round)

    def forward(self, x, logv, nbits=None):
        from idfcodec.modules import run_couple
        return run_couple(self, x, +1), logv

    def backward(self, z, nbits=None):
        from idfcodec.modules import run_couple
        return run_couple(self, z, -1)
