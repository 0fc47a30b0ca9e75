"""DenseLayer (mirror of nnlayer.py:22-51): conv1x1(c->c) -> conv3x3(c->g, pad 1)
-> act, concatenated after the input.  Same parameters (and creation order) as
the reference, so state_dicts and seeded initialisation carry over.  forward()
runs the HIP kernels (idfcodec.modules.run_dense_layer)."""
from torch import nn

import moduleregister
from activate import ActivateFunc


class NNLayer(moduleregister.Register):
    def __init__(self):
        super().__init__()


ACTS = {"ReLU": nn.ReLU, "Tanh": nn.Tanh, "LeakyReLU": nn.LeakyReLU}


@NNLayer.register
class DenseLayer(nn.Module):
    def __init__(self, i_channel, o_channel, act="ReLU"):
        super().__init__()
        self.i_channel = i_channel
        self.o_channel = o_channel
        self.act_name = act
        self.act = ACTS[act]() if act in ACTS else ActivateFunc.get(act)()
        self.layers = nn.Sequential(
            nn.Conv2d(i_channel, i_channel, kernel_size=1),
            nn.Conv2d(i_channel, o_channel - i_channel, kernel_size=3, padding=1),
            self.act,
        )

    def forward(self, x):
        from idfcodec.modules import run_dense_layer
        return run_dense_layer(self, x)
