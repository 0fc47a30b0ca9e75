"""DenseBlock (mirror of nnblock.py:24-56): `depth` DenseLayers growing the
channels by growth_channel in total, then a zero-initialised 1x1 head.  On the
device the whole block is ONE call into libidfcodec (idf_dense_block_f32): the
concatenations are column ranges of one pixel-major feature buffer.

ResBlock (nnblock.py:59-84) is the VQ-VAE's residual block (configs 3-5); on the
device it runs inside idfcodec.vq.VQEngine as two tap-table convs, the second
with the residual add and ReLU fused into its epilogue."""
from copy import deepcopy

from torch import nn

import moduleregister
from nnlayer import NNLayer


class NNBlock(moduleregister.Register):
    def __init__(self):
        super().__init__()


@NNBlock.register
class DenseBlock(nn.Module):
    def __init__(self, i_channel, o_channel, layer, growth_channel=512, depth=8):
        super().__init__()
        self.i_channel = i_channel
        self.o_channel = o_channel
        self.growth_channel = growth_channel
        self.depth = depth
        layer = dict(layer)
        self.layer_type = NNLayer.get(layer.pop("name"))
        self.act_name = layer.get("act", "ReLU")
        self.layers = nn.ModuleList()
        channel = i_channel
        for idx in range(depth):
            growth = (idx + 1) * growth_channel // depth - idx * growth_channel // depth
            self.layers.append(self.layer_type(i_channel=channel, o_channel=channel + growth,
                                               **deepcopy(layer)))
            channel += growth
        assert channel == i_channel + growth_channel
        self.layers.append(nn.Conv2d(i_channel + growth_channel, o_channel, 1))
        nn.init.zeros_(self.layers[-1].weight)
        nn.init.zeros_(self.layers[-1].bias)

    def forward(self, x):
        from idfcodec.modules import run_dense_block
        return run_dense_block(self, x)


@NNBlock.register
class ResBlock(nn.Module):
    """nnblock.py:59-84: relu(x + conv3x3(relu(conv3x3(x))))."""

    def __init__(self, channel: int, batch_norm: bool = False):
        super().__init__()
        self.channel = channel
        if batch_norm:
            self.resblock = nn.Sequential(
                nn.Conv2d(channel, channel, kernel_size=3, padding=1), nn.ReLU(True),
                nn.BatchNorm2d(channel),
                nn.Conv2d(channel, channel, kernel_size=3, padding=1), nn.BatchNorm2d(channel))
        else:
            self.resblock = nn.Sequential(
                nn.Conv2d(channel, channel, kernel_size=3, padding=1), nn.ReLU(True),
                nn.Conv2d(channel, channel, kernel_size=3, padding=1))
        self.act = nn.ReLU(True)

    def forward(self, x):
        raise NotImplementedError("ResBlock runs inside the VQ-VAE engine (idfcodec.vq); "
                                  "call VQVAE.forward / encode / decode")
