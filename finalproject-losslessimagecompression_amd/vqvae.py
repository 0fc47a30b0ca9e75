"""VQ-VAE of the residual configs (mirror of vqvae.py:17-168).

VQEncoder / VQDecoder / VQVAE keep the reference's constructor kwargs, registry names
(Register / EnDecoder), submodule tree and parameter creation order, so the same YAML
builds them, the same checkpoints load (state_dict keys `encoder.blocks.*`,
`decoder.blocks.*`, `vq.embed.weight`, ...), and a seeded init gives the same weights.

The forward pass runs in idfcodec.vq.VQEngine (HIP): every conv is a tap-table implicit
GEMM on MFMA, the quantiser a fused argmin kernel.  `forward` / `encode` / `decode` keep
the reference signatures (NCHW in the reference's [-1, 1] scaling); `indices` /
`reconstruct` are the codec entry points (trainer.py:604-608 residual split).
"""
from copy import deepcopy

import torch
from torch import nn

from moduleregister import Register
from nnblock import NNBlock
from roundlib import VectorQuantizer
from distlib import NNDistribution
from idfcodec._lib import require_device


class EnDecoder(Register):
    def __init__(self):
        super().__init__()


def _conv_seq(conv, batch_norm, dim, act=None):
    mods = [conv, act if act is not None else nn.LeakyReLU(inplace=True)]
    if batch_norm:
        mods.append(nn.BatchNorm2d(dim))
    return nn.Sequential(*mods)


@Register.register
class VQEncoder(nn.Module):
    """vqvae.py:22-63: [Conv4x4/s2 + LeakyReLU] per hidden dim, Conv3x3 + LeakyReLU,
    block_num blocks, 1x1 to the embedding dim, Tanh."""

    def __init__(self, in_channel, out_channel, block, block_num, hidden_dims=[128, 256],
                 batch_norm=False):
        super().__init__()
        self.blocks = nn.ModuleList()
        ch = in_channel
        for dim in hidden_dims:
            self.blocks.append(_conv_seq(nn.Conv2d(ch, dim, 4, 2, 1), batch_norm, dim))
            ch = dim
        self.blocks.append(_conv_seq(nn.Conv2d(ch, ch, 3, 1, 1), batch_norm, ch))
        block = dict(block)
        block_type = NNBlock.get(block.pop("name"))
        for _ in range(block_num):
            self.blocks.append(block_type(channel=ch, **deepcopy(block)))
        self.blocks.append(nn.Conv2d(ch, out_channel, 1))
        self.act = nn.Tanh()


@Register.register
class VQDecoder(nn.Module):
    """vqvae.py:66-113: 1x1 + LeakyReLU, block_num blocks, Conv3x3 + LeakyReLU,
    [ConvTranspose4x4/s2 + LeakyReLU] per further hidden dim, ConvTranspose to the image
    channels + Tanh."""

    def __init__(self, in_channel, out_channel, block, block_num, hidden_dims=[256, 128],
                 batch_norm=False):
        super().__init__()
        self.blocks = nn.ModuleList()
        ch = hidden_dims[0]
        self.blocks.append(_conv_seq(nn.Conv2d(in_channel, ch, 1), batch_norm, ch))
        block = dict(block)
        block_type = NNBlock.get(block.pop("name"))
        for _ in range(block_num):
            self.blocks.append(block_type(channel=ch, **deepcopy(block)))
        self.blocks.append(_conv_seq(nn.Conv2d(ch, ch, 3, 1, 1), False, ch))
        for dim in hidden_dims[1:]:
            self.blocks.append(_conv_seq(nn.ConvTranspose2d(ch, dim, 4, 2, 1), batch_norm, dim))
            ch = dim
        self.blocks.append(nn.Sequential(nn.ConvTranspose2d(ch, out_channel, 4, 2, 1), nn.Tanh()))


@EnDecoder.register
class VQVAE(nn.Module):
    """vqvae.py:116-168."""

    def __init__(self, channel, embed_num, embed_dim, encoder, decoder, distribution,
                 vectorquantizer={}, hidden_dims=[128, 256], batch_norm=False):
        super().__init__()
        self.channel = channel
        self.embed_num = embed_num
        self.embed_dim = embed_dim
        encoder, decoder, distribution = dict(encoder), dict(decoder), dict(distribution)
        self.encoder = Register.get(encoder.pop("name"))(
            in_channel=channel, out_channel=embed_dim, hidden_dims=hidden_dims,
            batch_norm=batch_norm, **encoder)
        self.decoder = Register.get(decoder.pop("name"))(
            in_channel=embed_dim, out_channel=channel, hidden_dims=hidden_dims[::-1],
            batch_norm=batch_norm, **decoder)
        self.vq = VectorQuantizer(num=embed_num, dim=embed_dim, **dict(vectorquantizer))
        self.dist = NNDistribution.get(distribution.pop("name"))(**distribution)
        self._engine = None
        self._engine_key = None

    # ------------------------------------------------------------ engine
    def engine(self):
        from idfcodec.vq import VQEngine
        dev = next(self.parameters()).device
        if dev.type != "cuda":
            raise RuntimeError("idfcodec: move the VQ-VAE to the HIP device (.cuda()) first; "
                               "there is no CPU path")
        key = tuple((p.data_ptr(), p._version) for p in self.parameters())
        if self._engine is None or self._engine_key != key:
            self._engine = VQEngine(self, dev)
            self._engine_key = key
        return self._engine

    def _to_pm(self, x):
        from idfcodec import _lib
        from idfcodec._lib import check, lib, ptr
        from idfcodec.packing import round_up
        B, C, H, W = x.shape
        pm = torch.zeros(B * H * W * round_up(C, 4), dtype=torch.float32, device=x.device)
        check(lib().idf_nchw_to_pm(_lib.stream_ptr(x.device), B, C, H, W, ptr(x), ptr(pm),
                                   round_up(C, 4)), "nchw->pm")
        return pm

    def _to_nchw(self, pm, B, C, H, W, ld):
        from idfcodec import _lib
        from idfcodec._lib import check, lib, ptr
        out = torch.empty((B, C, H, W), dtype=torch.float32, device=pm.device)
        check(lib().idf_pm_to_nchw(_lib.stream_ptr(pm.device), B, C, H, W, ptr(pm), ld, ptr(out)),
              "pm->nchw")
        return out

    # ------------------------------------------------------------ codec entry points
    def indices(self, data):
        """data [B, C, H, W] on the 1/256 grid (device) -> (int32 indices [B, h, w])."""
        require_device(data, "VQVAE input")
        data = data.float().contiguous()
        B, C, H, W = data.shape
        idx, (h, w), _ = self.engine().encode_pm(self._to_pm(data), B, H, W)
        return idx.view(B, h, w)

    def reconstruct(self, idx, conv=None):
        """indices [B, h, w] -> rec = round8(decoder(embed[idx]) * 0.5 + 0.5), NCHW.  conv: the
        decoder's conv arithmetic ("x3" / "f32", a bitstream's vq_conv); default the engine's
        mode with the range guard's fallback (engine().last_decode_mode tells which ran)."""
        require_device(idx, "VQ indices")
        B, h, w = idx.shape
        rec, (H, W) = self.engine().decode_pm(idx.to(torch.int32).contiguous().view(-1), B, h, w,
                                              conv)
        return self._to_nchw(rec, B, self.channel, H, W, 4)

    # ------------------------------------------------------------ reference API
    def encode(self, x, beta=0.25, gamma=1.0, require_loss=True):
        """vqvae.py:135-147: x in [-1, 1] -> quantised latent NCHW (and the VQ loss)."""
        require_device(x, "VQVAE input")
        x = x.float().contiguous()
        B, C, H, W = x.shape
        eng = self.engine()
        z, (h, w) = eng.encoder_raw_pm(self._to_pm(x), B, H, W)
        from idfcodec.packing import round_up
        D4 = round_up(self.embed_dim, 4)
        zr = z.view(-1, D4)[:, : self.embed_dim].contiguous()
        vq = self.vq.forward(zr, beta=beta, gamma=gamma, require_loss=require_loss)
        vq_x = vq[0] if require_loss else vq
        vq_nchw = vq_x.view(B, h, w, self.embed_dim).permute(0, 3, 1, 2).contiguous()
        return (vq_nchw, vq[1]) if require_loss else vq_nchw

    def decode(self, x):
        """vqvae.py:149-151: latent NCHW -> decoder output in [-1, 1]."""
        require_device(x, "VQVAE latent")
        x = x.float().contiguous()
        B, D, h, w = x.shape
        from idfcodec import _lib
        from idfcodec._lib import check, lib, ptr
        from idfcodec.packing import round_up
        D4 = round_up(D, 4)
        pm = torch.zeros(B * h * w * D4, dtype=torch.float32, device=x.device)
        check(lib().idf_nchw_to_pm(_lib.stream_ptr(x.device), B, D, h, w, ptr(x), ptr(pm), D4),
              "nchw->pm")
        y, (H, W) = self.engine().decoder_raw_pm(pm, B, h, w)
        return self._to_nchw(y, B, self.channel, H, W, 4)

    def forward(self, x, beta=0.25, gamma=1.0, require_loss=True):
        if require_loss:
            vq_x, loss = self.encode(x, beta=beta, gamma=gamma, require_loss=True)
            return self.decode(vq_x), loss
        return self.decode(self.encode(x, beta=beta, gamma=gamma, require_loss=False))
