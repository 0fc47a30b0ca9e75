"""oracle/vqvae_oracle.py -- TEST INFRASTRUCTURE ONLY (never imported by the product).

CPU restatement of the residual configs' VQ-VAE (vqvae.py:22-168), its ResBlock
(nnblock.py:59-84), the vector quantiser's index (roundlib.py:56-62), the residual split
(trainer.py:604-608) and Patching (extenddim.py:40-67), in torch fp32 on the CPU, working
from a state_dict with the reference's keys.  Pinned against tests/golden/vq_*.npz, which
tests/golden/make_golden_vq.py produced by running the reference modules themselves.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

LEAKY = 0.01


def _w(sd, k):
    return sd[k].float()


def resblock(x, sd, p):
    """nnblock.py:72-84 (batch_norm False): relu(x + conv(relu(conv(x))))."""
    t = F.relu(F.conv2d(x, _w(sd, p + "resblock.0.weight"), _w(sd, p + "resblock.0.bias"), 1, 1))
    r = F.conv2d(t, _w(sd, p + "resblock.2.weight"), _w(sd, p + "resblock.2.bias"), 1, 1)
    return F.relu(x + r)


def encoder(x, sd, n_hidden, block_num, prefix="encoder.blocks."):
    """vqvae.py:22-63: x in [-1, 1] -> tanh(latent)."""
    i = 0
    for _ in range(n_hidden):  # Conv2d(ch, dim, 4, 2, 1) + LeakyReLU (vqvae.py:38-41)
        x = F.leaky_relu(F.conv2d(x, _w(sd, f"{prefix}{i}.0.weight"), _w(sd, f"{prefix}{i}.0.bias"),
                                  2, 1), LEAKY)
        i += 1
    x = F.leaky_relu(F.conv2d(x, _w(sd, f"{prefix}{i}.0.weight"), _w(sd, f"{prefix}{i}.0.bias"), 1,
                              1), LEAKY)  # vqvae.py:49-52
    i += 1
    for _ in range(block_num):  # vqvae.py:53-55
        x = resblock(x, sd, f"{prefix}{i}.")
        i += 1
    x = F.conv2d(x, _w(sd, f"{prefix}{i}.weight"), _w(sd, f"{prefix}{i}.bias"))  # vqvae.py:56
    return torch.tanh(x)  # vqvae.py:57,62


def decoder(v, sd, n_hidden, block_num, prefix="decoder.blocks."):
    """vqvae.py:66-113: latent -> tanh image in [-1, 1]."""
    i = 0
    x = F.leaky_relu(F.conv2d(v, _w(sd, f"{prefix}{i}.0.weight"), _w(sd, f"{prefix}{i}.0.bias")),
                     LEAKY)  # vqvae.py:81-84
    i += 1
    for _ in range(block_num):  # vqvae.py:85-87
        x = resblock(x, sd, f"{prefix}{i}.")
        i += 1
    x = F.leaky_relu(F.conv2d(x, _w(sd, f"{prefix}{i}.0.weight"), _w(sd, f"{prefix}{i}.0.bias"), 1,
                              1), LEAKY)  # vqvae.py:88-91
    i += 1
    for _ in range(n_hidden - 1):  # ConvTranspose2d(ch, dim, 4, 2, 1) + LeakyReLU (vqvae.py:92-103)
        x = F.leaky_relu(F.conv_transpose2d(x, _w(sd, f"{prefix}{i}.0.weight"),
                                            _w(sd, f"{prefix}{i}.0.bias"), 2, 1), LEAKY)
        i += 1
    x = F.conv_transpose2d(x, _w(sd, f"{prefix}{i}.0.weight"), _w(sd, f"{prefix}{i}.0.bias"), 2, 1)
    return torch.tanh(x)  # vqvae.py:104-107


def vq_indices(z, embed):
    """roundlib.py:56-62: z [N, D] -> argmin_k (|z|^2 + |e_k|^2 - 2 z.e_k)."""
    x2 = torch.sum(z ** 2, dim=1, keepdim=True)
    z2 = torch.sum(embed ** 2, dim=1)
    d = x2 + z2 - 2 * torch.matmul(z, embed.t())
    return torch.argmin(d, dim=1)


def indices(data, sd, n_hidden, block_num):
    """trainer.py:606 scaling + vqvae.py:135-147: data [B,C,H,W] on the grid -> idx [B,h,w]."""
    z = encoder((data - 0.5) / 0.5, sd, n_hidden, block_num)
    B, D, h, w = z.shape
    idx = vq_indices(z.permute(0, 2, 3, 1).reshape(-1, D), _w(sd, "vq.embed.weight"))
    return idx.view(B, h, w), z


def reconstruct(idx, sd, n_hidden, block_num):
    """rec = round8(decoder(embed[idx]) * 0.5 + 0.5) (trainer.py:606-607 on embed[idx])."""
    e = _w(sd, "vq.embed.weight")
    B, h, w = idx.shape
    v = e[idx.reshape(-1)].view(B, h, w, -1).permute(0, 3, 1, 2)
    y = decoder(v, sd, n_hidden, block_num)
    return torch.round((y * 0.5 + 0.5) * 256) / 256, y


def patch(x, h, w):
    """Patching.forward (extenddim.py:52-58)."""
    B, C, H, W = x.shape
    x = x.view(B, C, H // h, h, W // w, w).permute(0, 2, 4, 1, 3, 5).contiguous()
    return x.view(-1, C, h, w)


def unpatch(x, H, W):
    """Patching.backward (extenddim.py:60-67)."""
    n, C, h, w = x.shape
    hh, ww = H // h, W // w
    x = x.view(n // hh // ww, hh, ww, C, h, w).permute(0, 3, 1, 4, 2, 5).contiguous()
    return x.view(-1, C, H, W)
