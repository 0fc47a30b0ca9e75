"""Coder API (mirror of coder.py:18-38): Encode / Decode over per-level latents
with the rANS state chained across levels.

Encode is bit-identical to the reference's.  Decode fixes the reference's
chained-state bug: after a level the reference decoder defers one
renormalisation read, which then consumes a word of the NEXT level's buffer.
Here, after each level, a state below L = 2^32 takes that level's first-pushed
word, which is exactly the word the encoder emitted before that level's first
symbol -- so Decode(Encode(...)) round-trips and ends at the initial state.

The batched device path (one stream per image and level, no Python lists) is
idfcodec.codec.StreamCoder / IDFlows.encode.
"""
import torch

from rans.rans import decode, encode

RANS_L = 1 << 32


def Encode(latents, means, logscales, x=(1 << 32)):
    buffers = []
    for i in range(len(latents)):
        latent = latents[i].reshape(-1).tolist()
        scale = torch.exp(logscales[i]).reshape(-1).tolist()
        mean = means[i].reshape(-1).tolist()
        x, buf = encode(x, len(latent), latent, mean, scale)
        buffers.append(buf)
    return x, buffers


def Decode(buffers, means, logscales, x):
    latents = []
    for i in range(len(means)):
        idx = len(means) - 1 - i
        mean = means[idx].reshape(-1).tolist()
        scale = torch.exp(logscales[idx]).reshape(-1).tolist()
        x, latent = decode(x, buffers[idx][::-1], len(mean), mean[::-1], scale[::-1])
        if x < RANS_L and len(buffers[idx]) > 0:
            x = (x << 32) | buffers[idx][0]  # the deferred read (F4 fix)
        latents.append(torch.tensor(latent[::-1]).to(means[idx]).reshape(*means[idx].shape))
    return x, latents[::-1]
