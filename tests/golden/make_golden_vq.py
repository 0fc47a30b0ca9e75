"""tests/golden/make_golden_vq.py -- golden fixtures of the residual configs' VQ-VAE.

Runs ONLY in the build container: builds the REFERENCE VQVAE (vqvae.py, imported from
/root/reference with a `colorama` stub and bytecode writing disabled) from small seeded
configs, and records data only -- the state_dict, a grid-valued input batch, the encoder
output, the quantiser indices (the reference's distance formula, roundlib.py:56-62), the
decoder output on embed[idx] and the rounded reconstruction (trainer.py:606-607), plus
Patching round trips (extenddim.py:40-67).  Re-run:  python tests/golden/make_golden_vq.py
"""
from __future__ import annotations

import os
import random
import sys
import types

sys.dont_write_bytecode = True
os.environ["PYTHONDONTWRITEBYTECODE"] = "1"

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.modules.setdefault("colorama", types.SimpleNamespace(reinit=None))
sys.path.insert(0, REF)

import vqvae as ref_vqvae  # noqa: E402
import extenddim as ref_extenddim  # noqa: E402

torch.set_num_threads(8)

CASES = {
    # name: (embed_num, embed_dim, hidden_dims, block_num, B, H, W)
    "vq_t1_3down": (64, 16, [8, 16, 24], 2, 2, 32, 32),
    "vq_t2_2down": (128, 20, [12, 20], 1, 3, 16, 24),
}


def build(embed_num, embed_dim, hidden, block_num):
    random.seed(0)
    torch.manual_seed(0)
    cfg = {"channel": 3, "embed_num": embed_num, "embed_dim": embed_dim,
           "encoder": {"name": "VQEncoder", "block_num": block_num,
                       "block": {"name": "ResBlock", "batch_norm": False}},
           "decoder": {"name": "VQDecoder", "block_num": block_num,
                       "block": {"name": "ResBlock", "batch_norm": False}},
           "distribution": {"name": "BinomialDistribution"},
           "vectorquantizer": {"reinit_interval": 1000, "threshold": 0.1},
           "hidden_dims": hidden, "batch_norm": False}
    m = ref_vqvae.EnDecoder.get("VQVAE")(**cfg)
    m.eval()
    return m


def main():
    for name, (K, D, hidden, nb, B, H, W) in CASES.items():
        m = build(K, D, hidden, nb)
        g = torch.Generator().manual_seed(3)
        k = torch.randint(0, 256, (B, 3, H, W), generator=g)
        data = (k + (k >= 128).long()).float() / 256  # trainer.py:101 dequant (R1)
        with torch.no_grad():
            z = m.encoder((data - 0.5) / 0.5)
            zf = z.permute(0, 2, 3, 1).reshape(-1, D)
            e = m.vq.embed.weight
            d = torch.sum(zf ** 2, dim=1, keepdim=True) + torch.sum(e ** 2, dim=1) - 2 * torch.matmul(zf, e.t())
            srt = torch.sort(d, dim=1).values
            margin = (srt[:, 1] - srt[:, 0]).numpy()
            idx = torch.argmin(d, dim=1)
            v = e[idx].view(B, z.shape[2], z.shape[3], D).permute(0, 3, 1, 2)
            y = m.decoder(v)
            rec = torch.round((y * 0.5 + 0.5) * 256) / 256
            full = m.forward((data - 0.5) / 0.5, require_loss=False)
        pt = ref_extenddim.Patching(H, W, H // 2, W // 2)
        patches, _ = pt.forward(data, None)
        out = {"data": data.numpy(), "z": z.numpy(), "idx": idx.view(B, z.shape[2], z.shape[3]).numpy(),
               "d_margin": margin, "dec": y.numpy(), "rec": rec.numpy(), "full": full.numpy(),
               "patches": patches.numpy(), "meta": np.array([K, D, len(hidden), nb, B, H, W])}
        for kk, vv in m.state_dict().items():
            out["sd/" + kk] = vv.numpy()
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
        print(name, {k2: v2.shape for k2, v2 in out.items() if not k2.startswith("sd/")})


if __name__ == "__main__":
    main()
