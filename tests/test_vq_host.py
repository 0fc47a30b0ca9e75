"""Host-side checks of the residual configs' VQ-VAE (no GPU): the oracle against the
reference-generated fixtures, the tap-table packing against torch's convolutions, and the
mirror modules' constructor parity (same seeded weights, same state_dict keys)."""
import os
import random
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "finalproject-losslessimagecompression_amd"))

import vqvae_oracle as VO  # noqa: E402

CASES = ["vq_t1_3down", "vq_t2_2down"]


def load(name):
    z = np.load(os.path.join(HERE, "golden", name + ".npz"))
    sd = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd/")}
    return z, sd


@pytest.mark.parametrize("name", CASES)
def test_oracle_matches_reference_fixtures(name):
    z, sd = load(name)
    K, D, nh, nb, B, H, W = [int(v) for v in z["meta"]]
    data = torch.from_numpy(z["data"])
    idx, zz = VO.indices(data, sd, nh, nb)
    assert torch.allclose(zz, torch.from_numpy(z["z"]), atol=1e-6, rtol=1e-5)
    assert torch.equal(idx, torch.from_numpy(z["idx"]))
    rec, y = VO.reconstruct(idx, sd, nh, nb)
    assert torch.allclose(y, torch.from_numpy(z["dec"]), atol=1e-6, rtol=1e-5)
    assert torch.equal(rec, torch.from_numpy(z["rec"]))
    # the reference's straight-through forward differs from decoder(embed[idx]) by ulps only
    assert np.abs(z["full"] - z["dec"]).max() < 1e-5
    p = VO.patch(data, H // 2, W // 2)
    assert torch.equal(p, torch.from_numpy(z["patches"]))
    assert torch.equal(VO.unpatch(p, H, W), data)


def tap_conv_np(x, c, Ho, Wo):
    """The device kernel's arithmetic contract in numpy (float64): x [B,Hi,Wi,C]."""
    B, Hi, Wi, C = x.shape
    Hc, Wc = (Hi, Wi) if c.osy == 2 else (Ho, Wo)
    out = np.zeros((B, Ho, Wo, c.cout))
    w = c.w[: c.cout, :, :C].astype(np.float64)
    for m in range(Hc):
        for n in range(Wc):
            acc = np.tile(c.bias[: c.cout].astype(np.float64), (B, 1))
            for t in range(len(c.dy)):
                iy, ix = m * c.isy + c.dy[t], n * c.isy + c.dx[t]
                if 0 <= iy < Hi and 0 <= ix < Wi:
                    acc = acc + x[:, iy, ix, :] @ w[:, t, :].T
            out[:, m * c.osy + c.oy0, n * c.osy + c.ox0, :] = acc
    return out


@pytest.mark.parametrize("k,s,p,ci,co,H", [(4, 2, 1, 3, 8, 8), (3, 1, 1, 5, 7, 6), (1, 1, 0, 6, 4, 5)])
def test_pack_conv_matches_conv2d(k, s, p, ci, co, H):
    from idfcodec.vq import pack_conv
    g = torch.Generator().manual_seed(k * 10 + ci)
    w = torch.randn(co, ci, k, k, generator=g, dtype=torch.float64)
    b = torch.randn(co, generator=g, dtype=torch.float64)
    x = torch.randn(2, ci, H, H + 2, generator=g, dtype=torch.float64)
    ref = F.conv2d(x, w, b, s, p).permute(0, 2, 3, 1).numpy()
    c = pack_conv(w.numpy(), b.numpy(), s, p)
    got = tap_conv_np(x.permute(0, 2, 3, 1).numpy(), c, ref.shape[1], ref.shape[2])
    assert np.abs(got - ref).max() < 1e-5


@pytest.mark.parametrize("ci,co,H,W", [(4, 3, 3, 5), (6, 8, 4, 4)])
def test_pack_convT_matches_conv_transpose2d(ci, co, H, W):
    from idfcodec.vq import pack_convT
    g = torch.Generator().manual_seed(ci * 7 + co)
    w = torch.randn(ci, co, 4, 4, generator=g, dtype=torch.float64)
    b = torch.randn(co, generator=g, dtype=torch.float64)
    x = torch.randn(2, ci, H, W, generator=g, dtype=torch.float64)
    ref = F.conv_transpose2d(x, w, b, 2, 1).permute(0, 2, 3, 1).numpy()
    got = np.zeros_like(ref)
    for c in pack_convT(w.numpy(), b.numpy()):
        part = tap_conv_np(x.permute(0, 2, 3, 1).numpy(), c, 2 * H, 2 * W)
        got[:, c.oy0::2, c.ox0::2, :] = part[:, c.oy0::2, c.ox0::2, :]
    assert np.abs(got - ref).max() < 1e-5  # packed weights are fp32


@pytest.mark.parametrize("name", CASES)
def test_mirror_modules_build_reference_weights(name):
    """The package's VQVAE (vqvae.py mirror) built from the same seeded config holds the
    reference's parameters under the reference's keys."""
    import vqvae as mirror
    z, sd = load(name)
    K, D, nh, nb, B, H, W = [int(v) for v in z["meta"]]
    hidden = {"vq_t1_3down": [8, 16, 24], "vq_t2_2down": [12, 20]}[name]
    random.seed(0)
    torch.manual_seed(0)
    cfg = {"channel": 3, "embed_num": K, "embed_dim": D,
           "encoder": {"name": "VQEncoder", "block_num": nb,
                       "block": {"name": "ResBlock", "batch_norm": False}},
           "decoder": {"name": "VQDecoder", "block_num": nb,
                       "block": {"name": "ResBlock", "batch_norm": False}},
           "distribution": {"name": "BinomialDistribution"},
           "vectorquantizer": {"reinit_interval": 1000, "threshold": 0.1},
           "hidden_dims": hidden, "batch_norm": False}
    m = mirror.EnDecoder.get("VQVAE")(**cfg)
    got = m.state_dict()
    assert sorted(got) == sorted(sd)
    for k in sd:
        assert torch.equal(got[k], sd[k]), k


def test_stage_lists_follow_reference_structure():
    import vqvae as mirror
    from idfcodec.vq import decoder_stages, encoder_stages
    z, sd = load("vq_t1_3down")
    random.seed(0)
    torch.manual_seed(0)
    m = mirror.EnDecoder.get("VQVAE")(
        channel=3, embed_num=64, embed_dim=16,
        encoder={"name": "VQEncoder", "block_num": 2, "block": {"name": "ResBlock"}},
        decoder={"name": "VQDecoder", "block_num": 2, "block": {"name": "ResBlock"}},
        distribution={"name": "BinomialDistribution"}, hidden_dims=[8, 16, 24])
    enc = encoder_stages(m.encoder)
    dec = decoder_stages(m.decoder)
    assert [s.kind for s in enc] == ["conv"] * 4 + ["res"] * 2 + ["conv"]
    assert [s.stride for s in enc[:3]] == [2, 2, 2]
    assert [s.kind for s in dec] == ["conv", "res", "res", "conv", "convT", "convT", "convT"]
    assert enc[-1].act == 2 and dec[-1].act == 2  # tanh
