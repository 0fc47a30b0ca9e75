"""GPU parity of the residual configs' VQ-VAE (csrc/vq_kernels.hip through idfcodec.vq)
against the reference-generated fixtures (tests/golden/vq_*.npz): encoder output and
decoder output within 1e-5, quantiser indices equal wherever the reference's distance
margin between the best two codes exceeds fp32 noise, reconstruction on the 1/256 grid
equal except at rounding ties, Patching exact; and the fused argmin at the config-3
codebook size (16384 x 512) against a float64 CPU search."""
import os
import random
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
CASES = {"vq_t1_3down": [8, 16, 24], "vq_t2_2down": [12, 20]}


def load(name):
    z = np.load(os.path.join(HERE, "golden", name + ".npz"))
    sd = {k[3:]: torch.from_numpy(z[k]) for k in z.files if k.startswith("sd/")}
    return z, sd


def model_for(name):
    import vqvae as mirror
    z, sd = load(name)
    K, D, nh, nb, B, H, W = [int(v) for v in z["meta"]]
    random.seed(0)
    torch.manual_seed(0)
    m = mirror.EnDecoder.get("VQVAE")(
        channel=3, embed_num=K, embed_dim=D,
        encoder={"name": "VQEncoder", "block_num": nb, "block": {"name": "ResBlock"}},
        decoder={"name": "VQDecoder", "block_num": nb, "block": {"name": "ResBlock"}},
        distribution={"name": "BinomialDistribution"}, hidden_dims=CASES[name])
    m.load_state_dict(sd)
    return m.cuda().eval(), z


@pytest.mark.parametrize("mode", ["x3", "f32"])
@pytest.mark.parametrize("name", list(CASES))
def test_vqvae_engine_matches_reference(name, mode):
    """Both conv modes of the ResBlock 3x3 convs: split-f16 products (the default) and the
    exact-f32 Winograd kernel; neither's range guard trips on the reference's data."""
    m, z = model_for(name)
    m.engine().conv_mode = mode
    data = torch.from_numpy(z["data"]).cuda()
    idx = m.indices(data)
    ok = z["d_margin"].reshape(idx.shape) > 1e-4
    got = idx.cpu().numpy()
    assert np.array_equal(got[ok], z["idx"][ok]), "quantiser indices differ"
    # encoder output through the reference API (x in [-1, 1])
    eng = m.engine()
    from idfcodec.packing import round_up
    B, C, H, W = data.shape
    zz, (h, w) = eng.encoder_raw_pm(m._to_pm((data - 0.5) / 0.5), B, H, W)
    D = m.embed_dim
    zz = zz.view(B, h, w, round_up(D, 4))[..., :D].permute(0, 3, 1, 2).cpu()
    err = (zz.double() - torch.from_numpy(z["z"]).double()).abs().max().item()
    assert err < 1e-5, err
    # decoder on the reference's indices
    ridx = torch.from_numpy(z["idx"]).cuda()
    rec = m.reconstruct(ridx).cpu().numpy()
    assert m.engine().last_decode_mode == mode
    dec = z["dec"]
    t = (dec * 0.5 + 0.5) * 256
    tie = np.abs(t - np.floor(t) - 0.5) < 1e-3
    assert np.array_equal(rec[~tie], z["rec"][~tie])
    e = m.vq.embed.weight.detach()
    v = e[ridx.long()].permute(0, 3, 1, 2).contiguous()
    y = m.decode(v).cpu().numpy()
    assert np.abs(y - dec).max() < 1e-5


def test_vq_range_guard_falls_back_to_f32():
    """A decoder input far outside the split-f16 range trips the guard: the pass is re-run in
    exact f32 and equals a pure-f32 run bit for bit; reconstruct(conv=...) reproduces each
    mode exactly (what a decoder does with the bitstream's vq_conv)."""
    m, z = model_for("vq_t2_2down")
    eng = m.engine()
    eng.conv_mode = "x3"
    B, D = 2, m.embed_dim
    from idfcodec.packing import round_up
    g = torch.Generator().manual_seed(3)
    h = w = 4
    v = torch.zeros(B * h * w, round_up(D, 4))
    v[:, :D] = torch.randn(B * h * w, D, generator=g)
    big = (v * 1e5).cuda().reshape(-1).contiguous()
    y, *_, mode = eng._guarded(eng.dec, big, B, h, w, D)
    assert mode == "f32"
    y32, *_, mode32 = eng._guarded(eng.dec, big, B, h, w, D, mode="f32")
    assert mode32 == "f32" and torch.equal(y, y32)
    ridx = torch.from_numpy(z["idx"]).cuda()
    for mode in ("x3", "f32"):
        a = m.reconstruct(ridx, conv=mode)
        assert eng.last_decode_mode == mode
        assert torch.equal(a, m.reconstruct(ridx, conv=mode))


@pytest.mark.parametrize("name", list(CASES))
def test_patching_matches_reference(name):
    from extenddim import Patching
    z, _ = load(name)
    data = torch.from_numpy(z["data"]).cuda()
    B, C, H, W = data.shape
    pt = Patching(H, W, H // 2, W // 2)
    p, _ = pt.forward(data, None)
    assert torch.equal(p.cpu(), torch.from_numpy(z["patches"]))
    assert torch.equal(pt.backward(p), data)


def test_vq_argmin_config3_codebook():
    """16384 x 512 codebook (resflow-cond-imagenet64.yaml), 2048 rows: the fused kernel's
    index equals a float64 search wherever the best two codes differ by > 1e-3."""
    from roundlib import VectorQuantizer
    torch.manual_seed(5)
    vq = VectorQuantizer(num=16384, dim=512).cuda()
    x = torch.tanh(torch.randn(2048, 512)).cuda()
    idx = vq.indices(x).cpu().long()
    e = vq.embed.weight.detach().cpu().double()
    xd = x.cpu().double()
    d = (xd ** 2).sum(1, keepdim=True) + (e ** 2).sum(1) - 2 * xd @ e.t()
    srt, order = torch.sort(d, dim=1)
    ok = (srt[:, 1] - srt[:, 0]) > 1e-3
    assert ok.float().mean() > 0.5
    assert torch.equal(idx[ok], order[ok, 0])


@pytest.mark.parametrize("P,K,D", [(8192, 8192, 512), (1000, 1100, 64), (77, 300, 20),
                                   (19872, 8192, 512)])
def test_vq_argmin_slices_equal_one_pass(P, K, D):
    """The codebook split into slices (idf_vq_argmin_ws with its workspace: separate blocks per
    slice, minima merged in slice order) gives the index of the one-pass search
    (idf_vq_argmin) bit for bit -- ragged row tiles, a K with a short or empty last slice, an
    odd D -- and both equal a float64 search wherever the best two codes differ by > 1e-3;
    ties (duplicated codes) go to the lowest index."""
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    g = torch.Generator().manual_seed(P + K)
    x = torch.tanh(torch.randn(P, D, generator=g)).cuda()
    e = (torch.randn(K, D, generator=g) * 0.5)
    e[K // 2] = e[K // 3]  # an exact tie: the lower index must win
    e = e.cuda()
    s = _lib.stream_ptr()
    en = torch.empty(K, device="cuda")
    check(lib().idf_vq_norms(s, K, D, ptr(e), D, ptr(en)), "norms")
    one = torch.empty(P, dtype=torch.int32, device="cuda")
    check(lib().idf_vq_argmin(s, P, D, ptr(x), D, ptr(e), D, K, ptr(en), ptr(one)), "argmin")
    nws = int(lib().idf_vq_argmin_workspace_bytes(P, K))
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device="cuda")
    sl = torch.empty(P, dtype=torch.int32, device="cuda")
    check(lib().idf_vq_argmin_ws(s, P, D, ptr(x), D, ptr(e), D, K, ptr(en), ptr(sl), ptr(ws), nws),
          "argmin ws")
    assert torch.equal(one, sl)
    if P * K <= 2_000_000:
        xd, ed = x.cpu().double(), e.cpu().double()
        d = (xd ** 2).sum(1, keepdim=True) + (ed ** 2).sum(1) - 2 * xd @ ed.t()
        srt, order = torch.sort(d, dim=1, stable=True)
        ok = (srt[:, 1] - srt[:, 0]) > 1e-3
        assert ok.float().mean() > 0.3
        assert torch.equal(one.cpu().long()[ok], order[ok, 0])
    assert not (one.cpu() == K // 2).any()  # the duplicate of code K // 3 never wins
