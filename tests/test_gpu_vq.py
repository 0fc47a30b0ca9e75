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


@pytest.mark.parametrize("mode", ["x3t", "x3", "f32"])
@pytest.mark.parametrize("name", list(CASES))
def test_vqvae_engine_matches_reference(name, mode):
    """The three VQ conv modes: every conv on split-f16 products ("x3t", the default), the
    ResBlock 3x3 convs only ("x3", round 5's) and exact f32; no range guard trips on the
    reference's data."""
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
    eng.conv_mode = "x3t"
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
    for mode in ("x3t", "x3", "f32"):
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


@pytest.mark.parametrize("P,K,D", [(8192, 16384, 512), (1000, 1100, 64), (77, 300, 20)])
def test_vq_argmin_x3_vs_fp64(P, K, D):
    """idf_vq_argmin_x3_ws (split-f16 x.e products): sliced and one-pass searches agree bit for
    bit, the index equals a float64 search (and the fp32 kernel's) wherever the best two codes
    differ by > 1e-3, ties go to the lowest index, and an input past the f16 pairs' range sets
    the flag."""
    from idfcodec import _lib, vq
    from idfcodec._lib import check, lib, ptr
    g = torch.Generator().manual_seed(P + K + 1)
    x = torch.tanh(torch.randn(P, D, generator=g)).cuda()
    e = (torch.randn(K, D, generator=g) * 0.5)
    e[K // 2] = e[K // 3]
    ex, ys = vq.taps_weights_x3(e.double().numpy().reshape(K, 1, D))
    ex = torch.from_numpy(ex.reshape(-1)).cuda()
    e = e.cuda()
    s = _lib.stream_ptr()
    en = torch.empty(K, device="cuda")
    check(lib().idf_vq_norms(s, K, D, ptr(e), D, ptr(en)), "norms")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    nws = int(lib().idf_vq_argmin_workspace_bytes(P, K))
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device="cuda")
    out = {}
    for name, (w, nw) in {"one": (None, 0), "sliced": (ws, nws)}.items():
        out[name] = torch.empty(P, dtype=torch.int32, device="cuda")
        check(lib().idf_vq_argmin_x3_ws(s, P, D, ptr(x), D, ptr(ex), D, ys, K, ptr(en),
                                        ptr(out[name]), ptr(w) if w is not None else None, nw,
                                        ptr(flag)), "argmin x3")
    assert torch.equal(out["one"], out["sliced"])
    assert int(flag.item()) == 0
    f32 = torch.empty(P, dtype=torch.int32, device="cuda")
    check(lib().idf_vq_argmin_ws(s, P, D, ptr(x), D, ptr(e), D, K, ptr(en), ptr(f32), ptr(ws), nws),
          "argmin")
    got = out["one"].cpu().long()
    xd, ed = x.cpu().double(), e.cpu().double()
    d = (xd ** 2).sum(1, keepdim=True) + (ed ** 2).sum(1) - 2 * xd @ ed.t()
    srt, order = torch.sort(d, dim=1, stable=True)
    ok = (srt[:, 1] - srt[:, 0]) > 1e-3
    assert ok.float().mean() > 0.3
    assert torch.equal(got[ok], order[ok, 0])
    assert torch.equal(got[ok], f32.cpu().long()[ok])
    assert not (got == K // 2).any()
    x[P // 2, D // 2] = 40000.0
    check(lib().idf_vq_argmin_x3_ws(s, P, D, ptr(x), D, ptr(ex), D, ys, K, ptr(en),
                                    ptr(out["one"]), None, 0, ptr(flag)), "argmin x3")
    assert int(flag.item()) == 1


@pytest.mark.parametrize("P,K,D", [(5, 1, 8), (130, 17, 12), (64, 129, 4)])
def test_vq_argmin_x3_small_codebooks(P, K, D):
    """The split-f16 search on codebooks smaller than one 128-code tile (and one past it): one
    code gives index 0 everywhere; otherwise the index equals the fp32 kernel's wherever a
    float64 search separates the best two codes by > 1e-3."""
    from idfcodec import _lib, vq
    from idfcodec._lib import check, lib, ptr
    g = torch.Generator().manual_seed(P * K)
    x = torch.tanh(torch.randn(P, D, generator=g)).cuda()
    e = torch.randn(K, D, generator=g) * 0.5
    ex, ys = vq.taps_weights_x3(e.double().numpy().reshape(K, 1, D))
    ex = torch.from_numpy(ex.reshape(-1)).cuda()
    e = e.cuda()
    s = _lib.stream_ptr()
    en = torch.empty(K, device="cuda")
    check(lib().idf_vq_norms(s, K, D, ptr(e), D, ptr(en)), "norms")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    nws = int(lib().idf_vq_argmin_workspace_bytes(P, K))
    ws = torch.empty(max(nws, 1), dtype=torch.uint8, device="cuda")
    got = torch.empty(P, dtype=torch.int32, device="cuda")
    check(lib().idf_vq_argmin_x3_ws(s, P, D, ptr(x), D, ptr(ex), D, ys, K, ptr(en), ptr(got),
                                    ptr(ws), nws, ptr(flag)), "argmin x3")
    f32 = torch.empty(P, dtype=torch.int32, device="cuda")
    check(lib().idf_vq_argmin_ws(s, P, D, ptr(x), D, ptr(e), D, K, ptr(en), ptr(f32), ptr(ws), nws),
          "argmin")
    assert int(flag.item()) == 0
    got, f32 = got.cpu().long(), f32.cpu().long()
    if K == 1:
        assert torch.all(got == 0)
        return
    xd, ed = x.cpu().double(), e.cpu().double()
    d = (xd ** 2).sum(1, keepdim=True) + (ed ** 2).sum(1) - 2 * xd @ ed.t()
    srt, order = torch.sort(d, dim=1, stable=True)
    ok = (srt[:, 1] - srt[:, 0]) > 1e-3
    assert torch.equal(got[ok], order[ok, 0]) and torch.equal(got[ok], f32[ok])


def test_vq_engine_argmin_modes_agree():
    """VQEngine's split-f16 codebook search (argmin_mode "x3", the default) and the fp32 one give
    the same indices on the reference's encoder data wherever its margin exceeds 1e-4."""
    m, z = model_for("vq_t1_3down")
    eng = m.engine()
    data = torch.from_numpy(z["data"]).cuda()
    got = {}
    for mode in ("x3", "f32"):
        eng.argmin_mode = mode
        got[mode] = m.indices(data).cpu().numpy()
    eng.argmin_mode = "x3"
    ok = z["d_margin"].reshape(got["x3"].shape) > 1e-4
    assert np.array_equal(got["x3"][ok], got["f32"][ok])
    assert np.array_equal(got["x3"][ok], z["idx"][ok])


@pytest.mark.parametrize("kind,ci,co,H,W", [("conv4s2", 3, 128, 64, 64), ("conv4s2", 128, 256, 32, 32),
                                            ("conv3", 40, 24, 9, 7), ("conv1", 384, 512, 8, 8),
                                            ("convT", 384, 256, 8, 8), ("convT", 256, 3, 16, 16),
                                            ("conv1", 16, 24, 5, 5), ("conv1", 20, 8, 3, 3),
                                            ("conv4s2", 20, 36, 10, 10)])
def test_conv_taps_x3_vs_fp64(kind, ci, co, H, W):
    """idf_conv_taps_x3 (split-f16 products on f16 MFMA) against a float64 conv of the same
    fp32 inputs and weights: within 1e-5 of the output scale and at most 4x the exact-f32
    kernel's own error; the strided, 3x3, 1x1 and transposed (four parity launches) forms, and
    k-loops of 1, 2 and 32 chunks (shorter than, and ragged against, the kernel's three chunks
    in flight); an input past the f16 pairs' range sets the flag."""
    import torch.nn.functional as F
    from idfcodec import _lib, vq
    from idfcodec._lib import check, ptr
    from idfcodec.packing import round_up
    g = torch.Generator().manual_seed(ci * 7 + co)
    B = 3
    x = torch.randn(B, ci, H, W, generator=g, dtype=torch.float64)
    x32 = x.float()  # the kernels see fp32 operands; so does the float64 reference
    if kind == "convT":
        w = (torch.randn(ci, co, 4, 4, generator=g, dtype=torch.float64) * 0.05).float()
        ref = F.conv_transpose2d(x32.double(), w.double(), stride=2, padding=1)
        convs = vq.pack_convT(w.double().numpy(), None)
    else:
        k, st, pd = {"conv4s2": (4, 2, 1), "conv3": (3, 1, 1), "conv1": (1, 1, 0)}[kind]
        w = (torch.randn(co, ci, k, k, generator=g, dtype=torch.float64) * 0.05).float()
        ref = F.conv2d(x32.double(), w.double(), stride=st, padding=pd)
        convs = [vq.pack_conv(w.double().numpy(), None, stride=st, padding=pd)]
    Ho, Wo = ref.shape[2], ref.shape[3]
    ldx = round_up(ci, 4)
    xp = torch.zeros(B, H, W, ldx)
    xp[..., :ci] = x32.permute(0, 2, 3, 1)
    xp = xp.cuda().contiguous()
    ldo = round_up(co, 4)
    L = _lib.lib()
    outs = {}
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    for mode in ("x3", "f32"):
        out = torch.zeros(B * Ho * Wo * ldo, device="cuda")
        for c in convs:
            dc = vq.DevConv(c, "cuda", wino=False)  # the fp32 tap weights and bias
            wt, ys = vq.taps_weights_x3(c.w)        # (a 3x3 conv's engine path is Winograd)
            wt = torch.from_numpy(wt.view(np.int16)).cuda()
            Hc, Wc = (H, W) if c.osy == 2 else (Ho, Wo)
            args = (_lib.stream_ptr(), B, H, W, ldx, ptr(xp), ldx, Hc, Wc, c.isy, c.isy, len(c.dy),
                    dc.dy, dc.dx)
            tail = (ptr(out), ldo, Ho, Wo, c.osy, c.osy, c.oy0, c.ox0, None, 0, 3, 0.0)
            if mode == "x3":
                check(L.idf_conv_taps_x3(*args, ptr(wt), c.ldw, c.n_alloc, ys, ptr(dc.b), co,
                                         *tail, ptr(flag)), "taps x3")
            else:
                check(L.idf_conv_taps_f32(*args, ptr(dc.w), c.ldw, c.n_alloc, ptr(dc.b), co, *tail),
                      "taps f32")
        outs[mode] = out.view(B, Ho, Wo, ldo)[..., :co].permute(0, 3, 1, 2).double().cpu()
    assert int(flag.item()) == 0
    scale = ref.abs().max().item()
    e3 = (outs["x3"] - ref).abs().max().item() / scale
    e32 = (outs["f32"] - ref).abs().max().item() / scale
    print(f"{kind} {ci}->{co}: split-f16 {e3:.2e}, f32 {e32:.2e}")
    assert e3 < 1e-5 and e3 <= 4 * e32 + 1e-7, (e3, e32)
    # past the f16 pairs' range: flagged
    xp[0, 0, 0, 0] = 1e5
    c = convs[0]
    dc = vq.DevConv(c, "cuda", wino=False)
    wt, ys = vq.taps_weights_x3(c.w)
    wt = torch.from_numpy(wt.view(np.int16)).cuda()
    Hc, Wc = (H, W) if c.osy == 2 else (Ho, Wo)
    out = torch.zeros(B * Ho * Wo * ldo, device="cuda")
    check(L.idf_conv_taps_x3(_lib.stream_ptr(), B, H, W, ldx, ptr(xp), ldx, Hc, Wc, c.isy, c.isy,
                             len(c.dy), dc.dy, dc.dx, ptr(wt), c.ldw, c.n_alloc,
                             ys, ptr(dc.b), co, ptr(out), ldo, Ho, Wo, c.osy, c.osy,
                             c.oy0, c.ox0, None, 0, 3, 0.0, ptr(flag)), "taps x3")
    assert int(flag.item()) == 1
