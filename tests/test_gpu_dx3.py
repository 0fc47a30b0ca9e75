"""GPU parity of the split-f16 direct conv (idf_conv3x3_dx3, conv3_dx3.hip) against fp64 conv2d
with the same folded weights: the 1e-5 bound of the flow contract, fp32-class error (within a
small factor of the exact-f32 Winograd kernel's own), the range guard, data far from unit scale,
and determinism (the same bits for an image coded alone or inside a batch)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def scaled_err(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs() / b.abs().clamp(min=1.0)).max().item()


def round_up_16(v):
    return (v + 15) // 16 * 16


def make_case(B, H, W, C, N, fold, scale=1.0, spike=None, seed=None):
    from idfcodec.packing import round_up
    g = torch.Generator().manual_seed(seed if seed is not None else B * 7 + H * 3 + C)
    ld = round_up(C + N, 16) + 4
    X = torch.randn(B * H * W, ld, generator=g) * scale
    if spike is not None:
        X[B * H * W // 2, 0] = spike
    ldw = round_up(C, 16)
    n_alloc = round_up(N, 16)
    Wt = torch.randn(n_alloc, 9, ldw, generator=g, dtype=torch.float64) / np.sqrt(9 * C)
    Wt[N:] = 0.0
    b3 = torch.randn(n_alloc, generator=g) * 0.1
    vt = torch.randn(9, n_alloc, generator=g) * 0.1 if fold else None
    bfull = None
    if fold:
        s = b3.clone()
        for t in range(9):
            s = s + vt[t]
        bfull = s
    return dict(B=B, H=H, W=W, C=C, N=N, ld=ld, X=X, Wt=Wt, b3=b3, vt=vt, bfull=bfull,
                n_alloc=n_alloc, ldw=ldw)


F16_NAN = 0x7E00  # poison for the split buffer: every slot a layer reads must be written first


def split_np(v):
    """The kernels' split of fp32 values: (f16(v), f16(v - f16(v))), as uint16 bits."""
    v = np.asarray(v, np.float32)
    h = v.astype(np.float16)
    lo = (v - h.astype(np.float32)).astype(np.float16)
    return h.view(np.uint16), lo.view(np.uint16)


def xs_channels(xs, P, nslab, c0, c1):
    """(hi, lo) uint16 [P, c1 - c0] of the split buffer [nslab][2][P][16]."""
    a = xs.view(nslab, 2, P, 16).permute(2, 0, 3, 1).reshape(P, nslab * 16, 2)
    a = a[:, c0:c1].numpy().view(np.uint16)
    return a[..., 0], a[..., 1]


def dx3_workspace(B, H, W, C, N, dev):
    """(zeroed workspace, bytes, counter bytes) for idf_conv3x3_dx3 (None, 0, 0 when the
    geometry does not split K)."""
    from idfcodec._lib import lib
    n = int(lib().idf_conv3x3_dx3_workspace(B, H, W, C, N))
    assert n >= 0
    if n == 0:
        return None, 0, 0
    ctr = int(lib().idf_conv3x3_dx3_counter_bytes(B, H, W, N))
    assert 0 < ctr < n and ctr % 256 == 0
    return torch.zeros(n // 4, dtype=torch.int32, device=dev), n, ctr


def run_dx3(cs, act, X=None, B=None, layer2=False):
    """split_cols of the input, then one dx3 layer (or two: the second reads the first's split
    outputs).  Returns (out, flag, xs, P, nslab_xs[, X after layer 1])."""
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    from idfcodec.packing import dx3_groups, dx3_weights
    B = cs["B"] if B is None else B
    X = (cs["X"] if X is None else X).clone()
    H, W, C, N, ld, n_alloc = cs["H"], cs["W"], cs["C"], cs["N"], cs["ld"], cs["n_alloc"]
    assert lib().idf_conv3x3_dx3_supported(H, W, N) == 1
    P = B * H * W
    dev = torch.device("cuda")
    nf, ngroup = dx3_groups(n_alloc)
    nft = nf * ngroup
    Wd, ysc = dx3_weights(cs["Wt"].numpy(), C)
    Wdd = torch.from_numpy(Wd.view(np.int16)).to(dev)
    Xd, b3d = X.to(dev), cs["b3"].to(dev)
    vtd = cs["vt"].to(dev) if cs["vt"] is not None else None
    bfd = cs["bfull"].to(dev) if cs["bfull"] is not None else None
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.zeros(P, ld, device=dev)
    c_top = C + N + (N if layer2 else 0)
    nslab = (c_top + 15) // 16
    xs = torch.full((nslab * 2 * P * 16,), F16_NAN, dtype=torch.int16, device=dev)
    assert lib().idf_dx3_split_bytes(P, nslab * 16) == xs.numel() * 2
    ws, wsb, ctr = dx3_workspace(B, H, W, C + (N if layer2 else 0), N, dev)
    s = _lib.stream_ptr()
    check(lib().idf_dx3_split_cols(s, P, 0, C, ptr(Xd), ld, ptr(xs), nslab, ptr(flag), None, 0),
          "split")

    def counters_zero():  # every launch leaves the split-K tile counters zero
        if ws is not None:
            torch.cuda.synchronize()
            assert not ws[:ctr // 4].any(), "dx3 left a split-K counter non-zero"

    if not layer2:
        check(lib().idf_conv3x3_dx3(s, B, H, W, C, ptr(xs), nslab, ptr(Wdd), nft, ysc,
                                    ptr(b3d), ptr(vtd), n_alloc, ptr(bfd), N, ptr(out), ld,
                                    _lib.ACT[act], 0.01, ptr(flag), ptr(ws), wsb, None), "dx3")
        torch.cuda.synchronize()
        counters_zero()
        return out.cpu(), int(flag.item()), xs.cpu(), P, nslab
    # layer 1 writes its fp32 outputs into X[:, C:C+N] and the split ones into xs
    check(lib().idf_conv3x3_dx3(s, B, H, W, C, ptr(xs), nslab, ptr(Wdd), nft, ysc,
                                ptr(b3d), ptr(vtd), n_alloc, ptr(bfd), N, ptr(Xd) + 4 * C, ld,
                                _lib.ACT[act], 0.01, ptr(flag), ptr(ws), wsb, None), "dx3 layer 1")
    counters_zero()
    C2 = C + N
    W2 = torch.from_numpy(np.random.default_rng(C2).normal(0, 1 / np.sqrt(9 * C2), (n_alloc, 9, C2)))
    W2[N:] = 0.0
    Wd2, ysc2 = dx3_weights(W2.numpy(), C2)
    Wdd2 = torch.from_numpy(Wd2.view(np.int16)).to(dev)
    check(lib().idf_conv3x3_dx3(s, B, H, W, C2, ptr(xs), nslab, ptr(Wdd2), nft, ysc2,
                                ptr(b3d), ptr(vtd), n_alloc, ptr(bfd), N, ptr(out), ld,
                                _lib.ACT[act], 0.01, ptr(flag), ptr(ws), wsb, None), "dx3 layer 2")
    torch.cuda.synchronize()
    counters_zero()
    return out.cpu(), int(flag.item()), xs.cpu(), P, nslab, Xd.cpu(), W2


def run_wino_f32(cs, act):
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    from idfcodec.packing import wino_weights
    B, H, W, C, N, ld, n_alloc = (cs[k] for k in ("B", "H", "W", "C", "N", "ld", "n_alloc"))
    dev = torch.device("cuda")
    U = torch.from_numpy(wino_weights(cs["Wt"].numpy(), cs["ldw"] // 16)).to(dev)
    vtd = cs["vt"].to(dev) if cs["vt"] is not None else None
    bfd = cs["bfull"].to(dev) if cs["bfull"] is not None else None
    wsn = lib().idf_conv3x3_wino_workspace(B, H, W, C, N)
    ws = torch.empty(max(wsn, 1), device=dev)
    out = torch.zeros(B * H * W, ld, device=dev)
    check(lib().idf_conv3x3_wino(_lib.stream_ptr(), B, H, W, C, ptr(cs["X"].to(dev)), ld, ptr(U),
                                 n_alloc // 16, ptr(cs["b3"].to(dev)), ptr(vtd), n_alloc, ptr(bfd), N,
                                 ptr(out), ld, _lib.ACT[act], 0.01, ptr(ws), wsn), "wino")
    torch.cuda.synchronize()
    return out.cpu()


def reference(cs, act):
    B, H, W, C, N = cs["B"], cs["H"], cs["W"], cs["C"], cs["N"]
    x4 = cs["X"][:, :C].double().view(B, H, W, C).permute(0, 3, 1, 2)
    w4 = cs["Wt"][:N, :, :C].permute(0, 2, 1).reshape(N, C, 3, 3)
    ref = F.conv2d(x4, w4, padding=1) + cs["b3"][:N].double().view(1, -1, 1, 1)
    if cs["vt"] is not None:
        mask = F.conv2d(torch.ones(1, 1, H, W, dtype=torch.float64),
                        torch.eye(9, dtype=torch.float64).view(9, 1, 3, 3), padding=1)
        ref = ref + torch.einsum("tn,bthw->bnhw", cs["vt"][:, :N].double(), mask)
    if act == "ReLU":
        return F.relu(ref)
    if act == "LeakyReLU":
        return F.leaky_relu(ref, 0.01)
    return ref


def got_nchw(out, cs):
    B, H, W, N = cs["B"], cs["H"], cs["W"], cs["N"]
    return out[:, :N].double().view(B, H, W, N).permute(0, 3, 1, 2)


@pytest.mark.parametrize("B,H,W,C,N,act,fold", [
    (3, 32, 32, 52, 44, "ReLU", True), (5, 16, 16, 100, 44, "ReLU", True),
    (3, 32, 32, 496, 44, "ReLU", True), (1, 16, 16, 520, 44, "ReLU", True),
    (2, 64, 64, 8, 16, "LeakyReLU", True), (2, 20, 32, 24, 32, "ReLU", True),
    (2, 16, 48, 12, 43, "LeakyReLU", True), (1, 5, 16, 40, 44, "ReLU", True),
    (4, 16, 16, 36, 12, "ReLU", False), (2, 32, 32, 100, 48, "LeakyReLU", True),
    (3, 17, 16, 20, 44, "None", True),
    # packed tiles: 8x8 images 2x2 to a tile with K split in 4 chunks (imagenet64's 8x8
    # level: a partial last band, 1 slab a chunk, 9 slabs a chunk), one group of 1 fragment
    (5, 8, 8, 36, 44, "ReLU", True), (6, 8, 8, 520, 44, "ReLU", True),
    (4, 8, 8, 52, 44, "ReLU", True), (2, 8, 8, 12, 16, "LeakyReLU", True),
    # 4x4 images 4x4 to a tile (config 4's first level): 64 outputs (4 fragments), 128 (two
    # groups of 4), a partial band
    (3, 4, 4, 100, 64, "ReLU", True), (2, 4, 4, 36, 128, "ReLU", True),
    (17, 4, 4, 20, 64, "ReLU", True),
    # gutter packing (images at pitch W + 1 / H + 1, the zero column / row between two images
    # shared): 27x23 (config 5's patches, 2 x 4 a band), 24- and 40-wide, 2x2 (config 4's
    # second level: 16 x 16 a band, 128 outputs), 7x7, 12x12, 8-wide with 4 rows (its segment
    # canvas would not fit); 8-wide segments with rows that do not pack
    (3, 27, 23, 40, 32, "LeakyReLU", True), (2, 8, 24, 20, 44, "ReLU", True),
    (1, 8, 40, 20, 44, "ReLU", True), (37, 2, 2, 24, 128, "ReLU", True),
    (5, 7, 7, 20, 44, "ReLU", True), (3, 12, 12, 36, 44, "LeakyReLU", True),
    (6, 4, 8, 40, 44, "ReLU", True), (2, 5, 8, 24, 44, "ReLU", True),
    (2, 16, 8, 24, 44, "ReLU", True),
    # 2-wide images with every lane on an image column (xskip): config 4's 2x2 level at 64
    # outputs, a batch over one 16 x 16 band (partial second band), odd heights, one row
    (5, 2, 2, 100, 64, "ReLU", True), (300, 2, 2, 36, 44, "LeakyReLU", True),
    (3, 5, 2, 20, 44, "ReLU", True), (4, 1, 2, 12, 16, "ReLU", True),
    (9, 2, 2, 20, 12, "None", False)])
def test_dx3_vs_fp64(B, H, W, C, N, act, fold):
    cs = make_case(B, H, W, C, N, fold)
    out, flag, xs, P, nslab = run_dx3(cs, act)
    ref = reference(cs, act)
    e = scaled_err(got_nchw(out, cs), ref)
    e32 = scaled_err(got_nchw(run_wino_f32(cs, act), cs), ref)
    print(f"dx3 {e:.2e} f32-wino {e32:.2e}")
    assert flag == 0
    assert torch.all(out[:, N:] == 0), "wrote outside the N output columns"
    assert e <= 1e-5, f"dx3 max scaled error {e:.3e}"
    assert e <= max(4 * e32, 1e-6), (e32, e)
    # the split copy: the block input as split, the layer's outputs as split, zeros after them
    # up to the next multiple of 16 channels, nothing past it touched
    hi, lo = xs_channels(xs, P, nslab, 0, C)
    h_ref, l_ref = split_np(cs["X"][:, :C].numpy())
    assert np.array_equal(hi, h_ref) and np.array_equal(lo, l_ref)
    zend = (C + N + 15) // 16 * 16
    hi, lo = xs_channels(xs, P, nslab, C, zend)
    vals = np.zeros((P, zend - C), np.float32)
    vals[:, :N] = out[:, :N].numpy()
    h_ref, l_ref = split_np(vals)
    assert np.array_equal(hi, h_ref) and np.array_equal(lo, l_ref)
    if nslab * 16 > zend:
        hi, _ = xs_channels(xs, P, nslab, zend, nslab * 16)
        assert (hi == F16_NAN).all()


@pytest.mark.parametrize("B,H,W,C,act", [(2, 32, 32, 52, "ReLU"), (3, 16, 16, 100, "LeakyReLU"),
                                         (1, 16, 32, 496, "ReLU"), (2, 9, 16, 8, "ReLU"),
                                         (6, 8, 8, 100, "ReLU"), (5, 4, 4, 36, "ReLU"),
                                         (3, 27, 23, 24, "LeakyReLU"), (40, 2, 2, 20, "ReLU")])
def test_dx3_two_layers_through_the_split_copy(B, H, W, C, act):
    """Layer 2 reads layer 1's split outputs (the producer side of the split copy): equal, within
    the 1e-5 contract, to an fp64 conv of layer 1's fp32 outputs."""
    N = 44
    cs = make_case(B, H, W, C, N, True, seed=C + 7)
    cs["ld"] = round_up_16(C + 2 * N) + 4
    cs["X"] = torch.randn(B * H * W, cs["ld"], generator=torch.Generator().manual_seed(3))
    out, flag, xs, P, nslab, X1, W2 = run_dx3(cs, act, layer2=True)
    assert flag == 0
    cs2 = dict(cs, C=C + N, X=X1, Wt=W2, ldw=W2.shape[2])
    ref = reference(cs2, act)
    e = scaled_err(got_nchw(out, cs2), ref)
    print(f"dx3 two layers {e:.2e}")
    assert e <= 1e-5
    # and layer 1's fp32 outputs are what a single layer produces
    out1, _, _, _, _ = run_dx3(cs, act)
    assert torch.equal(X1[:, C:C + N], out1[:, :N])


@pytest.mark.parametrize("scale", [1e-3, 30.0])
def test_dx3_far_from_unit_scale(scale):
    cs = make_case(2, 16, 16, 200, 44, True, scale=scale)
    out, flag = run_dx3(cs, "ReLU")[:2]
    ref = reference(cs, "ReLU")
    e = scaled_err(got_nchw(out, cs), ref)
    e32 = scaled_err(got_nchw(run_wino_f32(cs, "ReLU"), cs), ref)
    assert flag == 0
    assert e <= max(4 * e32, 1e-6), (e32, e)


def test_dx3_batch_invariant():
    """An image's outputs are the same bits alone and inside a batch (the decoder recomputes
    the encoder's couplings on other batch compositions) -- here also across the two block
    shapes: B = 130 (520 16x16 tiles) runs two tiles per block, B = 1 one."""
    cs = make_case(130, 32, 32, 140, 44, True, seed=11)
    full = run_dx3(cs, "ReLU")[0]
    P = 32 * 32
    for i in (3, 129):
        one = cs["X"][i * P: (i + 1) * P].clone()
        alone = run_dx3(cs, "ReLU", X=one, B=1)[0]
        assert torch.equal(full[i * P: (i + 1) * P], alone)


def test_dx3_range_guard_sets_flag():
    """The block input's split (idf_dx3_split_cols) flags NaN and |x| >= 32768."""
    for spike, want in ((40000.0, 1), (float("nan"), 1), (1000.0, 0)):
        cs = make_case(1, 16, 16, 16, 16, True, spike=spike)
        flag = run_dx3(cs, "ReLU")[1]
        assert flag == want, (spike, flag)


def test_dx3_output_guard_sets_flag():
    cs = make_case(1, 16, 16, 16, 16, True, scale=4000.0)
    assert run_dx3(cs, "None")[1] == 1
    cs = make_case(1, 16, 16, 16, 16, True, scale=100.0)
    assert run_dx3(cs, "None")[1] == 0


def test_dx3_supported_geometry():
    """The tilings (16-wide tiles, packed segments, gutter packing) cover every image geometry:
    imagenet64's three levels and configs 4/5's; only more than 1024 outputs are refused."""
    from idfcodec._lib import lib
    L = lib()
    for H, W, N in ((32, 32, 44), (16, 16, 44), (8, 8, 44), (27, 23, 32), (16, 16, 64),
                    (4, 4, 64), (4, 4, 128), (8, 40, 44), (5, 8, 44), (2, 2, 64), (2, 2, 128),
                    (8, 12, 44), (4, 8, 44), (7, 7, 44), (2, 4, 64), (1, 1, 16), (64, 64, 1024)):
        assert L.idf_conv3x3_dx3_supported(H, W, N) == 1, (H, W, N)
    for H, W, N in ((8, 8, 1025), (0, 8, 44), (8, 8, 0)):
        assert L.idf_conv3x3_dx3_supported(H, W, N) == 0, (H, W, N)
    # split K only where the tiles are few for any batch: the 8x8 level
    assert L.idf_conv3x3_dx3_workspace(256, 8, 8, 520, 44) > 0
    assert L.idf_conv3x3_dx3_workspace(256, 8, 8, 12, 44) == 0  # one slab: nothing to split
    assert L.idf_conv3x3_dx3_workspace(256, 16, 16, 520, 44) == 0
    assert L.idf_conv3x3_dx3_workspace(256, 4, 4, 520, 64) == 0


def test_dx3_split_k_batch_invariant():
    """8x8 images (split K, 2x2 images a tile): an image's outputs are the same bits alone, in
    another tile position and inside a batch -- the chunks are summed in chunk order whichever
    block finishes last."""
    cs = make_case(9, 8, 8, 300, 44, True, seed=5)
    full = run_dx3(cs, "ReLU")[0]
    again = run_dx3(cs, "ReLU")[0]
    assert torch.equal(full, again)
    P = 64
    for i in (0, 3, 8):
        one = cs["X"][i * P: (i + 1) * P].clone()
        alone = run_dx3(cs, "ReLU", X=one, B=1)[0]
        assert torch.equal(full[i * P: (i + 1) * P], alone), i
    # two images: the second at tile position 1 (top right) instead of i % 4
    two = cs["X"][7 * P: 9 * P].clone()
    pair = run_dx3(cs, "ReLU", X=two, B=2)[0]
    assert torch.equal(full[7 * P: 9 * P], pair)


def test_dx3_packed_batch_invariant():
    """4x4 images (16 a tile, segments), 27x23 and 2x2 images (gutter packing): outputs are the
    same bits at any position in any batch."""
    for B, H, W, C, N in ((21, 4, 4, 60, 64), (19, 27, 23, 40, 32), (300, 2, 2, 24, 128)):
        cs = make_case(B, H, W, C, N, True, seed=B)
        full = run_dx3(cs, "LeakyReLU")[0]
        P = H * W
        for i in (0, 5, B - 1):
            one = cs["X"][i * P: (i + 1) * P].clone()
            alone = run_dx3(cs, "LeakyReLU", X=one, B=1)[0]
            assert torch.equal(full[i * P: (i + 1) * P], alone), (H, W, i)


@pytest.mark.parametrize("B,H,W,nh,N", [(2, 32, 32, 3, 44), (3, 16, 16, 12, 44), (5, 8, 8, 16, 44),
                                        (3, 27, 23, 6, 44), (40, 2, 2, 12, 44), (37, 4, 4, 6, 64),
                                        (150, 2, 2, 12, 64), (9, 27, 23, 6, 64)])
def test_dx3_fused_head(B, H, W, nh, N):
    """The DenseBlock head fused into two dx3 layers (IdfDx3Head): running sums from the block
    input (idf_dx3_head_init), each layer's share, the last layer's epilogue -- STORE within 1e-5
    of an fp64 head over the kernels' own features; the fp32 stores skipped without changing a
    bit; COUPLE_ADD / COUPLE_SUB exact inverses that round the same sums; PRIOR = the sums as
    NCHW mean / logscale and exp(logscale); an image's head the same bits alone or inside a
    batch (the decoder runs other batch compositions than the encoder)."""
    from idfcodec import _lib
    from idfcodec._lib import IdfDx3Head, check, lib, ptr
    from idfcodec.packing import dx3_groups, dx3_weights
    import ctypes
    dev = torch.device("cuda")
    g = torch.Generator().manual_seed(B * 31 + nh)
    C0 = 20
    C1, C2 = C0 + N, C0 + 2 * N
    P = B * H * W
    n_alloc = (N + 15) // 16 * 16
    nf, ngroup = dx3_groups(n_alloc)
    ld = (C2 + 15) // 16 * 16 + 16
    X = torch.zeros(P, ld)
    X[:, :C0] = torch.randn(P, C0, generator=g)
    Xd = X.to(dev)
    Ws = [torch.randn(n_alloc, 9, (c + 15) // 16 * 16, generator=g, dtype=torch.float64) / np.sqrt(9 * c)
          for c in (C0, C1)]
    for w, c in zip(Ws, (C0, C1)):
        w[N:] = 0.0
        w[:, :, c:] = 0.0
    packs = [dx3_weights(w.numpy(), c) for w, c in zip(Ws, (C0, C1))]
    wdev = [torch.from_numpy(wd.view(np.int16)).to(dev) for wd, _ in packs]
    b3 = (torch.randn(n_alloc, generator=g) * 0.1).to(dev)
    ldwh = (C2 + 15) // 16 * 16
    wh = torch.zeros(nh, ldwh)
    wh[:, :C2] = torch.randn(nh, C2, generator=g) / np.sqrt(C2)
    bh = torch.randn(nh, generator=g) * 0.1
    whd, bhd = wh.to(dev), bh.to(dev)
    nslab = (C2 + 15) // 16
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    s = _lib.stream_ptr()

    def run(mode, skip_f32, base=None, n_mean=0, img=None):
        B_, X_ = (B, Xd) if img is None else (1, Xd[img * H * W:(img + 1) * H * W])
        return run_b(B_, X_, mode, skip_f32, base, n_mean)

    def run_b(B, Xd, mode, skip_f32, base, n_mean):
        P = B * H * W
        xs = torch.full((nslab * 2 * P * 16,), F16_NAN, dtype=torch.int16, device=dev)
        ws, wsb, ctr = dx3_workspace(B, H, W, C1, N, dev)
        acc = torch.empty(P * 16, device=dev)
        feat = Xd.clone()
        if skip_f32:
            feat[:, C0:] = float("nan")  # never written when the fp32 stores are skipped
        check(lib().idf_dx3_split_cols(s, P, 0, C0, ptr(feat), ld, ptr(xs), nslab, ptr(flag),
                                       ptr(ws) if ws is not None else None,
                                       ctr // 4 if ws is not None else 0), "split")
        check(lib().idf_dx3_head_init(s, P, C0, ptr(feat), ld, ptr(whd), ldwh, ptr(bhd), nh,
                                      ptr(acc)), "head init")
        out = torch.zeros(P, 16, device=dev)
        mean = torch.zeros(B * (nh // 2) * H * W, device=dev)
        logs, scale = torch.zeros_like(mean), torch.zeros_like(mean)
        for i, c in enumerate((C0, C1)):
            hd = IdfDx3Head()
            hd.w, hd.ldw, hd.n_head, hd.acc = ptr(whd), ldwh, nh, ptr(acc)
            hd.last, hd.skip_f32 = int(i == 1), int(skip_f32)
            hd.out.mode = mode
            hd.out.out, hd.out.ld_out = ptr(out), 16
            if base is not None:
                hd.out.base, hd.out.ld_base = ptr(base), 16
            hd.out.n_mean = n_mean
            hd.out.mean, hd.out.logscale, hd.out.scale = ptr(mean), ptr(logs), ptr(scale)
            check(lib().idf_conv3x3_dx3(s, B, H, W, c, ptr(xs), nslab, ptr(wdev[i]),
                                        nf * ngroup, packs[i][1], ptr(b3), None, n_alloc, None, N,
                                        ptr(feat) + 4 * c, ld, _lib.ACT["ReLU"], 0.01, ptr(flag),
                                        ptr(ws), wsb, ctypes.byref(hd)), "dx3")
        torch.cuda.synchronize()
        return out.cpu(), feat.cpu(), (mean.cpu(), logs.cpu(), scale.cpu())

    out, feat, _ = run(_lib.EPI_STORE, False)
    ref = feat[:, :C2].double() @ wh[:, :C2].double().T + bh.double()
    e = scaled_err(out[:, :nh], ref)
    print(f"fused head {e:.2e}")
    assert e <= 1e-5, e
    assert not out[:, nh:].any()
    hw = H * W
    for i in sorted({0, B // 2, B - 1}):
        alone = run(_lib.EPI_STORE, True, img=i)[0]
        assert torch.equal(alone, out[i * hw:(i + 1) * hw]), ("batch", i)
    out2, feat2, _ = run(_lib.EPI_STORE, True)
    assert torch.equal(out2, out), "skipping the fp32 stores changed the head"
    assert torch.isnan(feat2[:, C0:C2]).all(), "fp32 outputs written with skip_f32"
    base = torch.round(torch.randn(P, 16, generator=g) * 256) / 256
    r8 = torch.round(out[:, :nh] * 256) / 256
    for mode, sign in ((_lib.EPI_COUPLE_ADD, 1), (_lib.EPI_COUPLE_SUB, -1)):
        o3, _, _ = run(mode, True, base=base.to(dev))
        assert torch.equal(o3[:, :nh], base[:, :nh] + sign * r8), mode
    if nh % 2 == 0:
        _, _, (mean, logs, scale) = run(_lib.EPI_PRIOR, True, n_mean=nh // 2)
        h = out[:, :nh].view(B, H, W, nh).permute(0, 3, 1, 2)
        assert torch.equal(mean.view(B, nh // 2, H, W), h[:, :nh // 2])
        assert torch.equal(logs.view(B, nh // 2, H, W), h[:, nh // 2:])
        assert torch.allclose(scale, torch.exp(logs), rtol=1e-6, atol=0)


def test_dx3_split_copy_over_2gib():
    """A split copy larger than 2 GiB (config 5's 2048-patch batches have 2.8 GB): the halo DMA
    addresses it a slab at a time; images at both ends of the batch equal the same images
    alone."""
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    from idfcodec.packing import dx3_groups, dx3_weights
    dev = torch.device("cuda")
    B, H, W, C, N = 4400, 16, 16, 496, 44
    P = B * H * W
    ld = 560
    nslab = (C + N + 15) // 16
    assert lib().idf_dx3_split_bytes(P, 16 * nslab) > 2 ** 31
    g = torch.Generator(device=dev).manual_seed(3)
    X = torch.randn(P, ld, generator=g, device=dev)
    gw = torch.Generator().manual_seed(4)
    Wt = torch.randn(48, 9, C, generator=gw, dtype=torch.float64) / np.sqrt(9 * C)
    Wt[N:] = 0.0
    nf, ngroup = dx3_groups(48)
    Wd, ysc = dx3_weights(Wt.numpy(), C)
    Wdd = torch.from_numpy(Wd.view(np.int16)).to(dev)
    b3 = (torch.randn(48, generator=gw) * 0.1).to(dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    s = _lib.stream_ptr()

    def run(Xin, Bn):
        Pn = Bn * H * W
        xs = torch.empty(nslab * 2 * Pn * 16, dtype=torch.int16, device=dev)
        out = torch.zeros(Pn, ld, device=dev)
        check(lib().idf_dx3_split_cols(s, Pn, 0, C, ptr(Xin), ld, ptr(xs), nslab, ptr(flag),
                                       None, 0), "split")
        check(lib().idf_conv3x3_dx3(s, Bn, H, W, C, ptr(xs), nslab, ptr(Wdd), nf * ngroup, ysc,
                                    ptr(b3), None, 48, None, N, ptr(out), ld, _lib.ACT["ReLU"],
                                    0.01, ptr(flag), None, 0, None), "dx3")
        torch.cuda.synchronize()
        del xs
        return out[:, :N]

    full = run(X, B)
    hw = H * W
    for i in (0, B - 1):
        one = run(X[i * hw:(i + 1) * hw].contiguous(), 1)
        assert torch.equal(full[i * hw:(i + 1) * hw], one), i
    assert full.abs().sum() > 0


@pytest.mark.parametrize("name,lvl,which", [
    ("imagenet64", 1, "coupling"), ("imagenet64", 1, "prior"),
    ("resflows_smallpatch_split", 0, "coupling"), ("resflow-cond-imagenet64", 1, "coupling"),
    ("resflow-cond-imagenet64", 1, "prior")])
def test_fused_block_kernel_bit_identical(name, lvl, which):
    """The fused DenseBlock launch (IdfDenseBlock.fuse_layers: every layer in one launch, one
    workgroup per tile, conv3_dx3_block_kernel) gives the per-layer launches' bits: the head's
    outputs (fused head: its register sums and epilogue; GEMM head: over the fp32 features the
    layers stored) and the fp32 features.  imagenet64's 16x16 level, config 4's 4x4 patches,
    config 3's bf16 (dxb) blocks."""
    from idfcodec import _lib, configs, synthetic
    from idfcodec._lib import IdfHeadOut, ptr
    model = synthetic.build_model(configs.get(name)).cuda()
    model.idf_precision = configs.PRECISION.get(name, "f32")
    eng = model.engine()
    Lv = eng.levels[lvl]
    blk = eng.couple[lvl][0] if which == "coupling" else eng.prior[lvl]
    bf = 1 if blk.desc.dxb else 0
    assert blk.desc.dx3 == 1 or blk.desc.dxb == 1
    assert _lib.lib().idf_dx3_block_supported(Lv.h, Lv.w, blk.geom.g_pad, bf) == 1
    B = 48 if Lv.h * Lv.w >= 64 else 200
    P = B * Lv.h * Lv.w
    k0 = blk.geom.k_in[0]
    nh = blk.geom.n_head
    ldo = (nh + 3) // 4 * 4
    g = torch.Generator().manual_seed(11)
    x = (torch.randint(-64, 64, (P, k0), generator=g).float() / 256).cuda()
    if which == "coupling":
        x[:, Lv.a:] = 0.0
    ws = eng.workspace(B, 1)
    res = []
    for fuse in (0, 1):
        blk.desc.fuse_layers = fuse
        feat = ws["feat"].view(-1, eng.ld_feat)
        feat.zero_()
        feat[:P, :k0] = x
        out = torch.zeros(P, ldo, device="cuda")
        h = IdfHeadOut()
        h.mode, h.out, h.ld_out = _lib.EPI_STORE, ptr(out), ldo
        blk.run(_lib.stream_ptr(), B, Lv.h, Lv.w, ptr(ws["feat"]), eng.ld_feat, ptr(ws["tmp"]),
                eng.tmp_pitch(ws, P), h)
        torch.cuda.synchronize()
        res.append((out.clone(), feat[:P, :blk.geom.k_in[-1]].clone()))
    blk.desc.fuse_layers = 1
    (o0, f0), (o1, f1) = res
    assert torch.isfinite(o0).all() and o0.abs().sum() > 0
    assert torch.equal(o0, o1), int((o0 != o1).any(1).sum())
    assert torch.equal(f0, f1), int((f0 != f1).any(1).sum())


@pytest.mark.parametrize("P,C0,nh,ld,nslab", [(262144, 8, 12, 544, 2), (16384, 28, 16, 96, 3),
                                               (1000, 64, 5, 64, 4), (77, 4, 1, 8, 1)])
def test_split_cols_head_one_launch_bit_identical(P, C0, nh, ld, nslab):
    """idf_dx3_split_cols_head (what a per-layer DenseBlock with a fused head runs before its
    first layer) writes the same split copy, range flag, cleared counters and head sums, bit for
    bit, as idf_dx3_split_cols + idf_dx3_head_init; a NaN input still sets the flag."""
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    g = torch.Generator().manual_seed(P + C0)
    x = (torch.randn(P, ld, generator=g) * 3).cuda()
    w = torch.randn(nh, 68, generator=g).cuda()
    b = torch.randn(nh, generator=g).cuda()
    s = _lib.stream_ptr()
    res = []
    for one in (False, True):
        xs = torch.full((nslab * 2 * P * 16,), 0x7E00, dtype=torch.int16, device="cuda")
        acc = torch.full((P, 16), float("nan"), device="cuda")
        flag = torch.zeros(1, dtype=torch.int32, device="cuda")
        zero = torch.full((37,), 7, dtype=torch.int32, device="cuda")
        if one:
            check(lib().idf_dx3_split_cols_head(s, P, C0, ptr(x), ld, ptr(xs), nslab, ptr(flag),
                                                ptr(zero), 37, ptr(w), 68, ptr(b), nh, ptr(acc)),
                  "split+head")
        else:
            check(lib().idf_dx3_split_cols(s, P, 0, C0, ptr(x), ld, ptr(xs), nslab, ptr(flag),
                                           ptr(zero), 37), "split")
            check(lib().idf_dx3_head_init(s, P, C0, ptr(x), ld, ptr(w), 68, ptr(b), nh, ptr(acc)),
                  "head init")
        torch.cuda.synchronize()
        res.append((xs.cpu(), acc.cpu(), int(flag.item()), zero.cpu()))
    (xa, aa, fa, za), (xb, ab, fb, zb) = res
    assert torch.equal(xa, xb)
    assert torch.equal(aa.view(torch.int32), ab.view(torch.int32))
    assert fa == fb == 0 and int(za.abs().sum()) == 0 and int(zb.abs().sum()) == 0
    ref = b.cpu().double() + x.cpu().double()[:, :C0] @ w.cpu().double()[:, :C0].t()
    assert (ab[:, :nh].double() - ref).abs().max() < 1e-4 * (1 + ref.abs().max())
    assert torch.all(ab[:, nh:] == 0)
    x[P // 2, C0 - 1] = float("nan")
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    check(lib().idf_dx3_split_cols_head(s, P, C0, ptr(x), ld, ptr(xs), nslab, ptr(flag), None, 0,
                                        ptr(w), 68, ptr(b), nh, ptr(acc)), "split+head")
    assert int(flag.item()) == 1
