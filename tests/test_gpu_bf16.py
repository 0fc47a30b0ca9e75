"""GPU parity of the bf16-MFMA DenseLayer conv (conv3_bf16.hip) against fp64 conv2d of the
bf16-rounded operands (products of bf16 values are exact in fp32; only the fp32
accumulation differs: 1e-5), its batch invariance (what makes the bf16 codec lossless), and
lossless round trips of the bf16 flow (BASELINE configs[2] names bf16 coupling convs)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _run(X, Wt, b3, vt, bfull, B, H, W, C, N, act="ReLU"):
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    from idfcodec.packing import bf16_weights, round_up
    ld = X.shape[1]
    n_alloc = round_up(N, 16)
    wb = torch.from_numpy(bf16_weights(Wt.numpy().astype(np.float32), C).view(np.int16)).cuda()
    dev = torch.device("cuda")
    Xd, b3d = X.to(dev), b3.to(dev)
    vtd = vt.to(dev) if vt is not None else None
    bfd = bfull.to(dev) if bfull is not None else None
    P = B * H * W
    out = torch.zeros(P, ld, device=dev)
    # bf16 shadow of the input columns (zeros to the next multiple of 8), output columns
    # at C (the DenseBlock layout), poisoned so unwritten shadow columns show up
    ld16 = round_up(C + N + 8, 8)
    x16 = torch.full((P, ld16), 0x7FC0, dtype=torch.int16, device=dev)
    check(lib().idf_f32_to_bf16_cols(_lib.stream_ptr(), P, C, round_up(C, 8), ptr(Xd), ld,
                                     ptr(x16), ld16), "to bf16")
    n16 = round_up(C + N, 8) - C
    wsn = lib().idf_conv3x3_bf16_workspace(B, H, W, C, N)
    ws = torch.empty(max(wsn, 1), device=dev)
    check(lib().idf_conv3x3_bf16(_lib.stream_ptr(), B, H, W, C, ptr(x16), ld16, ptr(wb), n_alloc,
                                 ptr(b3d), ptr(vtd), n_alloc, ptr(bfd), N, ptr(out), ld,
                                 ptr(x16) + 2 * C, ld16, n16, _lib.ACT[act], 0.01, ptr(ws), wsn),
          "bf16 conv")
    torch.cuda.synchronize()
    # the shadow holds bf16(out) for the N output columns and zeros up to n16
    sh = x16[:, C:C + n16].cpu()
    want = out[:, :N].cpu().to(torch.bfloat16).view(torch.int16)
    assert torch.equal(sh[:, :N], want), "bf16 shadow of the output differs"
    assert torch.all(sh[:, N:] == 0), "shadow pad columns not zeroed"
    assert torch.all(x16[:, C + n16:].cpu() == 0x7FC0), "wrote past the shadow columns"
    return out.cpu()


@pytest.mark.parametrize("B,H,W,C,N,fold", [
    (3, 32, 32, 52, 43, True), (5, 16, 16, 100, 43, True), (9, 8, 8, 168, 43, True),
    (2, 6, 10, 24, 20, False), (1, 16, 16, 520, 43, True)])
def test_conv3x3_bf16_vs_fp64(B, H, W, C, N, fold):
    g = torch.Generator().manual_seed(B * 5 + H + C)
    ld = ((C + N + 15) // 16) * 16 + 4
    X = torch.randn(B * H * W, ld, generator=g)
    n_alloc = ((N + 15) // 16) * 16
    ldw = ((C + 15) // 16) * 16
    Wt = torch.randn(n_alloc, 9, ldw, generator=g) / np.sqrt(9 * C)
    Wt[:, :, C:] = 0
    b3 = torch.randn(n_alloc, generator=g) * 0.1
    vt = torch.randn(9, n_alloc, generator=g) * 0.1 if fold else None
    bfull = None
    if fold:
        s = b3.clone()
        for t in range(9):
            s = s + vt[t]
        bfull = s
    out = _run(X, Wt, b3, vt, bfull, B, H, W, C, N)
    xr = X[:, :C].to(torch.bfloat16).double().view(B, H, W, C).permute(0, 3, 1, 2)
    wr = Wt[:N, :, :C].to(torch.bfloat16).double().permute(0, 2, 1).reshape(N, C, 3, 3)
    ref = F.conv2d(xr, wr, padding=1) + b3[:N].double().view(1, -1, 1, 1)
    if fold:
        mask = F.conv2d(torch.ones(1, 1, H, W, dtype=torch.float64),
                        torch.eye(9, dtype=torch.float64).view(9, 1, 3, 3), padding=1)
        ref = ref + torch.einsum("tn,bthw->bnhw", vt[:, :N].double(), mask)
    ref = F.relu(ref)
    got = out[:, :N].double().view(B, H, W, N).permute(0, 3, 1, 2)
    err = ((got - ref).abs() / ref.abs().clamp(min=1.0)).max().item()
    assert err <= 1e-5, err
    assert torch.all(out[:, N:] == 0)


def test_conv3x3_bf16_batch_invariant():
    g = torch.Generator().manual_seed(7)
    B, H, W, C, N = 6, 8, 8, 100, 43
    ld = 160
    X = torch.randn(B * H * W, ld, generator=g)
    Wt = torch.randn(48, 9, 112, generator=g) / 30
    b3 = torch.randn(48, generator=g) * 0.1
    full = _run(X, Wt, b3, None, None, B, H, W, C, N)
    one = _run(X[2 * 64: 3 * 64].contiguous(), Wt, b3, None, None, 1, H, W, C, N)
    assert torch.equal(full[2 * 64: 3 * 64], one)


def test_bf16_flow_round_trip_config3():
    """resflow-cond-imagenet64 with bf16 coupling convs (its BASELINE precision), B=2."""
    from idfcodec import synthetic
    codec, fl, vq, size = synthetic.build_residual("resflow-cond-imagenet64")
    assert fl.engine().precision == "bf16"
    x = synthetic.images(2, H=size[0], W=size[1], seed=8).cuda()
    out, info = codec.decode(codec.encode(x))
    assert info["ok"] and torch.equal(out, x)


@pytest.mark.parametrize("H,growth,depth", [(16, 24, 3), (8, 40, 2), (12, 120, 4)])
def test_bf16_small_flow_round_trip_and_batch_invariance(H, growth, depth):
    """Small bf16 flows (narrow DenseBlocks: the bf16 shadow + split-K partials share tmp;
    8x8 levels take the 2-way split): exact round trip, and an image coded alone gives the
    same streams as inside the batch."""
    from idfcodec import synthetic
    from idfcodec.configs import _dense, _flows
    cfg = _flows("IDFlows", 2, 2, H, H, 3, _dense(growth, depth), _dense(growth, depth), 2)
    model = synthetic.build_model(cfg).cuda()
    model.idf_precision = "bf16"
    assert model.engine().precision == "bf16"
    x = synthetic.images(3, H=H, W=H, seed=H + growth).cuda()
    codec = model.codec()
    bs = codec.encode(x)
    out, info = codec.decode(bs)
    assert info["ok"] and torch.equal(out, x)
    one = codec.encode(x[1:2].contiguous())
    L = len(bs.level_shapes)
    for l in range(L):
        assert int(one.states[l]) == int(bs.states[l * 3 + 1])


def _run_dxb(X, Wt, b3, vt, bfull, B, H, W, C, N, act="ReLU"):
    """idf_conv3x3_dxb (the bf16 direct conv) as a DenseBlock runs it: the slab-major bf16 copy
    (idf_dxb_cols: zeros from C to the next 16 channels) poisoned past the columns the layer
    may write, the split-K workspace zeroed."""
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    from idfcodec.packing import dxb_weights, round_up
    ld = X.shape[1]
    n_alloc = round_up(N, 16)
    wd = torch.from_numpy(dxb_weights(Wt.numpy().astype(np.float32), C).view(np.int16)).cuda()
    dev = torch.device("cuda")
    Xd, b3d = X.to(dev), b3.to(dev)
    vtd = vt.to(dev) if vt is not None else None
    bfd = bfull.to(dev) if bfull is not None else None
    P = B * H * W
    out = torch.zeros(P, ld, device=dev)
    z = round_up(C + N, 16)
    nslab = z // 16 + 1
    assert lib().idf_dxb_bytes(P, 16 * nslab) == nslab * P * 32
    xb = torch.full((nslab, P, 16), 0x7FC0, dtype=torch.int16, device=dev)
    check(lib().idf_dxb_cols(_lib.stream_ptr(), P, 0, C, ptr(Xd), ld, ptr(xb), nslab, None, 0),
          "to bf16")
    wsn = int(lib().idf_conv3x3_dx3_workspace(B, H, W, C, N))
    ws = torch.zeros(max(wsn, 256) // 4, dtype=torch.int32, device=dev)
    check(lib().idf_conv3x3_dxb(_lib.stream_ptr(), B, H, W, C, ptr(xb), nslab, ptr(wd),
                                n_alloc // 16, ptr(b3d), ptr(vtd), n_alloc, ptr(bfd), N, ptr(out),
                                ld, _lib.ACT[act], 0.01, ptr(ws), wsn, None), "dxb conv")
    torch.cuda.synchronize()
    if wsn:
        ctr = int(lib().idf_conv3x3_dx3_counter_bytes(B, H, W, N))
        assert not ws[:ctr // 4].any(), "dxb left a split-K counter non-zero"
    x16 = xb.permute(1, 0, 2).reshape(P, nslab * 16)  # pixel-major view of the slab-major copy
    xin = X[:, :C].to(torch.bfloat16).view(torch.int16)
    assert torch.equal(x16[:, :C].cpu(), xin), "bf16 copy of the input differs"
    sh = x16[:, C:z].cpu()
    want = out[:, :N].cpu().to(torch.bfloat16).view(torch.int16)
    assert torch.equal(sh[:, :N], want), "bf16 shadow of the output differs"
    assert torch.all(sh[:, N:] == 0), "shadow pad columns not zeroed"
    assert torch.all(x16[:, z:].cpu() == 0x7FC0), "wrote past the shadow columns"
    return out.cpu()


def _case(B, H, W, C, N, seed, fold=True):
    g = torch.Generator().manual_seed(seed)
    ld = ((C + N + 15) // 16) * 16 + 4
    X = torch.randn(B * H * W, ld, generator=g)
    n_alloc = ((N + 15) // 16) * 16
    ldw = ((C + 15) // 16) * 16
    Wt = torch.randn(n_alloc, 9, ldw, generator=g) / np.sqrt(9 * C)
    Wt[:, :, C:] = 0
    Wt[N:] = 0
    b3 = torch.randn(n_alloc, generator=g) * 0.1
    vt = torch.randn(9, n_alloc, generator=g) * 0.1 if fold else None
    bfull = None
    if fold:
        s = b3.clone()
        for t in range(9):
            s = s + vt[t]
        bfull = s
    return X, Wt, b3, vt, bfull


@pytest.mark.parametrize("B,H,W,C,N", [
    (3, 32, 32, 52, 43), (130, 32, 32, 100, 44), (5, 16, 16, 100, 43), (9, 8, 8, 168, 43),
    (4, 27, 23, 40, 32), (1, 16, 16, 520, 43), (2, 32, 32, 12, 16), (3, 8, 8, 20, 20)])
def test_conv3x3_dxb_vs_fp64(B, H, W, C, N):
    """The bf16 direct conv: every geometry it tiles (16-wide tiles one and two per block,
    gutter packing, the 8 x 8 segments with split K) within 1e-5 of fp64 over the bf16-rounded
    operands; the shadow holds bf16 of the fp32 outputs."""
    from idfcodec._lib import lib
    assert lib().idf_conv3x3_dxb_supported(H, W, N) == 1
    X, Wt, b3, vt, bfull = _case(B, H, W, C, N, B * 5 + H + C)
    out = _run_dxb(X, Wt, b3, vt, bfull, B, H, W, C, N)
    xr = X[:, :C].to(torch.bfloat16).double().view(B, H, W, C).permute(0, 3, 1, 2)
    wr = Wt[:N, :, :C].to(torch.bfloat16).double().permute(0, 2, 1).reshape(N, C, 3, 3)
    ref = F.conv2d(xr, wr, padding=1) + b3[:N].double().view(1, -1, 1, 1)
    mask = F.conv2d(torch.ones(1, 1, H, W, dtype=torch.float64),
                    torch.eye(9, dtype=torch.float64).view(9, 1, 3, 3), padding=1)
    ref = F.relu(ref + torch.einsum("tn,bthw->bnhw", vt[:, :N].double(), mask))
    got = out[:, :N].double().view(B, H, W, N).permute(0, 3, 1, 2)
    err = ((got - ref).abs() / ref.abs().clamp(min=1.0)).max().item()
    assert err <= 1e-5, err
    assert torch.all(out[:, N:] == 0)


@pytest.mark.parametrize("B,H,W,C,N", [(6, 8, 8, 100, 43), (130, 32, 32, 60, 44),
                                       (7, 27, 23, 40, 32)])
def test_conv3x3_dxb_batch_invariant(B, H, W, C, N):
    """An image's outputs are the same bits alone and inside a batch (split K at 8 x 8, two
    tiles per block at B = 130, gutter packing at 27 x 23)."""
    X, Wt, b3, vt, bfull = _case(B, H, W, C, N, 7 + B)
    full = _run_dxb(X, Wt, b3, vt, bfull, B, H, W, C, N)
    P = H * W
    for i in (0, B // 2, B - 1):
        one = _run_dxb(X[i * P:(i + 1) * P].contiguous(), Wt, b3, vt, bfull, 1, H, W, C, N)
        assert torch.equal(full[i * P:(i + 1) * P], one), i


def test_dxb_and_bf16_modes_round_trip():
    """A bf16 engine codes in conv mode "dxb" by default; a bitstream records it and decodes
    in it; a "bf16" (conv3_bf16.hip) bitstream decodes by switching the engine's mode."""
    from idfcodec import configs, synthetic
    model = synthetic.build_model(configs.get("imagenet64")).cuda()
    model.idf_precision = "bf16"
    eng = model.engine()
    assert eng.conv_mode == "dxb" and eng.conv_family == "dxb"
    codec = model.codec()
    x = synthetic.images(3, seed=12).cuda()
    bs = codec.encode(x)
    assert bs.meta["conv"] == "dxb"
    out, info = codec.decode(bs)
    assert info["ok"] and torch.equal(out, x)
    eng.set_conv_mode("bf16")
    bs16 = codec.encode(x)
    eng.set_conv_mode("dxb")
    assert bs16.meta["conv"] == "bf16"
    out, info = codec.decode(bs16)
    assert info["ok"] and torch.equal(out, x)
    assert eng.conv_mode == "dxb"
