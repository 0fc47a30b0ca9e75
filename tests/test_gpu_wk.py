"""GPU parity of the K=32 split-f16 Winograd conv (idf_conv3x3_wk, conv3_wk.hip) against fp64
conv2d with the same folded weights: the geometries of the DenseBlocks it serves (imagenet64's
32x32 / 16x16 / 8x8 levels, config 5's 27x23 patches, odd sizes), the split-K levels, wide
outputs (VQ-VAE convs, several n-tiles), the residual variant, data far from unit scale, and the
range guard -- with the 1e-5 bound of the north star and within a small factor of the exact-f32
kernel's own rounding error (the reference is a plain fp32 conv, nnlayer.py:48-51)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def scaled_err(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs() / b.abs().clamp(min=1.0)).max().item()


def run_case(B, H, W, C, N, act, fold, scale=1.0, spike=None, res=False, check_in=1, sparse=False):
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    from idfcodec.packing import round_up, wino_weights, wk_weights
    g = torch.Generator().manual_seed(B * 7 + H * 3 + C + 1)
    ld = round_up(C + N, 16) + 4
    X = torch.randn(B * H * W, ld, generator=g) * scale
    if sparse:  # ReLU-like inputs: half the features exactly zero
        X = X.clamp(min=0)
    if spike is not None:
        X[B * H * W // 2, 0] = spike
    ldw = round_up(C, 16)
    n_alloc = round_up(N, 16)
    Wt = torch.randn(n_alloc, 9, ldw, generator=g, dtype=torch.float64) / np.sqrt(9 * C)
    U = wino_weights(Wt.numpy(), ldw // 16)
    Uk, ysc = wk_weights(Wt.numpy())
    b3 = torch.randn(n_alloc, generator=g) * 0.1
    vt = torch.randn(9, n_alloc, generator=g) * 0.1 if fold else None
    bfull = None
    if fold:
        s = b3.clone()
        for t in range(9):
            s = s + vt[t]
        bfull = s
    R = torch.randn(B * H * W, N, generator=g) if res else None
    dev = torch.device("cuda")
    Xd, Ud, Ukd, b3d = X.to(dev), torch.from_numpy(U).to(dev), \
        torch.from_numpy(Uk.view(np.int16)).to(dev), b3.to(dev)
    vtd = vt.to(dev) if fold else None
    bfd = bfull.to(dev) if fold else None
    Rd = R.to(dev) if res else None
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    assert lib().idf_conv3x3_wk_supported(H, W)
    wsn = max(lib().idf_conv3x3_wino_workspace(B, H, W, C, N), lib().idf_conv3x3_wk_workspace(B, H, W, C, N))
    ws = torch.empty(max(wsn, 1), device=dev)
    outs = []
    for wk in (False, True):
        out = torch.zeros(B * H * W, ld, device=dev)
        if res:
            if wk:
                check(lib().idf_conv3x3_wk_res(
                    _lib.stream_ptr(), B, H, W, C, ptr(Xd), ld, ptr(Ukd), n_alloc // 16, ysc,
                    ptr(b3d), N, ptr(out), ld, ptr(Rd), N, _lib.ACT[act], 0.01, ptr(flag), check_in,
                    ptr(ws), wsn), "wk_res")
            else:
                check(lib().idf_conv3x3_wino_res(
                    _lib.stream_ptr(), B, H, W, C, ptr(Xd), ld, ptr(Ud), n_alloc // 16, ptr(b3d),
                    N, ptr(out), ld, ptr(Rd), N, _lib.ACT[act], 0.01, ptr(ws), wsn), "wino_res")
        elif wk:
            check(lib().idf_conv3x3_wk(
                _lib.stream_ptr(), B, H, W, C, ptr(Xd), ld, ptr(Ukd), n_alloc // 16, ysc, ptr(b3d),
                ptr(vtd), n_alloc, ptr(bfd), N, ptr(out), ld, _lib.ACT[act], 0.01, ptr(flag), check_in,
                ptr(ws), wsn), "wk")
        else:
            check(lib().idf_conv3x3_wino(
                _lib.stream_ptr(), B, H, W, C, ptr(Xd), ld, ptr(Ud), n_alloc // 16, ptr(b3d),
                ptr(vtd), n_alloc, ptr(bfd), N, ptr(out), ld, _lib.ACT[act], 0.01, ptr(ws), wsn),
                "wino")
        torch.cuda.synchronize()
        outs.append(out.cpu())
    x4 = X[:, :C].double().view(B, H, W, C).permute(0, 3, 1, 2)
    w4 = Wt[:N, :, :C].permute(0, 2, 1).reshape(N, C, 3, 3)
    ref = F.conv2d(x4, w4, padding=1) + b3[:N].double().view(1, -1, 1, 1)
    if fold:
        mask = F.conv2d(torch.ones(1, 1, H, W, dtype=torch.float64),
                        torch.eye(9, dtype=torch.float64).view(9, 1, 3, 3), padding=1)
        ref = ref + torch.einsum("tn,bthw->bnhw", vt[:, :N].double(), mask)
    if res:
        ref = R.double().view(B, H, W, N).permute(0, 3, 1, 2) + ref
    ref = {"ReLU": F.relu, "LeakyReLU": lambda t: F.leaky_relu(t, 0.01),
           "None": lambda t: t}[act](ref)
    errs = []
    for out in outs:
        got = out[:, :N].double().view(B, H, W, N).permute(0, 3, 1, 2)
        errs.append(scaled_err(got, ref))
        assert torch.all(out[:, N:] == 0), "wrote outside the N output columns"
    return errs, int(flag.item())


GEOMS = [
    # imagenet64 DenseBlocks: L0 32x32 (TW 32), L1 16x16 (TW 16), L2 8x8 (TW 8, split-K)
    (3, 32, 32, 12, 43, "ReLU", True), (3, 32, 32, 52, 44, "ReLU", True),
    (3, 32, 32, 496, 43, "ReLU", True), (5, 16, 16, 100, 44, "ReLU", True),
    (1, 16, 16, 520, 43, "ReLU", True), (7, 8, 8, 168, 44, "ReLU", True),
    (5, 8, 8, 536, 43, "ReLU", True),
    # other geometries: runtime tile width, odd sizes, tiny images, wide images
    (2, 64, 64, 8, 16, "LeakyReLU", True),
    (2, 27, 23, 52, 44, "ReLU", True), (3, 5, 7, 24, 32, "LeakyReLU", True),
    (2, 9, 9, 100, 44, "ReLU", False),
    (1, 45, 37, 20, 44, "ReLU", True),
    # resflow-patches-vqvae's 27x23 patches: couplings N = 32, prior N = 43
    (3, 27, 23, 100, 32, "LeakyReLU", True), (2, 27, 23, 200, 43, "LeakyReLU", True)]


@pytest.mark.parametrize("B,H,W,C,N,act,fold", GEOMS)
def test_wk_vs_fp64(B, H, W, C, N, act, fold):
    (e32, ewk), flag = run_case(B, H, W, C, N, act, fold)
    print(f"f32 {e32:.2e} wk {ewk:.2e}")
    assert flag == 0
    assert ewk <= 1e-5, f"wk max scaled error {ewk:.3e}"
    assert ewk <= max(4 * e32, 1e-6), (e32, ewk)


@pytest.mark.parametrize("B,H,W,C,N", [(3, 32, 32, 200, 43), (2, 16, 16, 300, 43), (4, 8, 8, 400, 43)])
def test_wk_unchecked_and_sparse(B, H, W, C, N):
    """Every DenseLayer after a block's first runs without the input check, on ReLU outputs."""
    (e32, ewk), flag = run_case(B, H, W, C, N, "ReLU", True, check_in=0, sparse=True)
    assert flag == 0 and ewk <= 1e-5 and ewk <= max(4 * e32, 1e-6), (e32, ewk)


@pytest.mark.parametrize("scale", [1e-3, 30.0])
def test_wk_far_from_unit_scale(scale):
    (e32, ewk), flag = run_case(2, 16, 16, 200, 44, "ReLU", True, scale=scale)
    assert flag == 0
    assert ewk <= max(4 * e32, 1e-6), (e32, ewk)


@pytest.mark.parametrize("B,H,W,C,N", [(2, 16, 16, 128, 128), (3, 8, 8, 256, 256),
                                       (2, 16, 16, 96, 80)])
def test_wk_residual_and_wide_outputs(B, H, W, C, N):
    (e32, ewk), flag = run_case(B, H, W, C, N, "ReLU", False, res=True)
    assert flag == 0 and ewk <= 1e-5 and ewk <= max(4 * e32, 1e-6), (e32, ewk)


def test_wk_geometry_support():
    """Packed small images (config 4's 4x4 / 2x2 levels, the 1024-slot stage) stay on wx3."""
    from idfcodec._lib import lib
    for hw in ((32, 32), (16, 16), (8, 8), (27, 23), (5, 7), (64, 64)):
        assert lib().idf_conv3x3_wk_supported(*hw), hw
    for hw in ((4, 4), (2, 2), (2, 6), (1, 3)):
        assert not lib().idf_conv3x3_wk_supported(*hw), hw


def test_wk_range_guard_sets_flag():
    _, flag = run_case(1, 8, 8, 16, 16, "ReLU", True, spike=40000.0)
    assert flag == 1
    _, flag = run_case(1, 8, 8, 16, 16, "ReLU", True, spike=float("nan"))
    assert flag == 1
    _, flag = run_case(1, 8, 8, 16, 16, "ReLU", True, spike=1000.0)
    assert flag == 0


def test_wk_output_guard_sets_flag():
    _, flag = run_case(1, 16, 16, 16, 16, "None", True, scale=4000.0, check_in=0)
    assert flag == 1
    _, flag = run_case(1, 16, 16, 16, 16, "None", True, scale=100.0, check_in=0)
    assert flag == 0


def test_wk_batch_invariant():
    """An image's outputs do not depend on the batch it is computed in (the decoder
    recomputes the encoder's coupling outputs bit for bit)."""
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    from idfcodec.packing import round_up, wk_weights
    dev = torch.device("cuda")
    for (H, W, C, N) in ((32, 32, 100, 43), (16, 16, 200, 43), (8, 8, 300, 43), (27, 23, 60, 32)):
        g = torch.Generator().manual_seed(H + C)
        ld = round_up(C + N, 16)
        B = 6
        X = torch.randn(B * H * W, ld, generator=g)
        Wt = torch.randn(round_up(N, 16), 9, round_up(C, 16), generator=g, dtype=torch.float64) / 30
        Uk, ysc = wk_weights(Wt.numpy())
        Ukd = torch.from_numpy(Uk.view(np.int16)).to(dev)
        b3 = torch.zeros(round_up(N, 16), device=dev)
        outs = []
        for b0, nb in ((0, B), (2, 1), (3, 3)):
            Xd = X[b0 * H * W:(b0 + nb) * H * W].contiguous().to(dev)
            out = torch.zeros(nb * H * W, ld, device=dev)
            wsn = lib().idf_conv3x3_wk_workspace(nb, H, W, C, N)
            ws = torch.empty(max(wsn, 1), device=dev)
            check(lib().idf_conv3x3_wk(_lib.stream_ptr(), nb, H, W, C, ptr(Xd), ld, ptr(Ukd),
                                       Wt.shape[0] // 16, ysc, ptr(b3), None, 0, None, N, ptr(out),
                                       ld, _lib.ACT["ReLU"], 0.0, None, 0, ptr(ws), wsn), "wk")
            outs.append(out.cpu())
        full = outs[0].view(B, H * W, ld)
        assert torch.equal(full[2], outs[1].view(H * W, ld)), (H, W)
        assert torch.equal(full[3:6], outs[2].view(3, H * W, ld)), (H, W)
