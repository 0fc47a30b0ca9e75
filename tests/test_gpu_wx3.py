"""GPU parity of the split-f16 Winograd conv (idf_conv3x3_wx3: conv3_wino.hip with X3) against
fp64 conv2d with the same folded weights -- the same cases and the same 1e-5 bound as the fp32
Winograd kernel (tests/test_gpu_wino.py), plus its error next to the fp32 kernel's, the range
guard, and data far from unit scale."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def scaled_err(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs() / b.abs().clamp(min=1.0)).max().item()


def run_case(B, H, W, C, N, act, fold, scale=1.0, spike=None, res=False, check_in=1):
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    from idfcodec.packing import round_up, wino_weights, wino_weights_x3
    g = torch.Generator().manual_seed(B * 7 + H * 3 + C)
    ld = round_up(C + N, 16) + 4
    X = torch.randn(B * H * W, ld, generator=g) * scale
    if spike is not None:
        X[B * H * W // 2, 0] = spike
    ldw = round_up(C, 16)
    n_alloc = round_up(N, 16)
    Wt = torch.randn(n_alloc, 9, ldw, generator=g, dtype=torch.float64) / np.sqrt(9 * C)
    U = wino_weights(Wt.numpy(), ldw // 16)
    Ux, ysc = wino_weights_x3(Wt.numpy(), ldw // 16)
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
    Xd, Ud, Uxd, b3d = X.to(dev), torch.from_numpy(U).to(dev), \
        torch.from_numpy(Ux.view(np.int16)).to(dev), b3.to(dev)
    vtd = vt.to(dev) if fold else None
    bfd = bfull.to(dev) if fold else None
    Rd = R.to(dev) if res else None
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    wsn = lib().idf_conv3x3_wino_workspace(B, H, W, C, N)
    ws = torch.empty(max(wsn, 1), device=dev)
    outs = []
    for x3 in (False, True):
        out = torch.zeros(B * H * W, ld, device=dev)
        if res:
            if x3:
                check(lib().idf_conv3x3_wx3_res(
                    _lib.stream_ptr(), B, H, W, C, ptr(Xd), ld, ptr(Uxd), n_alloc // 16, ysc,
                    ptr(b3d), N, ptr(out), ld, ptr(Rd), N, _lib.ACT[act], 0.01, ptr(flag), 1,
                    ptr(ws), wsn), "wx3_res")
            else:
                check(lib().idf_conv3x3_wino_res(
                    _lib.stream_ptr(), B, H, W, C, ptr(Xd), ld, ptr(Ud), n_alloc // 16, ptr(b3d),
                    N, ptr(out), ld, ptr(Rd), N, _lib.ACT[act], 0.01, ptr(ws), wsn), "wino_res")
        elif x3:
            check(lib().idf_conv3x3_wx3(
                _lib.stream_ptr(), B, H, W, C, ptr(Xd), ld, ptr(Uxd), n_alloc // 16, ysc, ptr(b3d),
                ptr(vtd), n_alloc, ptr(bfd), N, ptr(out), ld, _lib.ACT[act], 0.01, ptr(flag), check_in,
                ptr(ws), wsn), "wx3")
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
    ref = F.relu(ref) if act == "ReLU" else F.leaky_relu(ref, 0.01)
    errs = []
    for out in outs:
        got = out[:, :N].double().view(B, H, W, N).permute(0, 3, 1, 2)
        errs.append(scaled_err(got, ref))
        assert torch.all(out[:, N:] == 0), "wrote outside the N output columns"
    return errs, int(flag.item())


@pytest.mark.parametrize("B,H,W,C,N,act,fold", [
    (3, 32, 32, 52, 44, "ReLU", True), (5, 16, 16, 100, 44, "ReLU", True),
    (7, 8, 8, 168, 44, "ReLU", True), (2, 64, 64, 8, 16, "LeakyReLU", True),
    (4, 4, 4, 24, 32, "ReLU", False), (2, 2, 6, 12, 44, "ReLU", True),
    (3, 32, 32, 496, 44, "ReLU", True), (1, 16, 16, 520, 44, "ReLU", True),
    (2, 27, 23, 52, 44, "ReLU", True), (3, 5, 7, 24, 32, "LeakyReLU", True),
    (4, 1, 3, 16, 16, "ReLU", True), (2, 9, 9, 100, 44, "ReLU", False),
    (1, 45, 37, 20, 44, "ReLU", True),
    (130, 2, 2, 40, 44, "ReLU", True), (33, 4, 4, 100, 44, "ReLU", True),
    (17, 3, 3, 24, 32, "LeakyReLU", False),
    # resflow-patches-vqvae's 27x23 patches (tiled 24 wide): couplings N = 32, prior N = 43
    (3, 27, 23, 100, 32, "LeakyReLU", True), (2, 27, 23, 200, 43, "LeakyReLU", True)])
def test_wx3_vs_fp64(B, H, W, C, N, act, fold):
    (e32, ex3), flag = run_case(B, H, W, C, N, act, fold)
    print(f"f32 {e32:.2e} x3 {ex3:.2e}")
    assert flag == 0
    assert ex3 <= 1e-5, f"wx3 max scaled error {ex3:.3e}"
    # fp32-class: within a small factor of the exact-f32 kernel's own rounding error
    assert ex3 <= max(4 * e32, 1e-6), (e32, ex3)


@pytest.mark.parametrize("scale", [1e-3, 30.0])
def test_wx3_far_from_unit_scale(scale):
    (e32, ex3), flag = run_case(2, 16, 16, 200, 44, "ReLU", True, scale=scale)
    assert flag == 0
    assert ex3 <= max(4 * e32, 1e-6), (e32, ex3)


@pytest.mark.parametrize("B,H,W,C,N", [(2, 16, 16, 128, 128), (3, 8, 8, 256, 256)])
def test_wx3_residual_variant(B, H, W, C, N):
    (e32, ex3), flag = run_case(B, H, W, C, N, "ReLU", False, res=True)
    assert flag == 0 and ex3 <= 1e-5 and ex3 <= max(4 * e32, 1e-6), (e32, ex3)


def test_wx3_range_guard_sets_flag():
    _, flag = run_case(1, 8, 8, 16, 16, "ReLU", True, spike=40000.0)
    assert flag == 1
    _, flag = run_case(1, 8, 8, 16, 16, "ReLU", True, spike=float("nan"))
    assert flag == 1
    _, flag = run_case(1, 8, 8, 16, 16, "ReLU", True, spike=1000.0)
    assert flag == 0


def test_wx3_output_guard_sets_flag():
    # no input check: inputs within the V guard, but outputs beyond +-8192 trip the
    # epilogue's output guard (what makes later layers' unchecked inputs safe)
    _, flag = run_case(1, 8, 8, 16, 16, "None", True, scale=4000.0, check_in=0)
    assert flag == 1
    _, flag = run_case(1, 8, 8, 16, 16, "None", True, scale=100.0, check_in=0)
    assert flag == 0


@pytest.mark.parametrize("B,H,W,C,N", [(3, 27, 23, 100, 32), (2, 27, 23, 200, 43),
                                       (2, 32, 32, 100, 43), (4, 8, 8, 100, 43)])
def test_wx3_unchecked_layers(B, H, W, C, N):
    """The instantiations without the input range check (every DenseLayer after the block's
    first) at the compile-time tile widths: 24 (two and three n-fragments), 32, 8."""
    (e32, ex3), flag = run_case(B, H, W, C, N, "LeakyReLU", True, check_in=0)
    assert flag == 0 and ex3 <= 1e-5 and ex3 <= max(4 * e32, 1e-6), (e32, ex3)
