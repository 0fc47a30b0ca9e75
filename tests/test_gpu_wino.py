"""GPU parity of the Winograd F(2x2,3x3) DenseLayer conv (conv3_wino.hip) against fp64
conv2d with the same folded weights, and of whole DenseBlocks on the Winograd path
against the oracle (1e-5, teacher-forced)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def close(a, b, tol):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    err = ((a - b).abs() / b.abs().clamp(min=1.0)).max().item()
    assert err <= tol, f"max scaled error {err:.3e} > {tol}"
    return err


@pytest.mark.parametrize("B,H,W,C,N,act,fold", [
    (3, 32, 32, 52, 44, "ReLU", True), (5, 16, 16, 100, 44, "ReLU", True),
    (7, 8, 8, 168, 44, "ReLU", True), (2, 64, 64, 8, 16, "LeakyReLU", True),
    (4, 4, 4, 24, 32, "ReLU", False), (2, 2, 6, 12, 44, "ReLU", True),
    (3, 32, 32, 496, 44, "ReLU", True), (1, 16, 16, 520, 44, "ReLU", True),
    # odd sizes (config 5's 27x23 patches): tiled as the next even size, overhang masked
    (2, 27, 23, 52, 44, "ReLU", True), (3, 5, 7, 24, 32, "LeakyReLU", True),
    (4, 1, 3, 16, 16, "ReLU", True), (2, 9, 9, 100, 44, "ReLU", False),
    (1, 45, 37, 20, 44, "ReLU", True),
    # many small images per block in the 1024-slot stage (config 4's 4x4 and 2x2 levels)
    (130, 2, 2, 40, 44, "ReLU", True), (33, 4, 4, 100, 44, "ReLU", True),
    (17, 3, 3, 24, 32, "LeakyReLU", False)])
def test_conv3x3_wino_vs_fp64(B, H, W, C, N, act, fold):
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    from idfcodec.packing import round_up, wino_weights
    g = torch.Generator().manual_seed(B * 7 + H * 3 + C)
    ld = round_up(C + N, 16) + 4
    X = torch.randn(B * H * W, ld, generator=g)
    ldw = round_up(C, 16)
    n_alloc = round_up(N, 16)
    Wt = torch.randn(n_alloc, 9, ldw, generator=g, dtype=torch.float64) / np.sqrt(9 * C)
    U = wino_weights(Wt.numpy(), ldw // 16)
    b3 = torch.randn(n_alloc, generator=g) * 0.1
    vt = torch.randn(9, n_alloc, generator=g) * 0.1 if fold else None
    bfull = None
    if fold:
        s = b3.clone()
        for t in range(9):
            s = s + vt[t]
        bfull = s
    dev = torch.device("cuda")
    Xd, Ud, b3d = X.to(dev), torch.from_numpy(U).to(dev), b3.to(dev)
    vtd = vt.to(dev) if fold else None
    bfd = bfull.to(dev) if fold else None
    out = torch.zeros(B * H * W, ld, device=dev)
    assert lib().idf_conv3x3_wino_supported(H, W)
    wsn = lib().idf_conv3x3_wino_workspace(B, H, W, C, N)
    ws = torch.empty(max(wsn, 1), device=dev)
    check(lib().idf_conv3x3_wino(_lib.stream_ptr(), B, H, W, C, ptr(Xd), ld, ptr(Ud), n_alloc // 16,
                                 ptr(b3d), ptr(vtd), n_alloc, ptr(bfd), N, ptr(out), ld,
                                 _lib.ACT[act], 0.01, ptr(ws), wsn), "wino")
    torch.cuda.synchronize()
    x4 = X[:, :C].double().view(B, H, W, C).permute(0, 3, 1, 2)
    w4 = Wt[:N, :, :C].permute(0, 2, 1).reshape(N, C, 3, 3)
    ref = F.conv2d(x4, w4, padding=1) + b3[:N].double().view(1, -1, 1, 1)
    if fold:
        mask = F.conv2d(torch.ones(1, 1, H, W, dtype=torch.float64),
                        torch.eye(9, dtype=torch.float64).view(9, 1, 3, 3), padding=1)
        ref = ref + torch.einsum("tn,bthw->bnhw", vt[:, :N].double(), mask)
    ref = F.relu(ref) if act == "ReLU" else F.leaky_relu(ref, 0.01)
    got = out[:, :N].cpu().double().view(B, H, W, N).permute(0, 3, 1, 2)
    close(got, ref, 1e-5)
    assert torch.all(out[:, N:].cpu() == 0), "wrote outside the N output columns"


def test_geometry_support_reported():
    from idfcodec._lib import lib
    assert lib().idf_conv3x3_wino_supported(27, 23) and lib().idf_conv3x3_wino_supported(8, 8)
    assert not lib().idf_conv3x3_wino_supported(0, 5)


def test_imagenet64_blocks_on_winograd_path():
    """Whole imagenet64 DenseBlocks (couplings and priors of every level) run through the
    engine's packing with Winograd enabled, teacher-forced against the oracle."""
    import flow_oracle as FO
    from idfcodec import configs, synthetic
    from idfcodec.engine import DeviceBlock
    from idfcodec.packing import pack_dense_block, round_up
    from idfcodec import _lib
    from idfcodec._lib import lib, ptr, check
    model = synthetic.build_model(configs.get("imagenet64"))
    gen = torch.Generator().manual_seed(11)
    dev = torch.device("cuda")
    for lvl, (hw, name) in enumerate(((32, "flows.1.dense"), (16, "flows.3.dense"), (8, "prior.NN"))):
        prefix = f"blocks.{lvl}.{name}."
        sd = {k[len(prefix):]: v for k, v in model.state_dict().items() if k.startswith(prefix)}
        pb = pack_dense_block(sd, "", 12, "ReLU", fold=True, wino=True)
        db = DeviceBlock(pb, dev)
        a = pb.geom.a
        x = torch.round(torch.rand(2, a, hw, hw, generator=gen) * 512 - 256) / 256
        ref = FO.dense_block(x, {k: v.detach() for k, v in sd.items()}, "", 12, "ReLU")
        P = 2 * hw * hw
        ld = pb.geom.ld_feat
        feat = torch.zeros(P, ld, device=dev)
        feat[:, :a] = x.permute(0, 2, 3, 1).reshape(P, a).to(dev)
        tmp = torch.zeros(P, ld, device=dev)
        s = _lib.stream_ptr()
        check(lib().idf_dense_block_f32(s, __import__("ctypes").byref(db.desc), 2, hw, hw, ptr(feat),
                                        ld, ptr(tmp), ld, None), "block")
        n = pb.geom.n_head
        out = torch.empty(P, round_up(n, 4), device=dev)
        check(lib().idf_conv1x1_f32(s, P, pb.geom.width, n, ptr(feat), ld, ptr(db.wh), pb.ldwh,
                                    pb.nh_alloc, ptr(db.bh), ptr(out), round_up(n, 4), 2, hw, hw,
                                    None), "head")
        got = out[:, :n].view(2, hw, hw, n).permute(0, 3, 1, 2)
        close(got, ref, 1e-5)


@pytest.mark.parametrize("B,H,W,C,N,act,res", [
    (4, 8, 8, 384, 384, "ReLU", True),      # config 3 ResBlock conv2 (8x8 latents)
    (2, 8, 8, 384, 384, "ReLU", False),     # ResBlock conv1
    (1, 32, 32, 64, 64, "ReLU", True), (3, 7, 5, 16, 20, "None", True)])
def test_conv3x3_wino_res_vs_fp64(B, H, W, C, N, act, res):
    """idf_conv3x3_wino_res (the VQ-VAE's 3x3 convs): act(res + conv3x3(x) + bias)."""
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    from idfcodec.packing import round_up, wino_weights
    g = torch.Generator().manual_seed(B + H * 5 + C)
    ld = round_up(C, 4)
    ldo = round_up(N, 4)
    X = torch.randn(B * H * W, ld, generator=g)
    R = torch.randn(B * H * W, ldo, generator=g)
    ldw = round_up(C, 16)
    n_alloc = round_up(N, 16)
    Wt = torch.randn(n_alloc, 9, ldw, generator=g, dtype=torch.float64) / np.sqrt(9 * C)
    bias = torch.randn(n_alloc, generator=g) * 0.1
    dev = torch.device("cuda")
    Ud = torch.from_numpy(wino_weights(Wt.numpy(), ldw // 16)).to(dev)
    Xd, Rd, bd = X.to(dev), R.to(dev), bias.to(dev)
    out = torch.zeros(B * H * W, ldo, device=dev)
    wsn = lib().idf_conv3x3_wino_workspace(B, H, W, C, N)
    ws = torch.empty(max(wsn, 1), device=dev)
    check(lib().idf_conv3x3_wino_res(_lib.stream_ptr(), B, H, W, C, ptr(Xd), ld, ptr(Ud),
                                     n_alloc // 16, ptr(bd), N, ptr(out), ldo,
                                     ptr(Rd) if res else None, ldo, _lib.ACT[act], 0.01, ptr(ws),
                                     wsn), "wino_res")
    torch.cuda.synchronize()
    x4 = X[:, :C].double().view(B, H, W, C).permute(0, 3, 1, 2)
    w4 = Wt[:N, :, :C].permute(0, 2, 1).reshape(N, C, 3, 3)
    ref = F.conv2d(x4, w4, padding=1) + bias[:N].double().view(1, -1, 1, 1)
    if res:
        ref = ref + R[:, :N].double().view(B, H, W, N).permute(0, 3, 1, 2)
    if act == "ReLU":
        ref = F.relu(ref)
    got = out[:, :N].cpu().double().view(B, H, W, N).permute(0, 3, 1, 2)
    close(got, ref, 1e-5)
