"""GPU parity of the flow kernels against the torch-fp32 oracle (itself pinned to
the reference by tests/test_oracle_golden.py).

Tolerance: flow activations within 1e-5 (|a-b| <= 1e-5 * max(1, |b|)) given
teacher-forced identical inputs (BASELINE.json north_star).  Rounded outputs
(latents) may differ where the un-rounded value sits within the tolerance of a
rounding boundary; those flips are counted and bounded, and the
exact round trip is checked on the build's own pipeline."""
import numpy as np
import pytest
import torch
import yaml

pytestmark = pytest.mark.gpu
TOL = 1e-5


def close(a, b, tol=TOL):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    err = ((a - b).abs() / b.abs().clamp(min=1.0)).max().item()
    assert err <= tol, f"max scaled error {err:.3e} > {tol}"
    return err


def _case(golden, name):
    d = golden(f"flow_{name}.npz")
    cfg = yaml.safe_load(bytes(d["cfg_yaml"]).decode())
    return d, cfg


def _model(cfg):
    from idfcodec import synthetic
    return synthetic.build_model(cfg).cuda()


def _oracle(model, cfg):
    import flow_oracle as FO
    return FO.FlowOracle(cfg, {k: v.detach().cpu() for k, v in model.state_dict().items()})


TINY = ["t1_idflows_2lvl", "t2_idflows_3lvl_leaky", "t3_cond_convcond", "t4_cond_s1_odd"]


@pytest.mark.parametrize("name", TINY)
def test_dense_blocks_teacher_forced(golden, name):
    """DenseBlock.forward on the recorded block inputs == the reference's outputs."""
    d, cfg = _case(golden, name)
    model = _model(cfg)
    mods = dict(model.named_modules())
    for i in range(4):
        if f"dense{i}/in" not in d.files:
            break
        x = torch.from_numpy(d[f"dense{i}/in"]).cuda()
        ref = torch.from_numpy(d[f"dense{i}/out"])
        blk = mods[bytes(d[f"dense{i}/name"]).decode()]
        close(blk(x), ref)


@pytest.mark.parametrize("H,W,c,g,act", [(8, 8, 9, 24, "ReLU"), (7, 5, 13, 40, "LeakyReLU"),
                                         (16, 16, 100, 44, "ReLU"), (3, 2, 4, 8, "ReLU")])
def test_dense_layer_vs_oracle(H, W, c, g, act):
    import flow_oracle as FO
    from nnlayer import DenseLayer
    torch.manual_seed(0)
    layer = DenseLayer(c, c + g, act).cuda()
    x = torch.randn(3, c, H, W).cuda()
    sd = {k: v.cpu() for k, v in layer.state_dict().items()}
    ref = FO.dense_layer(x.cpu(), {"layers." + k[len("layers."):]: v for k, v in sd.items()}, "", act)
    close(layer(x), ref)


@pytest.mark.parametrize("fold", [False, True])
def test_imagenet64_blocks_teacher_forced(fold):
    """The full-size DenseBlocks of configs/imagenet64.yaml (c up to 521, K up to 4689),
    with the reference's two convolutions per layer and with the 1x1 folded into the 3x3."""
    import flow_oracle as FO
    from idfcodec import configs
    from idfcodec.modules import run_dense_block
    model = _model(configs.get("imagenet64"))
    g = torch.Generator().manual_seed(7)
    for lvl, (c, hw) in enumerate(((9, 32), (18, 16), (36, 8))):
        blk = model.blocks[lvl]["flows"][1].dense
        x = (torch.round(torch.rand(2, c, hw, hw, generator=g) * 512 - 256) / 256)
        sd = {k: v.detach().cpu() for k, v in blk.state_dict().items()}
        ref = FO.dense_block(x, sd, "", 12, "ReLU")
        close(run_dense_block(blk, x.cuda(), fold=fold), ref)
        pr = model.blocks[lvl]["prior"]
        xin = torch.round(torch.rand(2, pr.NN.i_channel, hw, hw, generator=g) * 512 - 256) / 256
        m, ls = pr(xin.cuda())
        sdp = {k: v.detach().cpu() for k, v in pr.NN.state_dict().items()}
        refp = FO.dense_block(xin if pr.cond_channel > 0 else torch.zeros_like(xin), sdp, "", 12, "ReLU")
        close(torch.cat([m, ls], 1), refp)


@pytest.mark.parametrize("name", TINY)
def test_coupling_forward_backward_exact(golden, name):
    d, cfg = _case(golden, name)
    model = _model(cfg)
    cpl = model.blocks[0]["flows"][1]
    C = cpl.channel
    s = cfg["extenddim"]["scale"]
    x = torch.round(torch.randn(2, C, cfg["H"] // s, cfg["W"] // s, generator=torch.Generator().manual_seed(1)) * 64) / 256
    x = x.cuda()
    z, _ = cpl(x, None)
    assert torch.equal(cpl.backward(z), x), "AdditiveCouple backward is not the exact inverse"
    assert torch.equal(z[:, :cpl.a_ch], x[:, :cpl.a_ch])
    # z_b - x_b is on the 1/256 grid
    diff = (z[:, cpl.a_ch:] - x[:, cpl.a_ch:]) * 256
    assert torch.equal(diff, torch.round(diff))


@pytest.mark.parametrize("name", TINY)
def test_model_forward_vs_reference(golden, name):
    """Whole-model forward vs the reference's recorded outputs: means/logscales within
    tolerance where no upstream rounding flipped, flips rare; the device inverse is exact."""
    d, cfg = _case(golden, name)
    model = _model(cfg)
    x = torch.from_numpy(d["input"]).cuda()
    if cfg["name"] == "ConditionalFlows":
        cond = torch.from_numpy(d["cond"]).cuda()
        lat, me, ls, _ = model(x, None, cond)
    else:
        lat, me, ls, _ = model(x, None)
    nflip = ntot = 0
    for i in range(len(lat)):
        ref = torch.from_numpy(d[f"latent{i}"])
        nflip += int((lat[i].cpu() != ref).sum())
        ntot += ref.numel()
    assert nflip <= max(2, ntot // 1000), f"{nflip}/{ntot} latents flipped"
    if nflip == 0:
        for i in range(len(lat)):
            close(me[i], torch.from_numpy(d[f"mean{i}"]), 1e-4)
            close(ls[i], torch.from_numpy(d[f"logscale{i}"]), 1e-4)
    if cfg["name"] != "ConditionalFlows":
        gen = model.generated_from_latents(lat)
        assert torch.equal(gen, x)


@pytest.mark.parametrize("name", TINY)
def test_model_vs_oracle_teacher_forced_levels(golden, name):
    """Per level, feed the oracle the GPU's own level input: flows + prior agree."""
    d, cfg = _case(golden, name)
    model = _model(cfg)
    o = _oracle(model, cfg)
    x = torch.from_numpy(d["input"]).cuda()
    cond = torch.from_numpy(d["cond"]).cuda() if "cond" in d.files else None
    args = (x, None, cond) if cond is not None else (x, None)
    lat, me, ls, _ = model(*args)
    rl, rm, rs = o.forward(x.cpu(), cond.cpu() if cond is not None else None)
    nflip = sum(int((a.cpu() != b).sum()) for a, b in zip(lat, rl))
    ntot = sum(b.numel() for b in rl)
    assert nflip <= max(2, ntot // 1000)


# Round flips against a CPU fp32 run of the same model and images.  A flip cascades through
# the later couplings and levels, and any fp32 reassociation starts one.  Measured with the fused
# DenseBlock head (round 5, profiles/r05/fused_head/parity.log), per level of [12288, 6144, 6144]
# latents vs the reference's recorded B=2 run: [0, 0, 0]; of [98304, 49152, 49152] vs the oracle at
# B=16: [0, 0, 8]; per coupling, teacher-forced (no cascade): [0, 0, 1] of [393216, 196608,
# 98304].  (Before the fused head: [3, 18, 150], [5, 39, 379], [6, 2, 1].)  Each bound is
# max(2x the measured count, 4), so a summation-order change that moves roundings -- the paired
# split schedule gave [0, 4, 50] vs the reference (profiles/r05/pairs/) -- fails here.
FLIP_BOUND_REF_B2 = (4, 4, 4)
FLIP_BOUND_ORACLE_B16 = (4, 4, 16)
COUPLE_FLIP_BOUND = (4, 4, 4)


def test_imagenet64_forward_vs_oracle_b16():
    """The production path (dx3 at every level, the bench's conv mode) at B=16 against the
    torch-fp32 oracle (oracle/flow_oracle.py) on the same seeded model and images: the Round
    flips per level are counted, printed and bounded by FLIP_BOUND."""
    import flow_oracle as FO
    from idfcodec import configs, synthetic
    cfg = configs.get("imagenet64")
    model = _model(cfg)
    eng = model.engine()
    assert eng.conv_mode == "dx3"
    img = synthetic.images(16, seed=2)
    x = FO.dequant(img)
    lat, _, _, _ = model(x.cuda(), None)
    o = _oracle(model, cfg)
    rl, _, _ = o.forward(x)
    flips = [int((a.cpu() != b).sum()) for a, b in zip(lat, rl)]
    sizes = [b.numel() for b in rl]
    print(f"flips vs the fp32 oracle per level (B=16, dx3): {flips} of {sizes}; "
          f"bounds {FLIP_BOUND_ORACLE_B16}")
    for i in range(3):
        assert flips[i] <= FLIP_BOUND_ORACLE_B16[i], (i, flips[i], sizes[i])
    assert torch.equal(model.generated_from_latents(lat), x.cuda())


def test_imagenet64_coupling_flips_teacher_forced():
    """Round flips with no cascade: every imagenet64 coupling's DenseBlock as the engine packed
    it (dx3, the production path) on the oracle's own input to that coupling (B=16), rounded
    to the 1/256 grid (roundlib.py:34-38) against the oracle's rounded output.  Per coupling
    the flips come only from the last-bit differences of the two fp32 computations."""
    import flow_oracle as FO
    from idfcodec import configs, synthetic
    from idfcodec.modules import run_device_block
    cfg = configs.get("imagenet64")
    model = _model(cfg)
    eng = model.engine()
    assert eng.conv_mode == "dx3"
    o = _oracle(model, cfg)
    x = FO.dequant(synthetic.images(16, seed=2))
    per_level = []
    with torch.no_grad():
        for lvl in range(o.nsplit):
            x = FO.extend_fwd(x, o.scale)
            fl = tot = 0
            for k in range(o.nflows):
                x = FO.permute_fwd(x, o.sd[f"blocks.{lvl}.flows.{2 * k}.P"])
                a = int(x.shape[1] * o.split)
                ref = FO.round8(o.coupling_nn(lvl, k, x[:, :a]), o.nbits)
                dev, _ = run_device_block(eng.couple[lvl][k], x[:, :a].contiguous().cuda())
                fl += int((FO.round8(dev.cpu(), o.nbits) != ref).sum())
                tot += ref.numel()
                x = torch.cat([x[:, :a], x[:, a:] + ref], dim=1)
            x = FO.permute_fwd(x, o.sd[f"blocks.{lvl}.flows.{2 * o.nflows}.P"])
            per_level.append((fl, tot))
            if lvl < o.nsplit - 1:
                x = x[:, x.shape[1] // 2:]
    print(f"coupling Round flips per level, teacher-forced (B=16, dx3): {per_level}; "
          f"bounds {COUPLE_FLIP_BOUND}")
    for i, (fl, tot) in enumerate(per_level):
        assert fl <= COUPLE_FLIP_BOUND[i], (i, fl, tot)


def test_imagenet64_forward_vs_reference(golden):
    """configs/imagenet64.yaml, seeded model regenerated on the device, B=2:
    latents vs the reference's CPU run (few flips), exact inverse."""
    from idfcodec import configs, synthetic
    d = golden("imagenet64_b2.npz")
    model = _model(configs.get("imagenet64"))
    img = torch.from_numpy(d["image_u8"]).cuda()
    import flow_oracle as FO
    x = FO.dequant(img.cpu()).cuda()
    lat, me, ls, _ = model(x, None)
    # the CPU reference's oneDNN convolutions and the device GEMMs round differently;
    # a flipped Round cascades through later couplings (fp32 vs fp64
    # already flips 0.46% at the top level), so only the rate is bounded here --
    # the 1e-5 parity is asserted teacher-forced in test_imagenet64_x3_blocks_teacher_forced.
    # Bound: FLIP_BOUND_REF_B2, max(2x the measured counts, 4) (printed)
    flips = [int((lat[i].cpu() != torch.from_numpy(d[f"latent{i}"])).sum()) for i in range(3)]
    sizes = [int(d[f"latent{i}"].size) for i in range(3)]
    print(f"flips vs the reference per level: {flips} of {sizes}; bounds {FLIP_BOUND_REF_B2}")
    for i in range(3):
        assert flips[i] <= FLIP_BOUND_REF_B2[i], (i, flips[i], sizes[i])
    assert torch.equal(model.generated_from_latents(lat), x)
    lp, _ = model.log_likelihood(lat, me, ls)
    # theoretical bits per sub-pixel within 1% of the reference's
    assert abs(lp.mean().item() / d["log_prob"].mean() - 1) < 0.01
    del synthetic


@pytest.mark.parametrize("B,H,W,C,N,act,fold", [
    (3, 32, 32, 52, 44, "ReLU", True), (5, 16, 16, 100, 44, "ReLU", True),
    (7, 8, 8, 168, 44, "ReLU", True), (2, 27, 23, 40, 32, "LeakyReLU", True),
    (9, 4, 4, 24, 64, "ReLU", True), (4, 2, 2, 16, 128, "ReLU", False),
    (1, 8, 8, 12, 44, "ReLU", False), (2, 64, 64, 8, 16, "ReLU", True)])
def test_conv3x3_halo_kernel_vs_fp64(B, H, W, C, N, act, fold):
    """The LDS halo-tiled 3x3 conv (incl. split-K for small images, ragged tiles,
    several n-tiles) against an fp64 conv2d with the same padded weights."""
    import torch.nn.functional as F
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    from idfcodec.packing import round_up, tile_n
    g = torch.Generator().manual_seed(B * 1000 + H * 10 + C)
    ld = round_up(C + N, 16) + 4
    X = torch.randn(B * H * W, ld, generator=g)
    ldw = round_up(C, 16)
    n_alloc = round_up(N, 64)
    Wt = torch.randn(n_alloc, 9, ldw, generator=g) * 0.05
    b3 = torch.randn(n_alloc, generator=g) * 0.1
    vt = torch.randn(9, n_alloc, generator=g) * 0.1 if fold else None
    bfull = None
    if fold:
        s = b3.clone()
        for t in range(9):
            s = s + vt[t]
        bfull = s
    dev = torch.device("cuda")
    Xd, Wd_, b3d = X.to(dev), Wt.to(dev), b3.to(dev)
    vtd = vt.to(dev) if fold else None
    bfd = bfull.to(dev) if fold else None
    out = torch.zeros(B * H * W, ld, device=dev)
    wsn = lib().idf_conv3x3_halo_workspace(B, H, W, C, N)
    ws = torch.empty(max(wsn, 1), device=dev)
    check(lib().idf_conv3x3_halo(_lib.stream_ptr(), B, H, W, C, ptr(Xd), ld, ptr(Wd_), ldw, n_alloc,
                                 ptr(b3d), ptr(vtd), n_alloc, ptr(bfd), N, ptr(out), ld,
                                 _lib.ACT[act], 0.01, ptr(ws), wsn), "halo")
    torch.cuda.synchronize()
    x4 = X[:, :C].double().view(B, H, W, C).permute(0, 3, 1, 2)
    w4 = Wt[:N, :, :C].double().permute(0, 2, 1).reshape(N, C, 3, 3)
    ref = F.conv2d(x4, w4, padding=1) + b3[:N].double().view(1, -1, 1, 1)
    if fold:
        mask = F.conv2d(torch.ones(1, 1, H, W, dtype=torch.float64),
                        torch.eye(9, dtype=torch.float64).view(9, 1, 3, 3), padding=1)
        ref = ref + torch.einsum("tn,bthw->bnhw", vt[:, :N].double(), mask)
    ref = F.relu(ref) if act == "ReLU" else F.leaky_relu(ref, 0.01)
    got = out[:, :N].cpu().double().view(B, H, W, N).permute(0, 3, 1, 2)
    close(got, ref, 2e-5)
    assert torch.all(out[:, N:].cpu() == 0), "wrote outside the N output columns"
