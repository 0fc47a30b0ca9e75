"""Parity of the production path exactly as the codec runs it ("close
production-path parity"):

  * the imagenet64 DenseBlocks packed by the FlowEngine itself (Winograd, split-f16 "x3"
    products: the conv mode bench.py and ImageCodec run) -- every coupling and prior of
    every level, whole block teacher-forced against flow_oracle (the reference's modules,
    pinned by tests/test_oracle_golden.py) at 1e-5, every layer against an fp64 restatement
    of nnlayer.py:48-51 on the kernel's own layer input, bit-identical re-runs (the decoder
    recomputes the encoder's couplings) and batch invariance;
  * the same for the bf16 blocks of resflow-cond-imagenet64 (BASELINE configs[2] names bf16
    coupling convs): every layer against an fp64 conv of the bf16-rounded operands;
  * the reference-recorded imagenet64 rANS streams (tests/golden/imagenet64_b2.npz, from the
    reference coder on the reference model's latents) reproduced by the device coder --
    per (image, level) through StreamCoder as the codec runs it, and the trainer's
    whole-level contract (trainer.py:310-315);
  * DLogistic.log_prob / IDFlows.log_likelihood (idf_log_prob) against the reference's
    recorded log_prob;
  * the HIP dequant against the oracle for all 256 values;
  * the C-ABI host entries idf_rans_encode / idf_rans_decode on KAT1;
  * config 3 at its BASELINE batch (1024 images): exact round trip, sampled streams equal
    the C oracle;
  * configs 4 and 5: every DenseBlock of every level teacher-forced in
    x3 mode (packed 4x4 / 2x2 patches, 27x23 LeakyReLU blocks, cat(z, cond) priors), and
    full-size images' sampled flow streams equal the C oracle.
"""
import ctypes

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
TOL = 1e-5


def scaled_err(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).abs() / b.abs().clamp(min=1.0)).max().item()


def _grid(shape, g, amp=1.0):
    """random values on the 1/256 grid in [-amp, amp] (flow activations live on it)"""
    return torch.round((torch.rand(shape, generator=g) * 2 - 1) * amp * 256) / 256


@pytest.fixture(scope="module")
def in64():
    from idfcodec import configs, synthetic
    model = synthetic.build_model(configs.get("imagenet64")).cuda()
    eng = model.engine()
    assert eng.conv_mode == "dx3" and eng.wx3 and eng.dx3, \
        "imagenet64 must run the split-f16 direct convs (32x32 / 16x16 tiles; 8x8 packed 2x2)"
    return model, eng


def _blocks(model, eng, lvl):
    """(name, module DenseBlock, engine DeviceBlock) of every coupling and the prior of a level"""
    out = [(f"couple{k}", model.blocks[lvl]["flows"][2 * k + 1].dense, eng.couple[lvl][k])
           for k in range(eng.nflows)]
    out.append(("prior", model.blocks[lvl]["prior"].NN, eng.prior[lvl]))
    return out


def _layer_ref_fp64(feat, geom, sd, i, H, W, act, slope=0.01):
    """nnlayer.py:48-51 in fp64 on the kernel's own layer-i input (teacher-forced):
    act(conv3x3(pad0(W1 x + b1)) + b3), [P, g]."""
    c = geom.a + sum(geom.growth[:i])
    B = feat.shape[0] // (H * W)
    x = feat[:, torch.as_tensor(geom.positions(c))].double().view(B, H, W, c).permute(0, 3, 1, 2)
    w1 = sd[f"layers.{i}.layers.0.weight"].double()
    b1 = sd[f"layers.{i}.layers.0.bias"].double()
    w3 = sd[f"layers.{i}.layers.1.weight"].double()
    b3 = sd[f"layers.{i}.layers.1.bias"].double()
    t = F.conv2d(x, w1, b1)
    h = F.conv2d(t, w3, b3, padding=1)
    h = F.relu(h) if act == "ReLU" else F.leaky_relu(h, slope)
    return h.permute(0, 2, 3, 1).reshape(B * H * W, -1)


def _layer_out(feat, geom, i):
    c0 = geom.k_in[i]
    return feat[:, c0:c0 + geom.growth[i]]


@pytest.mark.parametrize("mode", ["dx3", "x3"])
@pytest.mark.parametrize("lvl", [0, 1, 2])
def test_imagenet64_x3_blocks_teacher_forced(in64, lvl, mode):
    """Every DenseBlock of level `lvl` as the engine packed it, in both split-f16 modes: 'dx3'
    (the default: the direct conv at every level -- 16x16 tiles at 32x32 and 16x16, 2x2 packed
    8x8 images with K split in 4 chunks at 8x8) and 'x3' (Winograd everywhere)."""
    import flow_oracle as FO
    from idfcodec.modules import run_device_block
    model, eng = in64
    eng.set_conv_mode(mode)
    try:
        _x3_blocks_teacher_forced(model, eng, lvl, mode, FO, run_device_block)
    finally:
        eng.set_conv_mode("dx3")


def _x3_blocks_teacher_forced(model, eng, lvl, mode, FO, run_device_block):
    Lv = eng.levels[lvl]
    hw = Lv.h
    g = torch.Generator().manual_seed(100 + lvl)
    worst_block = worst_layer = 0.0
    for name, mod, db in _blocks(model, eng, lvl):
        assert db.desc.wino and db.desc.wx3, (name, "not on the split-f16 path")
        assert db.desc.dx3 == (1 if eng._dx3_level_in(lvl, mode) else 0), (name, mode)
        assert db.desc.dx3 == (1 if mode == "dx3" else 0), (name, mode)  # every level, round 5
        c_in = mod.i_channel
        x = _grid((2, c_in, hw, hw), g)
        sd = {k: v.detach().cpu() for k, v in mod.state_dict().items()}
        eng.clear_range_flag()
        out, feat = run_device_block(db, x.cuda(), return_feat=True)
        torch.cuda.synchronize()
        assert not eng.range_flag_tripped(), (name, "split-f16 range guard tripped")
        ref = FO.dense_block(x, sd, "", mod.depth, mod.act_name)
        e = scaled_err(out, ref)
        worst_block = max(worst_block, e)
        assert e <= TOL, (lvl, name, e)
        featc = feat.cpu()
        for i in range(mod.depth):
            el = scaled_err(_layer_out(featc, db.geom, i),
                            _layer_ref_fp64(featc, db.geom, sd, i, hw, hw, mod.act_name))
            worst_layer = max(worst_layer, el)
            assert el <= TOL, (lvl, name, "layer", i, el)
        # the decoder re-runs the same packed block: bit-identical, and batch-invariant
        again, _ = run_device_block(db, x.cuda())
        assert torch.equal(again, out), (name, "re-run differs")
        one, _ = run_device_block(db, x[1:2].contiguous().cuda())
        assert torch.equal(one, out[1:2]), (name, "image 1 alone differs from inside the batch")
    print(f"{mode} level {lvl}: worst whole-block {worst_block:.2e}, worst layer {worst_layer:.2e}")


@pytest.mark.parametrize("lvl,n_dx3", [(0, 5), (1, 1)])
def test_imagenet64_dx3_prefix_block(in64, lvl, n_dx3):
    """A block packed with dx3 weights for its first n_dx3 layers only (pack_dense_block
    dx3_cmax): dense_block_run runs those on the direct conv over the split copy and the rest
    on wx3 (which reuses the copy's workspace and range-checks its first input) -- teacher-forced
    against flow_oracle and fp64 per layer at 1e-5, re-runs and batch slices bit-exact."""
    import flow_oracle as FO
    from idfcodec.engine import DeviceBlock
    from idfcodec.modules import run_device_block
    from idfcodec.packing import pack_dense_block
    model, eng = in64
    mod = model.blocks[lvl]["flows"][1].dense
    geom0 = eng.couple[lvl][0].geom
    sd_full = model.state_dict()
    pk = pack_dense_block(sd_full, f"blocks.{lvl}.flows.1.dense.", mod.depth, mod.act_name,
                          fold=True, wino=True, wx3=True, dx3=True,
                          dx3_cmax=geom0.k_in[n_dx3 - 1])
    assert len(pk.dx3_w) == n_dx3
    db = DeviceBlock(pk, torch.device("cuda"))
    db.desc.range_flag = eng.range_flag.data_ptr()
    assert db.desc.dx3 == 1
    hw = eng.levels[lvl].h
    g = torch.Generator().manual_seed(400 + lvl)
    x = _grid((3, mod.i_channel, hw, hw), g)
    sd = {k: v.detach().cpu() for k, v in mod.state_dict().items()}
    eng.clear_range_flag()
    out, feat = run_device_block(db, x.cuda(), return_feat=True)
    torch.cuda.synchronize()
    assert not eng.range_flag_tripped()
    assert scaled_err(out, FO.dense_block(x, sd, "", mod.depth, mod.act_name)) <= TOL
    featc = feat.cpu()
    for i in range(mod.depth):
        el = scaled_err(_layer_out(featc, db.geom, i),
                        _layer_ref_fp64(featc, db.geom, sd, i, hw, hw, mod.act_name))
        assert el <= TOL, ("layer", i, el)
    # the all-dx3 and the all-wx3 packings of the same block give other roundings: the
    # prefix block is its own arithmetic, and deterministic
    again, _ = run_device_block(db, x.cuda())
    assert torch.equal(again, out)
    part, _ = run_device_block(db, x[1:3].contiguous().cuda())
    assert torch.equal(part, out[1:3])


def test_imagenet64_x3_blocks_realistic_inputs(in64):
    """The level-0 couplings on the activations the codec actually feeds them (a forward of
    real synthetic images, captured from the engine's coupling inputs) -- the grid inputs
    above are uniform; these carry the image statistics."""
    import flow_oracle as FO
    from idfcodec import synthetic
    from idfcodec.modules import run_device_block
    model, eng = in64
    img = synthetic.images(2, seed=11).cuda()
    x = FO.dequant(img.cpu())
    # the level-0 input after squeeze and the first permutation: a realistic block input
    sq = FO.extend_fwd(x, eng.scale)
    P0 = model.state_dict()["blocks.0.flows.0.P"].detach().cpu()
    xin = FO.permute_fwd(sq, P0)[:, :eng.levels[0].a].contiguous()
    mod = model.blocks[0]["flows"][1].dense
    sd = {k: v.detach().cpu() for k, v in mod.state_dict().items()}
    out, _ = run_device_block(eng.couple[0][0], xin.cuda())
    assert scaled_err(out, FO.dense_block(xin, sd, "", mod.depth, mod.act_name)) <= TOL


@pytest.fixture(scope="module")
def cfg3():
    from idfcodec import configs, synthetic
    model = synthetic.build_model(configs.get("resflow-cond-imagenet64")).cuda()
    model.idf_precision = "bf16"
    eng = model.engine()
    assert eng.precision == "bf16"
    return model, eng


@pytest.mark.parametrize("lvl", [0, 1, 2])
def test_config3_bf16_blocks_teacher_forced(cfg3, lvl):
    """The bf16 DenseBlocks of resflow-cond-imagenet64 as the engine packed them: every layer
    equals an fp64 conv of the bf16-rounded operands (the folded weights the kernel holds,
    the bf16 shadow of its own fp32 layer input) within 1e-5; the head (fp32 GEMM) equals the
    fp64 head of the kernel's features; re-runs and batch invariance are bit-exact.  The
    whole block's distance from the fp32 oracle is the bf16 rounding the config asks for; it
    is reported and bounded loosely."""
    import flow_oracle as FO
    from idfcodec.modules import run_device_block
    model, eng = cfg3
    Lv = eng.levels[lvl]
    hw = Lv.h
    g = torch.Generator().manual_seed(200 + lvl)
    worst_fp32 = 0.0
    for name, mod, db in _blocks(model, eng, lvl):
        assert db.desc.bf16, name
        c_in = mod.i_channel
        x = _grid((2, c_in, hw, hw), g)
        sd = {k: v.detach().cpu() for k, v in mod.state_dict().items()}
        out, feat = run_device_block(db, x.cuda(), return_feat=True)
        featc = feat.cpu()
        geom, pk = db.geom, db.packed
        B, P = 2, 2 * hw * hw
        mask = F.conv2d(torch.ones(1, 1, hw, hw, dtype=torch.float64),
                        torch.eye(9, dtype=torch.float64).view(9, 1, 3, 3), padding=1)
        for i in range(mod.depth):
            k, gi = geom.k_in[i], geom.growth[i]
            xr = featc[:, :k].to(torch.bfloat16).double().view(B, hw, hw, k).permute(0, 3, 1, 2)
            w = torch.from_numpy(pk.w3[i][:gi, :, :k]).to(torch.bfloat16).double()
            w = w.permute(0, 2, 1).reshape(gi, k, 3, 3)
            ref = F.conv2d(xr, w, padding=1) + torch.from_numpy(pk.b3[i][:gi]).double().view(
                1, -1, 1, 1)
            ref = ref + torch.einsum("tn,bthw->bnhw",
                                     torch.from_numpy(pk.vtap[i][:, :gi]).double(), mask)
            ref = F.relu(ref) if mod.act_name == "ReLU" else F.leaky_relu(ref, 0.01)
            ref = ref.permute(0, 2, 3, 1).reshape(P, gi)
            el = scaled_err(_layer_out(featc, geom, i), ref)
            assert el <= TOL, (lvl, name, "layer", i, el)
        n = geom.n_head
        wh = torch.from_numpy(pk.wh[:n, :geom.width]).double()
        head = featc[:, :geom.width].double() @ wh.T + torch.from_numpy(pk.bh[:n]).double()
        got = out.cpu().permute(0, 2, 3, 1).reshape(P, n)
        assert scaled_err(got, head) <= TOL, (lvl, name, "head")
        again, _ = run_device_block(db, x.cuda())
        assert torch.equal(again, out)
        one, _ = run_device_block(db, x[1:2].contiguous().cuda())
        assert torch.equal(one, out[1:2])
        worst_fp32 = max(worst_fp32, scaled_err(out, FO.dense_block(x, sd, "", mod.depth,
                                                                        mod.act_name)))
    print(f"config 3 level {lvl}: whole-block distance from the fp32 oracle {worst_fp32:.2e}")
    assert worst_fp32 <= 5e-3  # measured 5.2e-4 .. 8.4e-4 (bf16 operands through 12 layers)


@pytest.fixture(scope="module")
def cfg45():
    """The flow models of BASELINE configs[3]/[4] as their residual codecs build them."""
    from idfcodec import synthetic
    out = {}
    for name in ("resflows_smallpatch_split", "resflow-patches-vqvae"):
        codec, fl, vq, size = synthetic.build_residual(name)
        out[name] = (fl, fl.engine())
    return out


# config 4: two levels (4x4, 2x2 after the squeezes of 8x8 patches); config 5: one level
# (ExtendDim scale 1 keeps the 27x23 patch)
CFG45_LEVELS = [("resflows_smallpatch_split", 0), ("resflows_smallpatch_split", 1),
                ("resflow-patches-vqvae", 0)]


@pytest.mark.parametrize("name,lvl", CFG45_LEVELS)
def test_config45_x3_blocks_teacher_forced(cfg45, name, lvl):
    """every coupling and prior DenseBlock of configs 4/5 as the engine
    packed them, in x3 mode, whole block teacher-forced against flow_oracle at 1e-5 and every
    layer against fp64 on the kernel's own input; re-runs bit-identical and batch-invariant.
    Config 4 (IDFlows on 8x8 patches): 4x4 / 2x2 levels, the packed-small-image stage, with a
    ragged batch of patches; config 5 (ConditionalFlows on 27x23 patches, ExtendDim scale 1,
    LeakyReLU, 32-channel couplings): the priors see cat(z, cond) (flows.py:278-327)."""
    import flow_oracle as FO
    from idfcodec.modules import run_device_block
    fl, eng = cfg45[name]
    assert len(eng.levels) == {"resflows_smallpatch_split": 2, "resflow-patches-vqvae": 1}[name]
    Lv = eng.levels[lvl]
    H, W = Lv.h, Lv.w
    B = 37 if H * W <= 16 else 3  # a ragged count of packed small patches
    g = torch.Generator().manual_seed(300 + lvl + 17 * len(name))
    worst = 0.0
    # round 5: dx3 at every level -- config 4's 4x4 level (16 patches a tile in segments, 64 /
    # 128 outputs in groups of 4 fragments), its 2x2 level and config 5's 27x23 level (gutter
    # packing: patches at pitch W + 1 / H + 1 sharing one zero column / row)
    want_dx3 = 1
    for bname, mod, db in _blocks(fl, eng, lvl):
        assert db.desc.wino and db.desc.wx3, (name, bname, "not on the split-f16 Winograd path")
        assert db.desc.dx3 == want_dx3, (name, lvl, bname, db.desc.dx3)
        x = _grid((B, mod.i_channel, H, W), g)
        sd = {k: v.detach().cpu() for k, v in mod.state_dict().items()}
        eng.clear_range_flag()
        out, feat = run_device_block(db, x.cuda(), return_feat=True)
        torch.cuda.synchronize()
        assert not eng.range_flag_tripped(), (name, bname, "split-f16 range guard tripped")
        e = scaled_err(out, FO.dense_block(x, sd, "", mod.depth, mod.act_name))
        worst = max(worst, e)
        assert e <= TOL, (name, lvl, bname, e)
        featc = feat.cpu()
        for i in range(mod.depth):
            el = scaled_err(_layer_out(featc, db.geom, i),
                            _layer_ref_fp64(featc, db.geom, sd, i, H, W, mod.act_name))
            assert el <= TOL, (name, lvl, bname, "layer", i, el)
        again, _ = run_device_block(db, x.cuda())
        assert torch.equal(again, out), (bname, "re-run differs")
        part, _ = run_device_block(db, x[1:3].contiguous().cuda())
        assert torch.equal(part, out[1:3]), (bname, "images 1-2 alone differ from the batch")
    print(f"{name} level {lvl} ({H}x{W}, dx3={want_dx3}): worst whole-block {worst:.2e}")


def _sampled_streams_vs_oracle(oracle, fl, rbs, seed, n_pick=24):
    """A sample of a residual bitstream's flow streams equals the C oracle's encode of the
    device's own latents / means / scales (first, last, level boundaries, random)."""
    eng = fl.engine()
    nimg = rbs.flow.n_images
    ws = eng.workspace(nimg)
    lat, mean, scale = (ws[k].cpu().numpy() for k in ("lat", "mean", "scale"))
    off = fl.codec().coder.sym_off(nimg).cpu().numpy()
    st = rbs.flow.states.cpu().numpy().view(np.uint64)
    nw = rbs.flow.nwords.cpu().numpy()
    words = rbs.flow.words.cpu().numpy().view(np.uint32)
    woff = np.concatenate([[0], np.cumsum(nw)[:-1]])
    ns = off.size - 1
    rng = np.random.default_rng(seed)
    pick = np.unique(np.concatenate([[0, ns - 1, nimg - 1, min(nimg, ns - 1)],
                                     rng.integers(0, ns, n_pick)]))
    for k in pick:
        a, b = int(off[k]), int(off[k + 1])
        rs, rw = oracle.encode(1 << 32, lat[a:b], mean[a:b], scale[a:b])
        assert int(st[k]) == rs, k
        assert np.array_equal(words[woff[k]:woff[k] + nw[k]], rw), k
    return len(pick)


@pytest.mark.parametrize("name,src,B", [("resflows_smallpatch_split", (256, 256), 2),
                                        ("resflow-patches-vqvae", (215, 178), 4)])
def test_config45_full_size_streams_vs_oracle(oracle, name, src, B):
    """configs 4/5 at full image size (256x256 -> 1024 8x8 patches per
    image; 215x178 replication-padded to 216x184 -> 64 27x23 patches), the whole residual
    codec in its production modes: sampled flow streams equal the C oracle on the device's
    own latents/means/scales, and the round trip is exact."""
    from idfcodec import synthetic
    codec, fl, vq, size = synthetic.build_residual(name)
    x = synthetic.images(B, H=src[0], W=src[1], seed=23).cuda()
    rbs = codec.encode(x)
    assert rbs.vq_conv == "x3t" and rbs.flow.meta.get("conv") == "dx3"
    n = _sampled_streams_vs_oracle(oracle, fl, rbs, seed=len(name))
    assert n >= 10
    out, info = codec.decode(rbs)
    assert info["ok"] and torch.equal(out, x)


def _fill_ws(eng, ws, d, B):
    """Write the fixture's per-level latents/means/scales into the engine's flat layout
    (level-major, image-minor, NCHW inside)."""
    offs = eng.sym_offsets(B)
    for l in range(len(eng.levels)):
        for key, src in (("lat", "latent"), ("mean", "mean"), ("scale", "scale"),
                         ("logscale", "logscale")):
            ws[key][offs[l]:offs[l + 1]].copy_(torch.from_numpy(d[f"{src}{l}"].reshape(-1)))


def test_reference_imagenet64_streams_on_device_coder(golden, in64):
    """The reference coder's streams for the reference model's own latents/means/scales
    (tests/golden/imagenet64_b2.npz) come out of the device coder bit for bit: per
    (image, level) through StreamCoder.encode exactly as ImageCodec runs it, and they decode
    back to the latents."""
    from test_gpu_rans import _dec_streams
    model, eng = in64
    d = golden("imagenet64_b2.npz")
    B = 2
    ws = eng.workspace(B)
    _fill_ws(eng, ws, d, B)
    bs = model.codec().coder.encode(ws, B)
    st = bs.states.cpu().numpy().view(np.uint64)
    nw = bs.nwords.cpu().numpy()
    words = bs.words.cpu().numpy().view(np.uint32)
    woff = np.concatenate([[0], np.cumsum(nw)[:-1]])
    assert (bs.status.cpu().numpy() & ~32 == 0).all()
    for l in range(3):
        for b in range(B):
            k = l * B + b
            assert int(st[k]) == int(d[f"enc{l}_{b}/state"]), (l, b)
            assert np.array_equal(words[woff[k]:woff[k] + nw[k]], d[f"enc{l}_{b}/words"]), (l, b)
    off = bs.meta.get("scratch_offsets")
    assert off is None  # compacted
    # decode every stream back (device decoder) to the fixture's latents
    sym = np.concatenate([[0], np.cumsum([d[f"latent{l}"][b].size for l in range(3)
                                          for b in range(B)])]).astype(np.int64)
    mean = np.concatenate([d[f"mean{l}"].reshape(-1) for l in range(3)])
    scale = np.concatenate([d[f"scale{l}"].reshape(-1) for l in range(3)])
    fs, out, dst = _dec_streams(sym, woff.astype(np.int64), nw, words, mean, scale, st)
    assert (fs == 1 << 32).all()
    assert np.array_equal(out, np.concatenate([d[f"latent{l}"].reshape(-1) for l in range(3)]))


def test_reference_imagenet64_whole_level_streams(golden):
    """trainer.py:310-315's contract: one stream per level over the whole batch, state reset
    per level -- the device coder reproduces the reference's recorded state, word count and
    word checksum."""
    from test_gpu_rans import _enc_streams
    d = golden("imagenet64_b2.npz")
    for l in range(3):
        x = d[f"latent{l}"].reshape(-1)
        fs, words, nw, st = _enc_streams(np.array([0, x.size]), x, d[f"mean{l}"].reshape(-1),
                                         d[f"scale{l}"].reshape(-1))
        assert int(fs[0]) == int(d[f"enclevel{l}/state"])
        assert int(nw[0]) == int(d[f"enclevel{l}/nwords"])
        assert sum(int(v) for v in words[: nw[0]]) % (1 << 64) == int(d[f"enclevel{l}/wordsum"])


def test_log_likelihood_matches_reference(golden, in64):
    """IDFlows.log_likelihood (flows.py:154-169) / DLogistic.log_prob (distlib.py:40-55) on
    the device, from the reference's own latents/means/logscales: the per-image log_prob
    the reference recorded, within 1e-5."""
    model, _ = in64
    d = golden("imagenet64_b2.npz")
    lat = [torch.from_numpy(d[f"latent{l}"]).cuda() for l in range(3)]
    me = [torch.from_numpy(d[f"mean{l}"]).cuda() for l in range(3)]
    ls = [torch.from_numpy(d[f"logscale{l}"]).cuda() for l in range(3)]
    lp, per_level = model.log_likelihood(lat, me, ls)
    ref = torch.from_numpy(d["log_prob"])
    rel = ((lp.cpu().double() - ref.double()).abs() / ref.double().abs()).max().item()
    assert rel <= 1e-5, rel
    assert len(per_level) == 3 and per_level[0].shape == (2,)
    # the per-symbol form against torch's fp32 ops (the reference's own arithmetic)
    x, m, s = lat[0].cpu(), me[0].cpu(), ls[0].cpu()
    sc = torch.exp(s)
    lpos = F.logsigmoid((x + 0.5 / 256 - m) / sc)
    lneg = F.logsigmoid((x - 0.5 / 256 - m) / sc)
    want = lpos + torch.log(1 - torch.exp(lneg - lpos) + 1e-8)
    got = model.dist.log_prob(lat[0], me[0], ls[0]).cpu()
    assert torch.allclose(got, want, rtol=1e-4, atol=1e-5)
    # the elementwise (grid-stride) launch and the grouped launch write the same logp
    from distlib import dlogistic_log_prob
    grouped = torch.empty_like(lat[0])
    dlogistic_log_prob(lat[0], me[0], ls[0], groups=2, logp=grouped)
    assert torch.equal(got, grouped.cpu())


def test_log_prob_broadcasts_and_validates(in64):
    """DLogistic.log_prob broadcasts like the reference's torch ops (0-dim CPU scalars, a
    [1,C,H,W] mean) and log_likelihood broadcasts per level; malformed inputs raise instead
    of reaching the kernel (distlib.py:36)."""
    from distlib import dlogistic_log_prob
    model, _ = in64
    g = torch.Generator().manual_seed(5)
    xc = torch.randint(0, 256, (2, 3, 8, 8), generator=g).float() / 256
    x = xc.cuda()
    m = xc[:1] + torch.randn(1, 3, 8, 8, generator=g) * 0.02  # one mean for both images
    ls = torch.tensor(-4.0)
    got = model.dist.log_prob(x, m, ls).cpu()
    mc = m.expand(2, 3, 8, 8)
    # bit for bit the launch on explicitly expanded device tensors
    full = model.dist.log_prob(x, mc.contiguous().cuda(), ls.expand(2, 3, 8, 8).contiguous().cuda())
    assert got.shape == (2, 3, 8, 8) and torch.equal(got, full.cpu())
    sc = torch.exp(ls)
    lpos = F.logsigmoid((xc + 0.5 / 256 - mc) / sc)
    lneg = F.logsigmoid((xc - 0.5 / 256 - mc) / sc)
    want = lpos + torch.log(1 - torch.exp(lneg - lpos) + 1e-8)
    near = want > -10  # away from the eps floor, where fp32 cancellation dominates
    assert near.float().mean() > 0.3
    assert torch.allclose(got[near], want[near], rtol=1e-4, atol=1e-5)
    lp, per_level = model.log_likelihood([x], [m.cuda()], [ls.expand(2, 3, 8, 8).cuda()])
    assert torch.allclose(per_level[0].cpu().double() * x[0].numel(),
                          got.double().sum(dim=(1, 2, 3)), rtol=1e-5)
    with pytest.raises(ValueError):
        dlogistic_log_prob(x, m.cuda(), ls.cuda())          # unbroadcast parameters
    with pytest.raises(ValueError):
        dlogistic_log_prob(x, x, x, logp=torch.empty(5, device="cuda"))
    with pytest.raises(ValueError):
        dlogistic_log_prob(x, x, x, logp=torch.empty(x.shape))  # host output


def test_dequant_kernel_all_256_values():
    """idf_dequant_u8 (trainer.py:101) == the oracle's dequant for every uint8 value, and
    idf_quant_u8 inverts it exactly (no off-grid values)."""
    import flow_oracle as FO
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    img = torch.arange(256, dtype=torch.uint8).view(1, 1, 16, 16).repeat(2, 3, 1, 1)
    img[1] = img[1].flip(-1)
    dev = img.cuda()
    out = torch.full((2 * 16 * 16 * 4,), -1.0, device="cuda")
    check(lib().idf_dequant_u8(_lib.stream_ptr(), 2, 3, 16, 16, ptr(dev), ptr(out), 4), "dq")
    got = out.view(2, 16, 16, 4)[..., :3].permute(0, 3, 1, 2).cpu()
    assert torch.equal(got, FO.dequant(img))
    back = torch.empty_like(dev)
    bad = torch.zeros(1, dtype=torch.int32, device="cuda")
    check(lib().idf_quant_u8(_lib.stream_ptr(), 2, 3, 16, 16, ptr(out), 4, ptr(back), ptr(bad)),
          "q")
    assert int(bad.item()) == 0 and torch.equal(back.cpu(), img)


def test_host_c_abi_rans_entries_kat1(golden):
    """idf_rans_encode / idf_rans_decode -- the entries INTEGRATION.md 2 binds for the
    reference's rans.encode / rans.decode -- on KAT1 through ctypes with host
    buffers: state 28772813360, 1102 words equal to the reference's, exact decode."""
    from idfcodec import _lib
    L = _lib.lib()
    d = golden("rans_kat.npz")
    x, m, s = (np.ascontiguousarray(d[f"kat1/{k}"], np.float32) for k in ("x", "mean", "scale"))
    n = x.size
    st = ctypes.c_uint64(1 << 32)
    words = np.zeros(n, np.uint32)
    nw = ctypes.c_int64()
    status = ctypes.c_int32()
    p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    assert L.idf_rans_encode(ctypes.byref(st), n, p(x), p(m), p(s), p(words), ctypes.byref(nw),
                             ctypes.byref(status)) == 0
    assert st.value == 28772813360 and nw.value == 1102 and status.value & ~16 == 0
    assert np.array_equal(words[:nw.value], d["kat1/words"])
    out = np.zeros(n, np.float32)
    w = np.ascontiguousarray(words[:nw.value])
    assert L.idf_rans_decode(ctypes.byref(st), p(w), nw.value, n, p(m), p(s), p(out),
                             ctypes.byref(status)) == 0
    assert st.value == 1 << 32 and np.array_equal(out, x) and status.value == 0
    # the chained-state form (coder.py:18-26): continue from a state, as the reference does
    st = ctypes.c_uint64(1 << 32)
    w0 = np.zeros(20, np.uint32)
    assert L.idf_rans_encode(ctypes.byref(st), 10, p(x), p(m), p(s), p(w0), ctypes.byref(nw),
                             ctypes.byref(status)) == 0
    assert st.value == int(d["chain/state0"]) and np.array_equal(w0[:nw.value], d["chain/words0"])
    # the stream forms: the caller's stream and device workspace (no allocation in the call);
    # an undersized workspace is refused before anything runs
    side = torch.cuda.Stream()
    need = L.idf_rans_host_workspace_bytes(n, 1102)
    assert need >= L.idf_rans_host_workspace_bytes(n, 0) > 0
    ws = torch.empty(need, dtype=torch.uint8, device="cuda")
    st = ctypes.c_uint64(1 << 32)
    words2 = np.zeros(n, np.uint32)
    assert L.idf_rans_encode_on(ctypes.c_void_p(side.cuda_stream), ctypes.c_void_p(ws.data_ptr()),
                                need, ctypes.byref(st), n, p(x), p(m), p(s), p(words2),
                                ctypes.byref(nw), ctypes.byref(status)) == 0
    assert st.value == 28772813360 and np.array_equal(words2[:nw.value], d["kat1/words"])
    out2 = np.zeros(n, np.float32)
    assert L.idf_rans_decode_on(ctypes.c_void_p(side.cuda_stream), ctypes.c_void_p(ws.data_ptr()),
                                need, ctypes.byref(st), p(w), 1102, n, p(m), p(s), p(out2),
                                ctypes.byref(status)) == 0
    assert st.value == 1 << 32 and np.array_equal(out2, x)
    st = ctypes.c_uint64(1 << 32)
    assert L.idf_rans_decode_on(ctypes.c_void_p(side.cuda_stream), ctypes.c_void_p(ws.data_ptr()),
                                need - 1, ctypes.byref(st), p(w), 1102, n, p(m), p(s), p(out2),
                                ctypes.byref(status)) != 0
    assert st.value == 1 << 32


def test_config3_full_batch_1024(oracle):
    """BASELINE configs[2] at its own batch size (B=1024, bf16 coupling convs): exact round
    trip of the whole residual codec, and a sample of its flow streams equal the C oracle on
    the device's own latents/means/scales (the 32-bit offset arithmetic of the ~2.3 GB
    feature buffers is exercised at this size)."""
    from idfcodec import synthetic
    codec, fl, vq, size = synthetic.build_residual("resflow-cond-imagenet64")
    assert fl.engine().precision == "bf16"
    B = 1024
    x = synthetic.images(B, H=size[0], W=size[1], seed=21).cuda()
    rbs = codec.encode(x)
    _sampled_streams_vs_oracle(oracle, fl, rbs, seed=5)
    out, info = codec.decode(rbs)
    assert info["ok"] and torch.equal(out, x)


def test_bench_config_b256_streams_vs_oracle(oracle, in64):
    """BASELINE configs[1] at its own batch (imagenet64, B = 256, the bench's workload): the
    codec's encode in its production mode (dx3 + x3 convs, side-stream level encode, lanes)
    -- a sample of its 768 (level, image) streams equal the C oracle's encode of the device's
    own latents / means / scales word for word, and the decode restores the images exactly."""
    from idfcodec import synthetic
    model, eng = in64
    codec = model.codec()
    B = 256
    img = synthetic.images(B, seed=31).cuda()
    bs = codec.encode(img)
    torch.cuda.synchronize()
    assert bs.meta.get("conv") == "dx3"
    ws = eng.workspace(B)
    lat, mean, scale = (ws[k].cpu().numpy() for k in ("lat", "mean", "scale"))
    off = codec.coder.sym_off(B).cpu().numpy()
    st = bs.states.cpu().numpy().view(np.uint64)
    nw = bs.nwords.cpu().numpy()
    words = bs.words.cpu().numpy().view(np.uint32)
    woff = np.concatenate([[0], np.cumsum(nw)[:-1]])
    ns = off.size - 1
    assert ns == 3 * B
    rng = np.random.default_rng(256)
    pick = np.unique(np.concatenate([[0, B - 1, B, 2 * B - 1, 2 * B, ns - 1],
                                     rng.integers(0, ns, 26)]))
    for k in pick:
        a, b = int(off[k]), int(off[k + 1])
        rs, rw = oracle.encode(1 << 32, lat[a:b], mean[a:b], scale[a:b])
        assert int(st[k]) == rs, k
        assert np.array_equal(words[woff[k]:woff[k] + nw[k]], rw), k
    out, info = codec.decode(bs)
    assert info["ok"] and torch.equal(out, img)
