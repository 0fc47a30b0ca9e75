"""End-to-end codec on the GPU: per-(image, level) streams bit-identical to the
oracle on the device's own (x, mean, scale); exact uint8 round trip at the
BASELINE sizes (imagenet64 B=256, config 2)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _imagenet64():
    from idfcodec import configs, synthetic
    return synthetic.build_model(configs.get("imagenet64")).cuda()


def _check_streams_vs_oracle(model, B, oracle, sample=None):
    codec = model.codec()
    eng = model.engine()
    ws = eng.workspace(B)
    off = codec.coder.sym_off(B).cpu().numpy()
    lat, mean, scale = (ws[k][: off[-1]].cpu().numpy() for k in ("lat", "mean", "scale"))
    return off, lat, mean, scale


@pytest.mark.parametrize("B", [1, 3, 16])
def test_streams_bit_identical_and_round_trip(oracle, B):
    from idfcodec import synthetic
    model = _imagenet64()
    img = synthetic.images(B, seed=10 + B).cuda()
    codec = model.codec()
    bs = codec.encode(img, compact=False)
    off, lat, mean, scale = _check_streams_vs_oracle(model, B, oracle)
    fs, words, nw, st = oracle.encode_streams(off, lat, mean, scale)
    assert (st == 0).all()
    assert np.array_equal(bs.states.cpu().numpy().view(np.uint64), fs)
    assert np.array_equal(bs.nwords.cpu().numpy(), nw)
    gw = bs.words.cpu().numpy().view(np.uint32)
    for k in range(off.size - 1):
        assert np.array_equal(gw[off[k]:off[k] + nw[k]], words[off[k]:off[k] + nw[k]])
    out, info = codec.decode(codec.encode(img))
    assert info["ok"] and torch.equal(out, img)


def test_baseline_config2_round_trip_b256():
    """BASELINE config 2: imagenet64, B=256 synthetic uint8, fp32 flow + HIP rANS."""
    from idfcodec import synthetic
    from idfcodec.codec import Bitstream
    model = _imagenet64()
    img = synthetic.images(256).cuda()
    codec = model.codec()
    bs = codec.encode(img)
    assert bs.n_streams == 768
    assert int((bs.status != 0).sum()) == 0
    raw = bs.to_bytes()
    bs2 = Bitstream.from_bytes(raw, device="cuda")
    out, info = codec.decode(bs2)
    assert info["ok"], {k: v for k, v in info.items() if k != "final_states"}
    assert torch.equal(out, img)
    bpd = bs.bpd()
    assert 3.0 < bpd < 16.0


def test_encode_deterministic_and_batch_invariant():
    """same image coded alone or inside a batch -> identical stream (decoder and
    encoder may run different batch compositions)."""
    from idfcodec import synthetic
    model = _imagenet64()
    img = synthetic.images(5, seed=3).cuda()
    codec = model.codec()
    a = codec.encode(img)
    b = codec.encode(img)
    assert torch.equal(a.words, b.words) and torch.equal(a.states, b.states)
    one = codec.encode(img[2:3])
    for l in range(3):
        k = l * 5 + 2
        assert int(one.states[l]) == int(a.states[k])
        woff = a.word_offsets()
        ooff = one.word_offsets()
        assert torch.equal(a.words[woff[k]: woff[k] + a.nwords[k]],
                           one.words[ooff[l]: ooff[l] + one.nwords[l]])


@pytest.mark.parametrize("name", ["t3_cond_convcond", "t4_cond_s1_odd"])
def test_conditional_codec_round_trip(golden, name):
    import yaml
    from idfcodec import synthetic
    d = golden(f"flow_{name}.npz")
    cfg = yaml.safe_load(bytes(d["cfg_yaml"]).decode())
    model = synthetic.build_model(cfg).cuda()
    B, H, W = 4, cfg["H"], cfg["W"]
    img = synthetic.images(B, 3, H, W, seed=9).cuda()
    cond = torch.round(torch.rand(B, 3, H, W, generator=torch.Generator().manual_seed(4)) * 256).cuda() / 256
    bs = model.encode(img, cond)
    out, info = model.decode(bs, cond)
    assert info["ok"] and torch.equal(out, img)


def test_coder_api_chained_round_trip(golden):
    """coder.Encode (bit-identical chaining) + fixed coder.Decode round trip on device."""
    import coder
    d = golden("imagenet64_b2.npz")
    lat = [torch.from_numpy(d[f"latent{i}"]).cuda() for i in range(3)]
    mean = [torch.from_numpy(d[f"mean{i}"]).cuda() for i in range(3)]
    logs = [torch.from_numpy(d[f"logscale{i}"]).cuda() for i in range(3)]
    x, bufs = coder.Encode(lat, mean, logs)
    x2, rec = coder.Decode(bufs, mean, logs, x)
    assert x2 == 1 << 32
    for a, b in zip(rec, lat):
        assert torch.equal(a, b)


def test_conv_modes_and_range_guard_fallback(monkeypatch):
    """imagenet64 runs the split-f16 direct convs at every level (conv 'dx3'; 'dx3w16' is
    round 4's: direct at 32x32 / 16x16, Winograd at 8x8, container code 6); a bitstream records
    the conv mode, the decoder follows it whatever mode the engine is in (dx3 / dx3w16 / x3 /
    f32), and a tripped range guard re-encodes the batch with the exact-f32 convs."""
    from idfcodec import synthetic
    from idfcodec.codec import Bitstream
    model = _imagenet64()
    codec = model.codec()
    eng = model.engine()
    assert eng.conv_mode == "dx3"
    img = synthetic.images(4, seed=77).cuda()
    bs_dx3 = codec.encode(img)
    assert bs_dx3.meta["conv"] == "dx3"
    eng.set_conv_mode("x3")
    bs_x3 = codec.encode(img)
    assert bs_x3.meta["conv"] == "x3"
    eng.set_conv_mode("f32")
    bs_f32 = codec.encode(img)
    assert bs_f32.meta["conv"] == "f32"
    eng.set_conv_mode("dx3w16")
    bs_w16 = codec.encode(img)
    assert bs_w16.meta["conv"] == "dx3w16"
    assert Bitstream.from_bytes(bs_w16.to_bytes()).meta["conv"] == "dx3w16"
    eng.set_conv_mode("dx3")
    # the modes give (slightly) different couplings, so different streams, all lossless
    for a_, b_ in ((bs_dx3, bs_x3), (bs_x3, bs_f32), (bs_dx3, bs_f32), (bs_dx3, bs_w16)):
        assert not (torch.equal(a_.states, b_.states) and torch.equal(a_.words, b_.words))
    for bs in (bs_dx3, bs_x3, bs_f32, bs_w16, Bitstream.from_bytes(bs_f32.to_bytes(), "cuda"),
               Bitstream.from_bytes(bs_x3.to_bytes(), "cuda"),
               Bitstream.from_bytes(bs_dx3.to_bytes(), "cuda"),
               Bitstream.from_bytes(bs_w16.to_bytes(), "cuda")):
        out, info = codec.decode(bs)
        assert info["ok"] and torch.equal(out.cpu(), img.cpu()), bs.meta
        assert eng.conv_mode == "dx3"
    # guard tripped -> exact-f32 re-encode, identical to an f32-mode encode
    monkeypatch.setattr(type(eng), "range_flag_tripped", lambda self: True)
    bs_fb = codec.encode(img)
    assert bs_fb.meta["conv"] == "f32" and eng.conv_mode == "dx3"
    assert torch.equal(bs_fb.states, bs_f32.states) and torch.equal(bs_fb.words, bs_f32.words)


def test_range_guard_clean_on_real_batch():
    """The guard must not trip on the benchmark workload (else every batch pays twice)."""
    from idfcodec import synthetic
    model = _imagenet64()
    codec = model.codec()
    eng = model.engine()
    eng.clear_range_flag()
    bs = codec.encode(synthetic.images(64, seed=5).cuda())
    assert bs.meta["conv"] == "dx3" and not eng.range_flag_tripped()


@pytest.mark.parametrize("fixture,conv", [("imagenet64_code6_r4.npz", "dx3w16"),
                                          ("imagenet64_code7_r5.npz", "dx3"),
                                          ("config3_code8_r5.npz", "dxb")])
def test_earlier_build_bitstreams_decode_exactly(golden, fixture, conv):
    """Bitstreams written by earlier builds themselves (tests/golden/make_conv_fixture.py): conv
    code 6 at 23b932c (round 4's dx3 at the 16-wide levels, read today as "dx3w16"), code 7 and
    code 8 at 92c5486 (round 5's dx3 and dxb, the latter inside a config-3 residual bitstream)
    decode with today's library to the exact images: each recorded conv code still names the
    arithmetic it was written with, bit for bit."""
    from idfcodec import configs, synthetic
    from idfcodec.codec import Bitstream
    from idfcodec.residual import ResidualBitstream
    d = golden(fixture)
    raw = d["bitstream"].tobytes()
    if fixture.startswith("imagenet64"):
        bs = Bitstream.from_bytes(raw)
        assert bs.meta["conv"] == conv
        out, info = _imagenet64().codec().decode(bs)
    else:
        name = str(d["config"])
        rbs = ResidualBitstream.from_bytes(raw)
        assert rbs.flow.meta["conv"] == conv
        codec, _, _, _ = synthetic.build_residual(name)
        out, info = codec.decode(rbs)
    assert info["ok"], info
    assert torch.equal(out.cpu(), torch.from_numpy(d["images"])), "an earlier file decodes wrong"
