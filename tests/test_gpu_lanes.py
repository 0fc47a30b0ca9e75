"""Decode lanes (ImageCodec: sub-batches on their own HIP streams, staggered so one lane's
serial rANS decode runs beside another lane's flow convs) must give exactly the single-lane
decode: same pixels, same final rANS states, same stream status."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _decode_all(codec, bs, lanes, cond=None):
    codec.lanes = lanes
    out, info = codec.decode(bs, cond=cond) if cond is not None else codec.decode(bs)
    torch.cuda.synchronize()
    return out, info


@pytest.mark.parametrize("B", [16, 18, 32])
def test_lanes_decode_identical(B):
    from idfcodec import configs, synthetic
    from idfcodec.codec import Bitstream
    model = synthetic.build_model(configs.get("imagenet64")).cuda()
    codec = model.codec()
    img = synthetic.images(B, seed=40 + B).cuda()
    bs = codec.encode(img)
    ref, rinfo = _decode_all(codec, bs, 1)
    assert rinfo["ok"] and torch.equal(ref, img)
    for lanes in (2, 4):
        assert codec._n_lanes(B) >= 1
        out, info = _decode_all(codec, bs, lanes)
        assert info["ok"], lanes
        assert torch.equal(out, img), lanes
        assert torch.equal(info["final_states"], rinfo["final_states"])
        assert torch.equal(info["status"], rinfo["status"])
    # unequal lanes (IDF_LANE_SPLIT) under each cross-lane order (IDF_LANE_STAGGER)
    import os
    saved = {k: os.environ.get(k) for k in ("IDF_LANE_SPLIT", "IDF_LANE_STAGGER")}
    try:
        for split, stagger in (("0.375", "levels"), ("0.375", "top"), ("0.625", "none"),
                               ("0.5", "flows"), ("0.625", "flows0")):
            os.environ["IDF_LANE_SPLIT"], os.environ["IDF_LANE_STAGGER"] = split, stagger
            out, info = _decode_all(codec, bs, 2)
            assert info["ok"] and torch.equal(out, img), (split, stagger)
            assert torch.equal(info["final_states"], rinfo["final_states"])
            assert torch.equal(info["status"], rinfo["status"])
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    # through the container, with the non-compact (scratch-offset) bitstream as well
    bs2 = Bitstream.from_bytes(bs.to_bytes(), device="cuda")
    out, info = _decode_all(codec, bs2, 2)
    assert info["ok"] and torch.equal(out, img)
    raw = codec.encode(img, compact=False)
    out, info = _decode_all(codec, raw, 2)
    assert info["ok"] and torch.equal(out, img)
    codec.lanes = 2


def test_lanes_conditional_decode_identical(golden):
    import yaml
    from idfcodec import synthetic
    d = golden("flow_t3_cond_convcond.npz")
    cfg = yaml.safe_load(bytes(d["cfg_yaml"]).decode())
    model = synthetic.build_model(cfg).cuda()
    B, H, W = 16, cfg["H"], cfg["W"]
    img = synthetic.images(B, 3, H, W, seed=19).cuda()
    cond = torch.round(torch.rand(B, 3, H, W, generator=torch.Generator().manual_seed(5))
                       * 256).cuda() / 256
    codec = model.codec()
    bs = model.encode(img, cond)
    ref, rinfo = _decode_all(codec, bs, 1, cond)
    out, info = _decode_all(codec, bs, 2, cond)
    assert rinfo["ok"] and info["ok"]
    assert torch.equal(ref, img) and torch.equal(out, img)
    assert torch.equal(info["final_states"], rinfo["final_states"])
    codec.lanes = 2


@pytest.mark.parametrize("B", [3, 32])
def test_overlapped_level_encode_identical(B):
    """Per-level rANS encode on a side stream (overlapped with the next levels' flow) gives
    the bitstream of the one-pass encode, compact and not."""
    from idfcodec import configs, synthetic
    model = synthetic.build_model(configs.get("imagenet64")).cuda()
    codec = model.codec()
    img = synthetic.images(B, seed=70 + B).cuda()
    codec.overlap_encode = False
    ref = codec.encode(img)
    ref_raw = codec.encode(img, compact=False)
    ref_raw = (ref_raw.states.clone(), ref_raw.nwords.clone(), ref_raw.status.clone())
    codec.overlap_encode = True
    got = codec.encode(img)
    torch.cuda.synchronize()
    assert torch.equal(got.states, ref.states) and torch.equal(got.nwords, ref.nwords)
    assert torch.equal(got.words, ref.words)
    assert torch.equal(got.status, ref.status)
    raw = codec.encode(img, compact=False)
    assert torch.equal(raw.states, ref_raw[0]) and torch.equal(raw.nwords, ref_raw[1])
    out, info = codec.decode(got)
    assert info["ok"] and torch.equal(out, img)


@pytest.mark.parametrize("B,lanes", [(16, 2), (48, 2), (64, 4), (18, 2)])
def test_encode_lanes_identical(B, lanes):
    """Encode lanes (IDF_ENC_LANES): the flow as sub-batches on the lanes' streams, each lane
    rANS-encoding its images' streams into the shared arrays -- the bitstream must equal the
    one-lane encode's bit for bit (states, word counts, words, status), compact or not, and
    decode exactly."""
    from idfcodec import configs, synthetic
    model = synthetic.build_model(configs.get("imagenet64")).cuda()
    codec = model.codec()
    img = synthetic.images(B, seed=70 + B).cuda()
    codec.enc_lanes = 1
    ref = codec.encode(img)
    ref_raw = codec.encode(img, compact=False)
    codec.enc_lanes = lanes
    try:
        got = codec.encode(img)
        got_raw = codec.encode(img, compact=False)
    finally:
        codec.enc_lanes = 1
    torch.cuda.synchronize()
    for a, b in ((got, ref), (got_raw, ref_raw)):
        assert torch.equal(a.states, b.states)
        assert torch.equal(a.nwords, b.nwords)
        assert torch.equal(a.status, b.status)
    assert torch.equal(got.words, ref.words)
    n = int(ref_raw.nwords.sum())
    off = ref_raw.meta["scratch_offsets"]
    for k in range(0, ref_raw.nwords.numel(), max(1, ref_raw.nwords.numel() // 7)):
        o, m = int(off[k]), int(ref_raw.nwords[k])
        assert torch.equal(got_raw.words[o:o + m], ref_raw.words[o:o + m]), k
    assert n > 0
    out, info = codec.decode(got)
    assert info["ok"] and torch.equal(out, img)


def test_encode_beside_decode_exact():
    """bench.py --pipeline 1: batch A's decode (its own stream, the lanes' workspaces) runs
    while batch B is encoded on another stream in workspace slot ENC_SLOT.  A decodes exactly,
    and B's bitstream is bit-identical to B encoded alone."""
    from idfcodec import _lib, configs, synthetic
    model = synthetic.build_model(configs.get("imagenet64")).cuda()
    codec = model.codec()
    a = synthetic.images(32, seed=71).cuda()
    b = synthetic.images(32, seed=72).cuda()
    bs_a = codec.encode(a)
    ref_b = codec.encode(b)
    torch.cuda.synchronize()
    E, D = _lib.new_stream(), _lib.new_stream()
    done_a = torch.cuda.Event()
    done_a.record()
    for _ in range(2):  # the second time with every cache warm
        with torch.cuda.stream(D):
            D.wait_event(done_a)
            out_a, info_a = codec.decode(bs_a, verify=False)
        with torch.cuda.stream(E):
            bs_b = codec.encode(b, slot=codec.ENC_SLOT)
        torch.cuda.synchronize()
        assert torch.equal(out_a, a)
        assert bool((info_a["final_states"] == 1 << 32).all())
        assert torch.equal(bs_b.states, ref_b.states) and torch.equal(bs_b.nwords, ref_b.nwords)
        assert torch.equal(bs_b.words, ref_b.words) and bs_b.meta["conv"] == ref_b.meta["conv"]


def test_encode_fallback_beside_decode_exact(monkeypatch):
    """The range guard's f32 recompute inside an encode on stream E (forced here) switches the
    engine's conv mode while batch A's decode on stream D still has queued copies of the dx3
    top prior: the per-mode top-prior cache keeps that tensor alive, so A decodes exactly and
    B's bitstream equals B encoded alone in f32."""
    from idfcodec import _lib, configs, synthetic
    model = synthetic.build_model(configs.get("imagenet64")).cuda()
    codec = model.codec()
    eng = model.engine()
    a = synthetic.images(32, seed=81).cuda()
    b = synthetic.images(32, seed=82).cuda()
    bs_a = codec.encode(a)
    assert bs_a.meta["conv"] == eng.conv_mode != "f32"
    mode = eng.conv_mode
    eng.set_conv_mode("f32")
    ref_b = codec.encode(b)
    eng.set_conv_mode(mode)
    assert ref_b.meta["conv"] == "f32"
    torch.cuda.synchronize()
    E, D = _lib.new_stream(), _lib.new_stream()
    done_a = torch.cuda.Event()
    done_a.record()
    monkeypatch.setattr(type(eng), "range_flag_tripped", lambda self: True)
    for _ in range(2):
        with torch.cuda.stream(D):
            D.wait_event(done_a)
            out_a, info_a = codec.decode(bs_a, verify=False)
        with torch.cuda.stream(E):
            bs_b = codec.encode(b, slot=codec.ENC_SLOT)
        torch.cuda.synchronize()
        assert eng.conv_mode == mode
        assert torch.equal(out_a, a)
        assert bool((info_a["final_states"] == 1 << 32).all())
        assert bs_b.meta["conv"] == "f32"
        assert torch.equal(bs_b.states, ref_b.states) and torch.equal(bs_b.words, ref_b.words)


@pytest.mark.parametrize("name,lvl,which", [("resflow-patches-vqvae", 0, "coupling"),
                                            ("resflow-patches-vqvae", 0, "prior"),
                                            ("resflows_smallpatch_split", 0, "coupling"),
                                            ("resflows_smallpatch_split", 1, "coupling"),
                                            ("resflow-cond-imagenet64", 0, "coupling")])
def test_fused_blocks_two_streams(name, lvl, which):
    """A dense block with the fused head (dx3 layers + idf_dx3_head_init) run on two HIP streams
    at once, each on its own workspace, gives the bits it gives alone: what two decode lanes
    do.  (A head init staging its weights in LDS diverged here in 5-20 of 40 runs.)"""
    from idfcodec import _lib, configs, synthetic
    from idfcodec._lib import IdfHeadOut, ptr
    model = synthetic.build_model(configs.get(name)).cuda()
    model.idf_precision = configs.PRECISION.get(name, "f32")  # config 3: bf16 (dxb)
    eng = model.engine()
    Lv = eng.levels[lvl]
    blk = eng.couple[lvl][0] if which == "coupling" else eng.prior[lvl]
    assert blk.desc.fuse_head == 1 and (blk.desc.dx3 == 1 or blk.desc.dxb == 1)
    B = 64
    P = B * Lv.h * Lv.w
    k0 = blk.geom.k_in[0]
    g = torch.Generator().manual_seed(5)

    def setup(slot):
        ws = eng.workspace(B, slot)
        x = (torch.randint(-64, 64, (P, k0), generator=g).float() / 256).cuda()
        if which == "coupling":
            x[:, Lv.a:] = 0.0  # the pad columns past a_ch
        return ws, x, torch.zeros(P, 16, device="cuda")

    def run(ws, x, out):
        ws["feat"].view(-1, eng.ld_feat)[:P, :k0] = x
        h = IdfHeadOut()
        h.mode, h.out, h.ld_out = _lib.EPI_STORE, ptr(out), 16
        blk.run(_lib.stream_ptr(), B, Lv.h, Lv.w, ptr(ws["feat"]), eng.ld_feat, ptr(ws["tmp"]),
                eng.tmp_pitch(ws, P), h)

    sets = [setup(1), setup(2)]
    refs = []
    for ws, x, out in sets:
        run(ws, x, out)
        torch.cuda.synchronize()
        refs.append(out.clone())
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for rep in range(20):
        for _, _, out in sets:
            out.zero_()
        torch.cuda.synchronize()
        for st, (ws, x, out) in zip(streams, sets):
            with torch.cuda.stream(st):
                run(ws, x, out)
        torch.cuda.synchronize()
        for i, (_, _, out) in enumerate(sets):
            assert torch.equal(out, refs[i]), (rep, i, int((out != refs[i]).any(1).sum()))
