"""GPU end-to-end lossless round trips of the residual configs' codec (idfcodec.residual:
VQ-VAE indices + reconstruction, residual through the flow model over patches, rANS,
fixed-width index code), on small synthetic models (conditional and plain flows, with and
without patching) and on the config-3/4/5 models at full size (config 5 from its 215x178
source through the dataloader's replication pad)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _vq_small(hidden, K=64, D=16, nb=1):
    from idfcodec import synthetic
    blk = {"name": "ResBlock", "batch_norm": False}
    return synthetic.build_vqvae({
        "name": "VQVAE", "channel": 3, "embed_num": K, "embed_dim": D,
        "encoder": {"name": "VQEncoder", "block_num": nb, "block": dict(blk)},
        "decoder": {"name": "VQDecoder", "block_num": nb, "block": dict(blk)},
        "distribution": {"name": "BinomialDistribution"}, "hidden_dims": hidden}).cuda()


def _flows(name, H, W, nsplit, scale=2, **extra):
    from idfcodec import synthetic
    from idfcodec.configs import _dense, _flows
    return synthetic.build_model(_flows(name, 2, nsplit, H, W, 3, _dense(24, 3), _dense(16, 2),
                                        scale, **extra)).cuda()


@pytest.mark.parametrize("kind,img,patch", [
    ("cond_conv", (32, 32), (32, 32)),      # config-3 shape: one patch per image
    ("plain", (32, 32), (16, 16)),          # config-4 shape: IDFlows over patches
    ("cond_s1", (24, 32), (12, 8)),         # config-5 shape: ExtendDim scale 1, odd-ish patches
])
def test_residual_round_trip_small(kind, img, patch):
    from idfcodec import synthetic
    from idfcodec.residual import ResidualBitstream, ResidualCodec
    H, W = img
    h, w = patch
    if kind == "cond_conv":
        fl = _flows("ConditionalFlows", h, w, 2, conv_for_cond=True)
    elif kind == "plain":
        fl = _flows("IDFlows", h, w, 2)
    else:
        fl = _flows("ConditionalFlows", h, w, 1, scale=1, conv_for_cond=False)
    vq = _vq_small([8, 16])
    codec = ResidualCodec(fl, vq, (H, W))
    x = synthetic.images(3, H=H, W=W, seed=21).cuda()
    rbs = codec.encode(x)
    assert rbs.vq_conv == "x3t"  # every VQ conv ran split-f16, guard not tripped
    raw = rbs.to_bytes()
    rbs2 = ResidualBitstream.from_bytes(raw, device="cuda")
    assert rbs2.vq_conv == "x3t"
    out, info = codec.decode(rbs2)
    assert info["ok"], info
    assert torch.equal(out, x)
    assert rbs.bits() > 0 and rbs.index_bits == 6
    # an "x3" (round 5's: split-f16 ResBlocks only) or exact-f32 VQ encode is recorded as such
    # and decodes exactly on the same engine
    eng = vq.engine()
    for mode in ("x3", "f32"):
        eng.conv_mode = mode
        try:
            r32 = codec.encode(x)
        finally:
            eng.conv_mode = "x3t"
        assert r32.vq_conv == mode
        out, info = codec.decode(ResidualBitstream.from_bytes(r32.to_bytes(), device="cuda"))
        assert info["ok"] and torch.equal(out, x)


def test_config3_round_trip():
    """resflow-cond-imagenet64 (BASELINE configs[2]) at its full model sizes, B=2."""
    from idfcodec import synthetic
    from idfcodec.residual import ResidualBitstream
    codec, fl, vq, size = synthetic.build_residual("resflow-cond-imagenet64")
    x = synthetic.images(2, H=size[0], W=size[1], seed=4).cuda()
    rbs = codec.encode(x)
    out, info = codec.decode(ResidualBitstream.from_bytes(rbs.to_bytes(), device="cuda"))
    assert info["ok"] and torch.equal(out, x)
    assert rbs.index_bits == 14


def test_residual_shards_merge_to_one_bitstream():
    """Two shards coded separately (the per-rank work of configs 4/5) merge into the
    bitstream of the whole batch (idfcodec.dist.merge_residual, the core of gather_residual)."""
    from idfcodec import synthetic
    from idfcodec.dist import merge_residual
    from idfcodec.residual import ResidualCodec
    fl = _flows("IDFlows", 16, 16, 2)
    vq = _vq_small([8, 16], K=100)       # 7-bit indices: runs not word-aligned per index
    codec = ResidualCodec(fl, vq, (32, 32))
    x = synthetic.images(4, H=32, W=32, seed=33).cuda()
    parts = [codec.encode(x[:2]), codec.encode(x[2:])]
    merged = merge_residual(parts)
    out, info = codec.decode(merged)
    assert info["ok"] and torch.equal(out, x)
    whole = codec.encode(x)
    assert torch.equal(merged.idx_words.cpu(), whole.idx_words.cpu())
    assert torch.equal(merged.flow.states.cpu(), whole.flow.states.cpu())


@pytest.mark.parametrize("Hi,Wi,Ho,Wo", [(215, 178, 216, 184), (5, 3, 5, 9), (7, 7, 7, 7),
                                         (216, 184, 215, 178)])
def test_pad_edge_matches_replication_pad(Hi, Wi, Ho, Wo):
    """idf_pad_edge_u8 == nn.ReplicationPad2d((0, right, 0, bottom)) (trainer.py:62) and,
    shrinking, the crop that undoes it."""
    from idfcodec import _lib, synthetic
    from idfcodec._lib import check, lib, ptr
    x = synthetic.images(2, H=Hi, W=Wi, seed=5).cuda()
    out = torch.empty((2, 3, Ho, Wo), dtype=torch.uint8, device="cuda")
    check(lib().idf_pad_edge_u8(_lib.stream_ptr(x.device), 2, 3, Hi, Wi, Ho, Wo, ptr(x), ptr(out)),
          "pad")
    if Ho >= Hi:
        ref = torch.nn.ReplicationPad2d((0, Wo - Wi, 0, Ho - Hi))(x.cpu().float()).to(torch.uint8)
    else:
        ref = x.cpu()[:, :, :Ho, :Wo]
    assert torch.equal(out.cpu(), ref)


def test_residual_round_trip_with_source_pad():
    """A codec with pad=(bottom, right) takes the unpadded source, codes the replication-
    padded image (what the reference's dataloader hands its trainer) and returns the source."""
    from idfcodec import synthetic
    from idfcodec.residual import ResidualBitstream, ResidualCodec
    fl = _flows("ConditionalFlows", 12, 8, 1, scale=1, conv_for_cond=False)
    codec = ResidualCodec(fl, _vq_small([8, 16]), (24, 32), pad=(1, 6))
    x = synthetic.images(2, H=23, W=26, seed=8).cuda()
    rbs = codec.encode(x)
    assert rbs.source_hw == (23, 26) and rbs.image_shape == (3, 24, 32)
    out, info = codec.decode(ResidualBitstream.from_bytes(rbs.to_bytes(), device="cuda"))
    assert info["ok"] and torch.equal(out, x)
    padded = torch.nn.ReplicationPad2d((0, 6, 0, 1))(x.cpu().float()).to(torch.uint8).cuda()
    same = codec.encode(padded)          # the padded image codes to the same streams
    assert same.source_hw is None and torch.equal(same.idx_words, rbs.idx_words)
    assert torch.equal(same.flow.words, rbs.flow.words)
    with pytest.raises(ValueError):
        codec.encode(synthetic.images(1, H=20, W=20, seed=1).cuda())


@pytest.mark.parametrize("name,src", [("resflows_smallpatch_split", (256, 256)),
                                      ("resflow-patches-vqvae", (215, 178))])
def test_config45_round_trip_full_size(name, src):
    """BASELINE configs[3]/[4] at their full model and image sizes, one image each:
    1024 8x8 patches of a 256x256 image (IDFlows), and 64 27x23 patches of a 215x178 image
    replication-padded to 216x184 (ConditionalFlows, ExtendDim scale 1)."""
    from idfcodec import synthetic
    from idfcodec.residual import ResidualBitstream
    codec, fl, vq, size = synthetic.build_residual(name)
    x = synthetic.images(1, H=src[0], W=src[1], seed=6).cuda()
    rbs = codec.encode(x)
    assert rbs.image_shape == (3,) + tuple(size) and rbs.index_bits == 13
    out, info = codec.decode(ResidualBitstream.from_bytes(rbs.to_bytes(), device="cuda"))
    assert info["ok"] and torch.equal(out, x)
