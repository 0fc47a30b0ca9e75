"""GPU end-to-end lossless round trips of the residual configs' codec (idfcodec.residual:
VQ-VAE indices + reconstruction, residual through the flow model over patches, rANS,
fixed-width index code), on small synthetic models (conditional and plain flows, with and
without patching) and on the config-3 model (resflow-cond-imagenet64) at full size."""
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
    raw = rbs.to_bytes()
    rbs2 = ResidualBitstream.from_bytes(raw, device="cuda")
    out, info = codec.decode(rbs2)
    assert info["ok"], info
    assert torch.equal(out, x)
    assert rbs.bits() > 0 and rbs.index_bits == 6


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
