"""Host-side logic on CPU: C-ABI exports, weight packing, mirror modules,
bitstream container, coder chaining, expf restatement (exhaustive)."""
import os
import re
import subprocess

import numpy as np
import pytest
import torch
import torch.nn.functional as F
import yaml

from conftest import PKG, REPO


# ------------------------------------------------------------------ C ABI
def _header_functions():
    src = open(os.path.join(REPO, "include", "idf_codec.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[A-Za-z_0-9]+\s*\*?\s*(idf_[a-z0-9_]+)\s*\(", src,
                                 flags=re.M)))


def test_library_exports_every_declared_symbol():
    import ctypes
    from idfcodec import _lib
    names = _header_functions()
    assert len(names) >= 20
    L = ctypes.CDLL(_lib.LIB_PATH)
    for n in names:
        assert hasattr(L, n), f"{n} declared in include/idf_codec.h but not exported"
    assert set(names) == set(_lib.SIGNATURES), "ctypes signatures out of sync with the header"
    lib = _lib.lib()
    assert lib.idf_version().decode().startswith("idfcodec")


def test_fused_head_tmp_is_required_not_optional():
    """A dx3 block whose head fuses (by its geometry alone) needs idf_dense_block_dx3_tmp_bytes of
    tmp: one byte less is IDF_ERR_WORKSPACE (no quiet switch to the head GEMM, whose sums run in
    another order), and the need does not depend on the room offered.  Host-side checks only:
    the call returns before any launch."""
    import ctypes
    from idfcodec import _lib
    lib = _lib.lib()
    d = _lib.IdfDenseBlock()
    d.depth, d.g_pad, d.n_head, d.fold, d.wx3, d.dx3, d.fuse_head = 2, 44, 12, 1, 1, 1, 1
    for i, c in enumerate((12, 56, 100)):
        d.k_in[i] = c
    for i in range(2):
        d.dx3_w[i] = 0x100000 * (i + 1)  # never dereferenced before the workspace check
    B, H, W = 4, 8, 8  # the split-K level: its partial sums make the need exceed P * k_in[2] * 4
    P = B * H * W
    need = int(lib.idf_dense_block_dx3_tmp_bytes(ctypes.byref(d), B, H, W))
    assert need >= P * (4 * 64 + 64)  # at least the split copy (4 slabs) and the head sums
    d.fuse_head = 0
    need_nf = int(lib.idf_dense_block_dx3_tmp_bytes(ctypes.byref(d), B, H, W))
    assert need - need_nf >= P * 64
    d.fuse_head = 1
    head = _lib.IdfHeadOut()
    head.mode = _lib.EPI_STORE
    ld_tmp = (need - 1) // (4 * P)  # floats per pixel: P * ld_tmp * 4 < need
    assert P * ld_tmp * 4 < need and ld_tmp >= 100 and (need - P * 64) < P * ld_tmp * 4
    fake = ctypes.c_void_p(0x7f0000000000)  # 256-B aligned, never touched
    rc = lib.idf_dense_block_f32(None, ctypes.byref(d), B, H, W, fake, 112, fake, ld_tmp,
                                 ctypes.byref(head))
    assert rc == 3, _lib.ERR_NAMES.get(rc, rc)  # IDF_ERR_WORKSPACE
    d.n_head = 17  # no fusion for heads of > 16 outputs: only the copy and split-K part
    assert int(lib.idf_dense_block_dx3_tmp_bytes(ctypes.byref(d), B, H, W)) == need_nf


def test_struct_layout_matches_header():
    """ctypes mirror of IdfDenseBlock / IdfHeadOut == the C layout (compiled probe)."""
    from idfcodec import _lib
    import ctypes
    probe = r'''
#include <stdio.h>
#include <stddef.h>
#include "idf_codec.h"
int main(){printf("%zu %zu %zu %zu %zu %zu\n", sizeof(IdfDenseBlock), offsetof(IdfDenseBlock,w1),
 offsetof(IdfDenseBlock,n_head), offsetof(IdfDenseBlock,bh), sizeof(IdfHeadOut), offsetof(IdfHeadOut,scale));}
'''
    import tempfile
    with tempfile.TemporaryDirectory() as t:
        c = os.path.join(t, "p.c")
        open(c, "w").write(probe)
        exe = os.path.join(t, "p")
        subprocess.run(["gcc", "-I", os.path.join(REPO, "include"), c, "-o", exe], check=True)
        got = list(map(int, subprocess.run([exe], capture_output=True, text=True).stdout.split()))
    D, H = _lib.IdfDenseBlock, _lib.IdfHeadOut
    assert got == [ctypes.sizeof(D), D.w1.offset, D.n_head.offset, D.bh.offset, ctypes.sizeof(H),
                   H.scale.offset]


# ------------------------------------------------------------------ packing
def _simulate_packed_block(pb, x):
    """The device algorithm (padded pixel-major GEMMs) replayed with torch on CPU."""
    from idfcodec.packing import round_up
    g = pb.geom
    B, C, H, W = x.shape
    P = B * H * W
    feat = torch.zeros(P, g.ld_feat, dtype=torch.float64)
    feat[:, :C] = x.permute(0, 2, 3, 1).reshape(P, C).double()
    act = {"ReLU": F.relu, "LeakyReLU": lambda v: F.leaky_relu(v, 0.01)}[pb.act]
    for i in range(g.depth):
        k = g.k_in[i]
        if pb.fold:
            X = feat[:, :k].view(B, H, W, k).permute(0, 3, 1, 2)
            w3 = torch.from_numpy(pb.w3[i]).double()[: g.g_pad, :, :k]
            wc = w3.permute(0, 2, 1).reshape(g.g_pad, k, 3, 3)
            o = F.conv2d(X, wc, padding=1)
            v = torch.from_numpy(pb.vtap[i]).double()[:, : g.g_pad]          # [tap, n]
            ones = torch.ones(1, 1, H, W, dtype=torch.float64)
            # number of in-image taps per pixel and tap, as a 9-channel mask
            mask = F.conv2d(ones, torch.eye(9, dtype=torch.float64).view(9, 1, 3, 3), padding=1)
            bias = torch.einsum("tn,bthw->bnhw", v, mask) + \
                torch.from_numpy(pb.b3[i]).double()[: g.g_pad].view(1, -1, 1, 1)
            feat[:, k:k + g.g_pad] = act(o + bias).permute(0, 2, 3, 1).reshape(P, g.g_pad)
            continue
        w1 = torch.from_numpy(pb.w1[i]).double()
        T = feat[:, :k] @ w1[:k, :k].T + torch.from_numpy(pb.b1[i]).double()[:k]
        Tn = T.view(B, H, W, k).permute(0, 3, 1, 2)
        w3 = torch.from_numpy(pb.w3[i]).double()[: g.g_pad, :, :k]  # [g, tap, c]
        w3c = w3.permute(0, 2, 1).reshape(g.g_pad, k, 3, 3)
        o = F.conv2d(Tn, w3c, torch.from_numpy(pb.b3[i]).double()[: g.g_pad], padding=1)
        feat[:, k:k + g.g_pad] = act(o).permute(0, 2, 3, 1).reshape(P, g.g_pad)
    kh = g.k_in[g.depth]
    out = feat[:, :kh] @ torch.from_numpy(pb.wh).double()[: g.n_head, :kh].T + \
        torch.from_numpy(pb.bh).double()[: g.n_head]
    del round_up
    return out.view(B, H, W, g.n_head).permute(0, 3, 1, 2)


@pytest.mark.parametrize("fold", [False, True])
@pytest.mark.parametrize("name", ["t1_idflows_2lvl", "t2_idflows_3lvl_leaky", "t4_cond_s1_odd"])
def test_packed_layout_reproduces_dense_block(golden, name, fold):
    import flow_oracle as FO
    from idfcodec.packing import pack_dense_block
    d = golden(f"flow_{name}.npz")
    cfg = yaml.safe_load(bytes(d["cfg_yaml"]).decode())
    sd = {k[3:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("sd/")}
    depth = cfg["couple"]["nn"]["depth"]
    act = cfg["couple"]["nn"]["layer"]["act"]
    prefix = "blocks.0.flows.1.dense."
    pb = pack_dense_block(sd, prefix, depth, act, fold=fold)
    a = pb.geom.a
    x = torch.randn(2, a, cfg["H"] // cfg["extenddim"]["scale"], cfg["W"] // cfg["extenddim"]["scale"],
                    generator=torch.Generator().manual_seed(5))
    ref = FO.dense_block(x.double(), {k: v.double() for k, v in sd.items()}, prefix, depth, act)
    got = _simulate_packed_block(pb, x)
    # unfolded: exact layout check; folded: W3.W1 is rounded once to fp32 (~1e-7 rel)
    tol = 1e-6 if fold else 1e-9
    torch.testing.assert_close(got, ref, rtol=tol, atol=tol)
    # padding columns are exactly zero in every weight
    g = pb.geom
    pad_cols = sorted(set(range(g.width)) - set(g.positions(g.a + sum(g.growth)).tolist()))
    assert np.all(pb.wh[:, pad_cols] == 0)


def test_tile_n_matches_kernel_source():
    from idfcodec.packing import tile_n
    src = open(os.path.join(PKG, "csrc", "flow_kernels.hip")).read()
    assert "static int tile_n(int N)" in src
    assert [tile_n(n) for n in (3, 16, 17, 44, 48, 64, 65, 96, 128, 200, 540)] == \
        [16, 16, 32, 48, 48, 64, 128, 128, 128, 128, 64]


def test_flops_per_image_imagenet64():
    """51.41 GFLOP per image per direction (measured with hooks)."""
    from idfcodec.packing import BlockGeometry, growths
    tot = 0
    for C, hw in ((12, 32 * 32), (24, 16 * 16), (48, 8 * 8)):
        a = int(C * 0.75)
        cg = BlockGeometry(a=a, depth=12, growth=growths(512, 12), n_head=C - a)
        tot += 8 * hw * cg.flops_per_pixel()
    for cin, out, hw in ((6, 12, 32 * 32), (12, 24, 16 * 16), (48, 96, 8 * 8)):
        pg = BlockGeometry(a=cin, depth=12, growth=growths(512, 12), n_head=out)
        tot += hw * pg.flops_per_pixel()
    assert abs(tot / 1e9 - 51.41) < 0.05, tot


# ------------------------------------------------------------------ mirror modules
@pytest.mark.parametrize("name", ["t1_idflows_2lvl", "t2_idflows_3lvl_leaky", "t3_cond_convcond",
                                  "t4_cond_s1_odd"])
def test_seeded_mirror_model_equals_reference(golden, name):
    from idfcodec import synthetic
    d = golden(f"flow_{name}.npz")
    cfg = yaml.safe_load(bytes(d["cfg_yaml"]).decode())
    sd = synthetic.build_model(cfg).state_dict()
    ref = {k[3:]: d[k] for k in d.files if k.startswith("sd/")}
    assert list(sd) == list(ref)
    for k in ref:
        assert np.array_equal(sd[k].numpy(), ref[k]), k


@pytest.mark.slow
def test_seeded_imagenet64_equals_reference(golden):
    from idfcodec import configs, synthetic
    d = golden("imagenet64_b2.npz")
    sd = synthetic.build_model(configs.get("imagenet64")).state_dict()
    assert list(sd) == bytes(d["param_names"]).decode().split("\n")
    sums = np.array([float(v.double().sum()) for v in sd.values()])
    assert np.array_equal(sums, d["param_sums"])


def test_configs_restate_reference_yaml():
    from idfcodec import configs
    ref_dir = "/root/reference/configs"
    if not os.path.isdir(ref_dir):
        pytest.skip("reference tree not present (GPU box)")
    for n in configs.CONFIGS:
        assert configs.load_yaml(os.path.join(ref_dir, n + ".yaml")) == configs.get(n)


def test_registry_names():
    import flows  # noqa: F401
    from moduleregister import Register
    for n in ("IDFlows", "ConditionalFlows", "AdditiveCouple", "DenseBlock", "DenseLayer", "Prior",
              "ExtendDim", "DLogistic", "Round"):
        assert Register.get(n).__name__ == n
    with pytest.raises(Exception, match="Can not find object"):
        Register.get("NoSuchThing")


def test_product_modules_refuse_cpu_tensors():
    from idfcodec import configs, synthetic
    from idfcodec._lib import IdfError
    m = synthetic.build_model(configs.get("imagenet64"))
    with pytest.raises((IdfError, RuntimeError)):
        m.forward(torch.zeros(1, 3, 64, 64), None)
    with pytest.raises((IdfError, RuntimeError)):
        m.blocks[0]["flows"][1].dense(torch.zeros(1, 9, 4, 4))


# ------------------------------------------------------------------ bitstream
def test_bitstream_container_roundtrip():
    from idfcodec.codec import Bitstream
    g = torch.Generator().manual_seed(0)
    nw = torch.randint(0, 50, (6,), generator=g).to(torch.int64)
    st = torch.randint(-(2 ** 62), 2 ** 62, (6,), generator=g, dtype=torch.int64)
    w = torch.randint(-(2 ** 31), 2 ** 31 - 1, (int(nw.sum()),), generator=g, dtype=torch.int32)
    bs = Bitstream(2, [(6, 32, 32), (12, 16, 16), (48, 8, 8)], st, nw, w,
                   meta={"n_subpixels": 2 * 3 * 64 * 64})
    raw = bs.to_bytes()
    bs2 = Bitstream.from_bytes(raw)
    assert bs2.n_images == 2 and bs2.level_shapes == bs.level_shapes
    assert torch.equal(bs2.states, st) and torch.equal(bs2.nwords, nw) and torch.equal(bs2.words, w)
    assert bs2.bits() == 64 * 6 + 32 * int(nw.sum())
    assert len(raw) == 20 + 36 + 8 + 8 * 6 + 4 * 6 + 4 * int(nw.sum())
    with pytest.raises(ValueError):
        Bitstream.from_bytes(b"XXXX" + raw[4:])


def test_residual_container_roundtrip_and_source_size():
    """IDFR container: index code + flow streams; version 2 carries the pre-pad source size
    (config 5's 215x178 -> 216x184 ReplicationPad2d), version 1 streams still read."""
    import struct
    from idfcodec.codec import Bitstream
    from idfcodec.residual import ResidualBitstream
    nw = torch.tensor([2, 0, 1], dtype=torch.int64)
    st = torch.tensor([5, -7, 2 ** 40], dtype=torch.int64)
    w = torch.arange(3, dtype=torch.int32)
    flow = Bitstream(1, [(6, 4, 4), (12, 2, 2), (48, 1, 1)], st, nw, w)
    idx = torch.tensor([1, -2, 3], dtype=torch.int32)
    for src in (None, (215, 178)):
        rbs = ResidualBitstream(flow, idx, 1, (3, 216, 184), (27, 23), 8192, src)
        r2 = ResidualBitstream.from_bytes(rbs.to_bytes())
        assert r2.source_hw == src and r2.image_shape == (3, 216, 184) and r2.grid == (27, 23)
        assert r2.source_shape == (3,) + (src or (216, 184))
        assert torch.equal(r2.idx_words, idx) and torch.equal(r2.flow.words, w)
        assert r2.bits() == flow.bits() + 27 * 23 * 13
    raw = ResidualBitstream(flow, idx, 1, (3, 216, 184), (27, 23), 8192).to_bytes()
    v1 = raw[:4] + struct.pack("<H", 1) + raw[6:36] + raw[44:]   # drop the v2 size words
    r1 = ResidualBitstream.from_bytes(v1)
    assert r1.source_hw is None and torch.equal(r1.idx_words, idx)
    with pytest.raises(ValueError):
        ResidualBitstream.from_bytes(b"IDFX" + raw[4:])
    # header flags bit 0: the VQ decoder's conv mode (0 = exact f32, every older stream)
    assert r1.vq_conv == "f32" and struct.unpack_from("<H", raw, 6)[0] == 0
    x3 = ResidualBitstream(flow, idx, 1, (3, 216, 184), (27, 23), 8192, None, "x3").to_bytes()
    assert struct.unpack_from("<H", x3, 6)[0] == 1
    assert ResidualBitstream.from_bytes(x3).vq_conv == "x3"
    x3t = ResidualBitstream(flow, idx, 1, (3, 216, 184), (27, 23), 8192, None, "x3t").to_bytes()
    assert struct.unpack_from("<H", x3t, 6)[0] == 3
    assert ResidualBitstream.from_bytes(x3t).vq_conv == "x3t"
    for bad in (6, 2):  # an unknown bit; the taps bit without the ResBlocks' bit
        with pytest.raises(ValueError, match="flags"):
            ResidualBitstream.from_bytes(x3[:6] + struct.pack("<H", bad) + x3[8:])


# ------------------------------------------------------------------ coder chaining (F4)
def test_coder_decode_fix_roundtrips_with_oracle(golden, oracle, monkeypatch):
    """coder.Encode chains the state across levels; the reference Decode does not
    round-trip, the fixed Decode does.  Exercised on CPU with the
    oracle standing in for rans.rans (same list API)."""
    import coder

    def enc(state, n, x, m, s):
        st, w = oracle.encode(state, x[:n], m[:n], s[:n])
        return st, w.tolist()

    def dec(state, buf, n, m, s):
        # reference convention: buf, m, s reversed; result reversed
        st, out = oracle.decode(state, np.asarray(buf[::-1], np.uint32), n, np.asarray(m[::-1]),
                                np.asarray(s[::-1]))
        return st, out[::-1].astype(np.float64).tolist()

    monkeypatch.setattr(coder, "encode", enc)
    monkeypatch.setattr(coder, "decode", dec)
    d = golden("imagenet64_b2.npz")
    lat = [torch.from_numpy(d[f"latent{i}"]) for i in range(3)]
    mean = [torch.from_numpy(d[f"mean{i}"]) for i in range(3)]
    logs = [torch.from_numpy(d[f"logscale{i}"]) for i in range(3)]
    x, bufs = coder.Encode(lat, mean, logs)
    assert any(len(b) for b in bufs)
    x2, rec = coder.Decode(bufs, mean, logs, x)
    assert x2 == 1 << 32
    for a, b in zip(rec, lat):
        assert torch.equal(a, b)


# ------------------------------------------------------------------ expf restatement
@pytest.mark.slow
def test_restated_expf_equals_libm_on_all_floats(tmp_path):
    exe = tmp_path / "expf_check"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fopenmp", "-I", os.path.join(PKG, "csrc"),
                    os.path.join(REPO, "tests", "native", "expf_check.cpp"), "-o", str(exe)],
                   check=True, capture_output=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    assert "mismatches=0" in r.stdout


def test_bf16_weight_packing_layout():
    """bf16_weights: uint16 bf16 bits of the fp32 folded weights in the fragment order
    [slab][tap][k-block][n][8] that conv3_bf16.hip reads."""
    import numpy as np
    import torch
    from idfcodec.packing import bf16_weights
    rng = np.random.default_rng(4)
    n_alloc, C, ldw = 48, 52, 64
    w = rng.normal(0, 1, (n_alloc, 9, ldw)).astype(np.float32)
    w[:, :, C:] = 0
    b = bf16_weights(w, C)
    nslab = (C + 31) // 32
    assert b.shape == (nslab, 9, 4, n_alloc, 8) and b.dtype == np.uint16
    ref = torch.from_numpy(w).to(torch.bfloat16).float().numpy()
    back = torch.from_numpy(b.astype(np.int16)).view(torch.bfloat16).float().numpy()
    for s in range(nslab):
        for kb in range(4):
            for e in range(8):
                c = 32 * s + 8 * kb + e
                want = ref[:, :, c] if c < C else np.zeros((n_alloc, 9), np.float32)
                assert np.array_equal(back[s, :, kb, :, e].T, want)


def test_dx3_weight_packing_layout_and_prefix(golden):
    """dx3_weights: [slab][group][hi, lo][tap][nf][out][ch] f16 pairs with (hi + lo) 2^-k equal
    to the float64 weight within f16-pair precision, zeros past C (and past n_alloc in the last
    group); groups of up to 4 fragments (dx3_groups); pack_dense_block(dx3_cmax) packs them for
    the leading layers whose input is at most dx3_cmax wide, nothing after."""
    import numpy as np
    from idfcodec.packing import dx3_groups, dx3_weights, pack_dense_block
    assert [dx3_groups(n) for n in (16, 48, 64, 80, 128, 192)] == \
        [(1, 1), (3, 1), (4, 1), (4, 2), (4, 2), (4, 3)]
    rng = np.random.default_rng(6)
    for n_alloc, C, ldw, shape in ((48, 40, 48, (3, 1, 2, 9, 3, 16, 16)),
                                   (80, 36, 48, (3, 2, 2, 9, 4, 16, 16))):
        w = rng.normal(0, 0.05, (n_alloc, 9, ldw))
        w[:, :, C:] = 0
        d, ysc = dx3_weights(w, C)
        assert d.shape == shape and d.dtype == np.uint16
        f = d.view(np.float16).astype(np.float64)
        back = (f[:, :, 0] + f[:, :, 1]) * ysc               # slab, group, tap, nf, out, ch
        nft = shape[1] * shape[4]
        back = back.transpose(1, 3, 4, 2, 0, 5).reshape(nft * 16, 9, shape[0] * 16)
        assert np.abs(back[:n_alloc, :, :C] - w[:, :, :C]).max() <= 2.0 ** -20 * np.abs(w).max()
        assert not back[:, :, C:].any() and not back[n_alloc:].any()
    g = golden("flow_t1_idflows_2lvl.npz")
    cfg = yaml.safe_load(bytes(g["cfg_yaml"]).decode())
    sd = {k[3:]: torch.from_numpy(g[k]) for k in g.files if k.startswith("sd/")}
    depth = cfg["couple"]["nn"]["depth"]
    assert depth >= 3
    pre = "blocks.0.flows.1.dense."
    full = pack_dense_block(sd, pre, depth, fold=True, wino=True, wx3=True, dx3=True)
    assert len(full.dx3_w) == depth
    k_in = full.geom.k_in
    part = pack_dense_block(sd, pre, depth, fold=True, wino=True, wx3=True, dx3=True,
                            dx3_cmax=k_in[1])
    assert len(part.dx3_w) == 2
    for a, b in zip(part.dx3_w, full.dx3_w):
        assert np.array_equal(a, b)


def test_bitstream_conv_flag_round_trips():
    import torch
    from idfcodec.codec import Bitstream
    st = torch.tensor([1 << 32, 5], dtype=torch.int64)
    nw = torch.tensor([1, 2], dtype=torch.int64)
    w = torch.tensor([7, 8, 9], dtype=torch.int32)
    for mode in ("x3", "f32", "halo", "gemm", "unfold", "bf16"):
        bs = Bitstream(1, [(6, 4, 4), (12, 2, 2)], st, nw, w, meta={"n_subpixels": 48, "conv": mode})
        back = Bitstream.from_bytes(bs.to_bytes())
        assert back.meta["conv"] == mode
    legacy = Bitstream(1, [(6, 4, 4), (12, 2, 2)], st, nw, w)  # no conv in meta: exact f32
    back = Bitstream.from_bytes(legacy.to_bytes())
    assert back.meta["conv"] == "f32"
    assert torch.equal(back.host_nwords, nw) and not back.host_nwords.is_cuda


def test_version1_container_without_conv_field():
    """ADVICE r2 (codec.py:432): version-1 files with flags 0 were written by every engine
    before the conv field existed.  They read as conv 'unrecorded', which every engine but a
    split-f16 one accepts (the pre-field behaviour); version-1 files with a conv code and
    version-2 files keep the exact check; an unrecorded file cannot be re-written as v2."""
    import struct
    from idfcodec.codec import VERSION, Bitstream
    shapes = [(6, 4, 4), (12, 2, 2)]
    st = torch.zeros(4, dtype=torch.int64)
    nw = torch.ones(4, dtype=torch.int64)
    raw = Bitstream(2, shapes, st, nw, torch.zeros(4, dtype=torch.int32),
                    meta={"conv": "f32"}).to_bytes()
    assert struct.unpack_from("<H", raw, 4)[0] == VERSION == 2
    v1 = raw[:4] + struct.pack("<HH", 1, 0) + raw[8:]
    old = Bitstream.from_bytes(v1)
    assert old.meta["conv"] == "unrecorded"
    for fam in ("f32", "halo", "gemm", "unfold", "bf16"):
        _codec_for(shapes, family=fam, wx3=False).check_bitstream(old)
    with pytest.raises(ValueError, match="predates the conv field"):
        _codec_for(shapes, family="x3").check_bitstream(old)
    with pytest.raises(ValueError, match="re-encode"):
        old.to_bytes()
    v1_x3 = raw[:4] + struct.pack("<HH", 1, 1) + raw[8:]
    assert Bitstream.from_bytes(v1_x3).meta["conv"] == "x3"
    with pytest.raises(ValueError, match="coded with 'bf16'"):
        _codec_for(shapes, family="x3").check_bitstream(
            Bitstream.from_bytes(raw[:4] + struct.pack("<HH", 2, 5) + raw[8:]))


def _codec_for(levels, family="x3", wx3=True):
    from types import SimpleNamespace
    from idfcodec.codec import ImageCodec
    c = ImageCodec.__new__(ImageCodec)
    # an fp32 engine without dx3 weights (FlowEngine.can_run's rule for it)
    c.engine = SimpleNamespace(levels=[SimpleNamespace(z=z, h=h, w=w) for z, h, w in levels],
                               conv_family=family, wx3=wx3,
                               can_run=lambda conv: conv == "f32" or (conv == "x3" and wx3))
    return c


def test_decode_rejects_mismatched_container():
    """A truncated, corrupted or other-config container raises before any device launch
    (the rANS decode indexes streams by (level, image): no out-of-bounds reads)."""
    import pytest
    import torch
    from idfcodec.codec import Bitstream
    shapes = [(6, 4, 4), (12, 2, 2)]
    c = _codec_for(shapes)

    def bs(n_img=2, ns=4, nwords=None, nw_total=None, sh=shapes, conv="x3"):
        nw = torch.tensor(nwords if nwords is not None else [1] * ns, dtype=torch.int64)
        tot = int(nw.sum()) if nw_total is None else nw_total
        return Bitstream(n_img, sh, torch.zeros(ns, dtype=torch.int64), nw,
                         torch.zeros(tot, dtype=torch.int32), meta={"conv": conv})
    c.check_bitstream(bs())  # well-formed
    c.check_bitstream(bs(conv="f32"))  # switchable mode
    with pytest.raises(ValueError, match="level shapes"):
        c.check_bitstream(bs(sh=[(6, 4, 4), (12, 4, 4)]))
    with pytest.raises(ValueError, match="level shapes"):
        c.check_bitstream(bs(sh=shapes[:1], ns=2))
    with pytest.raises(ValueError, match="streams"):
        c.check_bitstream(bs(ns=3))
    with pytest.raises(ValueError, match="negative"):
        c.check_bitstream(bs(nwords=[1, -1, 1, 1]))
    with pytest.raises(ValueError, match="word table"):
        c.check_bitstream(bs(nw_total=2))
    with pytest.raises(ValueError, match="coded with 'bf16'"):
        c.check_bitstream(bs(conv="bf16"))
    with pytest.raises(ValueError, match="coded with 'x3'"):
        _codec_for(shapes, family="f32", wx3=False).check_bitstream(bs())
    # a truncated container does not parse
    good = bs().to_bytes()
    with pytest.raises(ValueError):
        Bitstream.from_bytes(good[:-3])
    bad = bytearray(good)
    bad[6] = 0x3F  # unknown conv code in the flags
    with pytest.raises(ValueError):
        Bitstream.from_bytes(bytes(bad))


def test_earlier_build_fixture_headers(golden):
    """The earlier builds' fixtures (tests/golden/make_conv_fixture.py) read with their conv codes
    -- 6 ("dx3w16"), 7 ("dx3") -- and re-serialise byte for byte; their decodes are
    tests/test_gpu_codec.py's."""
    from idfcodec.codec import Bitstream
    for name, conv in (("imagenet64_code6_r4.npz", "dx3w16"), ("imagenet64_code7_r5.npz", "dx3")):
        d = golden(name)
        bs = Bitstream.from_bytes(d["bitstream"].tobytes())
        assert bs.meta["conv"] == conv and bs.n_images == d["images"].shape[0] == 4
        assert bs.to_bytes() == d["bitstream"].tobytes()  # re-serialises byte for byte


def test_fused_block_geometries():
    """The fused DenseBlock launch (idf_dx3_block_supported) takes exactly the geometries whose
    tiles hold whole images, with one output group and no split K: 16x16 and the packed 4x4
    images -- not 8x8 (split K: the per-layer launches are faster), 32x32 (four tiles an
    image), 27x23 or 2x2 (gutter bands crossing tiles), nor 128 outputs (two output groups)."""
    from idfcodec import _lib
    sup = _lib.lib().idf_dx3_block_supported
    for (H, W, N, bf), want in [((16, 16, 48, 0), 1), ((8, 8, 48, 0), 0), ((4, 4, 32, 0), 1),
                                ((16, 16, 48, 1), 1), ((8, 8, 48, 1), 0), ((32, 32, 48, 0), 0),
                                ((27, 23, 32, 0), 0), ((2, 2, 32, 0), 0), ((4, 4, 128, 0), 0),
                                ((64, 64, 48, 0), 0)]:
        assert sup(H, W, N, bf) == want, (H, W, N, bf)
