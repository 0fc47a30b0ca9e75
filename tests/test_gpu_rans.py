"""GPU parity of the rANS coder: bit-identical to the reference (golden vectors
recorded from the reference's compiled coder) and to the C oracle."""
import os
import subprocess

import numpy as np
import pytest
import torch

from conftest import PKG, REPO

pytestmark = pytest.mark.gpu

CASES = ["kat1", "rand1", "rand96", "rand1863", "rand3072", "rand6144", "narrow", "edge_window",
         "out_of_window"]


def _enc_streams(off, x, mean, scale, init=None):
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    dev = torch.device("cuda")
    t = lambda a, dt=torch.float32: torch.as_tensor(np.ascontiguousarray(a)).to(dev, dt)  # noqa
    off_t = t(off, torch.int64)
    ns = off.size - 1
    nsym = int(off[-1])
    init_t = torch.full((ns,), 1 << 32, dtype=torch.int64, device=dev) if init is None else \
        t(np.asarray(init, np.uint64).view(np.int64), torch.int64)
    fs = torch.empty(ns, dtype=torch.int64, device=dev)
    nw = torch.empty(ns, dtype=torch.int64, device=dev)
    st = torch.empty(ns, dtype=torch.int32, device=dev)
    words = torch.empty(max(nsym, 1), dtype=torch.int32, device=dev)
    wb = lib().idf_rans_encode_workspace_bytes(nsym)
    ws = torch.empty(wb, dtype=torch.uint8, device=dev)
    # keep every device buffer referenced until the kernels have run
    dx, dm, ds = t(x), t(mean), t(scale)
    check(lib().idf_rans_encode_streams(_lib.stream_ptr(), ns, nsym, ptr(off_t), ptr(dx), ptr(dm),
                                        ptr(ds), ptr(init_t), ptr(fs), ptr(words), ptr(nw),
                                        ptr(st), ptr(ws), wb), "enc")
    torch.cuda.synchronize()
    return (fs.cpu().numpy().view(np.uint64), words.cpu().numpy().view(np.uint32),
            nw.cpu().numpy(), st.cpu().numpy())


def _dec_streams(off, woff, nw, words, mean, scale, init):
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    dev = torch.device("cuda")
    t = lambda a, dt: torch.as_tensor(np.ascontiguousarray(a)).to(dev, dt)  # noqa
    ns = off.size - 1
    fs = torch.empty(ns, dtype=torch.int64, device=dev)
    out = torch.empty(max(int(off[-1]), 1), dtype=torch.float32, device=dev)
    st = torch.empty(ns, dtype=torch.int32, device=dev)
    w = t(np.asarray(words, np.uint32).view(np.int32) if len(words) else np.zeros(1, np.int32), torch.int32)
    bufs = [t(off, torch.int64), t(woff, torch.int64), t(nw, torch.int64), w,
            t(mean, torch.float32), t(scale, torch.float32),
            t(np.asarray(init, np.uint64).view(np.int64), torch.int64)]
    nsym = int(off[-1])
    wb = lib().idf_rans_decode_workspace_bytes(nsym)
    ws = torch.empty(wb, dtype=torch.uint8, device=dev)
    check(lib().idf_rans_decode_streams(_lib.stream_ptr(), ns, nsym, *[ptr(b) for b in bufs],
                                        ptr(fs), ptr(out), ptr(st), ptr(ws), wb), "dec")
    torch.cuda.synchronize()
    return fs.cpu().numpy().view(np.uint64), out.cpu().numpy()[: int(off[-1])], st.cpu().numpy()


@pytest.mark.parametrize("case", CASES)
def test_device_encode_matches_reference_goldens(golden, case):
    d = golden("rans_kat.npz")
    x, m, s = d[f"{case}/x"], d[f"{case}/mean"], d[f"{case}/scale"]
    fs, words, nw, st = _enc_streams(np.array([0, x.size]), x, m, s, [int(d[f"{case}/init_state"])])
    assert int(fs[0]) == int(d[f"{case}/state"])
    assert np.array_equal(words[: nw[0]], d[f"{case}/words"])
    if case != "out_of_window":
        assert st[0] & ~16 == 0


@pytest.mark.parametrize("case", CASES)
def test_device_decode_matches_reference_goldens(golden, case):
    d = golden("rans_kat.npz")
    m, s, w = d[f"{case}/mean"], d[f"{case}/scale"], d[f"{case}/words"]
    n = m.size
    fs, out, st = _dec_streams(np.array([0, n]), np.array([0]), np.array([w.size]), w, m, s,
                               [int(d[f"{case}/state"])])
    assert int(fs[0]) == int(d[f"{case}/dec_state"])
    assert np.array_equal(out, d[f"{case}/dec_x"])


def test_rans_shim_api_matches_reference(golden):
    """rans.rans.encode/decode: the reference's Python signatures and conventions."""
    from rans.rans import decode, encode
    d = golden("rans_kat.npz")
    x, m, s = (d[f"kat1/{k}"].astype(np.float64).tolist() for k in ("x", "mean", "scale"))
    st, buf = encode(1 << 32, len(x), x, m, s)
    assert st == 28772813360 and buf == d["kat1/words"].tolist()
    st2, msg = decode(st, buf[::-1], len(x), m[::-1], s[::-1])
    assert st2 == 1 << 32 and msg[::-1] == x
    with pytest.raises(TypeError):
        encode(1 << 32, 1, np.zeros(1), [0.0], [1.0])
    with pytest.raises(ZeroDivisionError):
        encode(1 << 32, 1, [0.0], [0.0], [0.0])
    assert encode(1 << 32, 0, [], [], []) == (1 << 32, [])


def test_chained_states_match_reference(golden):
    from rans.rans import encode
    d = golden("rans_kat.npz")
    x, m, s = (d[f"kat1/{k}"].astype(np.float64).tolist() for k in ("x", "mean", "scale"))
    st, w0 = encode(1 << 32, 10, x[:10], m[:10], s[:10])
    assert st == int(d["chain/state0"]) and w0 == d["chain/words0"].tolist()
    st2, w1 = encode(st, 10, x[10:20], m[10:20], s[10:20])
    assert st2 == int(d["chain/state1"]) and w1 == d["chain/words1"].tolist()


def test_many_ragged_streams_match_oracle(oracle):
    """2000 independent streams of ragged lengths (0..3000), test.py-style inputs."""
    g = np.random.default_rng(1)
    lens = g.integers(0, 3000, 2000)
    lens[:5] = [0, 1, 2, 0, 7]
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    n = int(off[-1])
    mean = (g.integers(-256, 257, n) / 256).astype(np.float32)
    scale = (np.exp(10 * g.random(n) - 5) / 256).astype(np.float32)
    x = (np.round((mean + scale * (10 * g.random(n) - 5)) * 256) / 256).astype(np.float32)
    fs, words, nw, st = _enc_streams(off, x, mean, scale)
    rfs, rwords, rnw, rst = oracle.encode_streams(off, x, mean, scale)
    assert np.array_equal(fs, rfs) and np.array_equal(nw, rnw)
    for k in range(lens.size):
        a = off[k]
        assert np.array_equal(words[a:a + nw[k]], rwords[a:a + nw[k]]), k
    dfs, out, dst = _dec_streams(off, off[:-1], nw, words, mean, scale, fs)
    assert (dfs == 1 << 32).all()
    assert np.array_equal(out, x)
    assert (dst == 0).all()


def test_large_single_stream_matches_oracle(oracle):
    """one stream of 1M symbols (the trainer's whole-level contract at B~170)."""
    g = np.random.default_rng(2)
    n = 1 << 20
    mean = (g.integers(-64, 64, n) / 256).astype(np.float32)
    scale = np.exp(g.normal(-4, 1.5, n)).astype(np.float32)
    x = (np.round((mean + scale * g.logistic(0, 1, n)) * 256) / 256).astype(np.float32)
    lo = np.round(mean.astype(np.float64) * 256 - 1024)
    x = np.clip(x, (lo + 1) / 256, (lo + 2046) / 256).astype(np.float32)
    fs, words, nw, st = _enc_streams(np.array([0, n]), x, mean, scale)
    rs, rw = oracle.encode(1 << 32, x, mean, scale)
    assert int(fs[0]) == rs and np.array_equal(words[: nw[0]], rw)
    dfs, out, dst = _dec_streams(np.array([0, n]), np.array([0]), nw, words[: nw[0]], mean, scale, fs)
    assert int(dfs[0]) == 1 << 32 and np.array_equal(out, x)


def test_device_cdf_matches_oracle(oracle):
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    g = np.random.default_rng(3)
    n = 200000
    mean = g.normal(0, 2, n).astype(np.float32)
    scale = np.exp(g.normal(-2, 3, n)).astype(np.float32)
    x = (np.round((mean + g.normal(0, 4, n)) * 256) / 256).astype(np.float32)
    dev = torch.device("cuda")
    st = torch.empty(n, dtype=torch.int32, device=dev)
    fr = torch.empty(n, dtype=torch.int32, device=dev)
    dx, dm, ds = (torch.from_numpy(a).to(dev) for a in (x, mean, scale))
    check(lib().idf_rans_cdf_freq(_lib.stream_ptr(), n, ptr(dx), ptr(dm), ptr(ds), ptr(st), ptr(fr)),
          "cdf")
    rst, rfr = oracle.cdf_freq(x, mean, scale)
    assert np.array_equal(st.cpu().numpy(), rst) and np.array_equal(fr.cpu().numpy(), rfr)


def test_device_expf_sampled(oracle):
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    g = np.random.default_rng(4)
    bits = g.integers(0, 1 << 32, 1 << 22, dtype=np.uint64).astype(np.uint32)
    special = np.array([0, 0x80000000, 0x7f800000, 0xff800000, 0x7fc00000, 0x42b17218, 0xc2cff1b5,
                        0xc2cff1b4, 0x42b0c0a5, 0x42b00000, 0xc2aeac50], np.uint32)
    xs = np.concatenate([bits, special]).view(np.float32)
    dev = torch.device("cuda")
    inp = torch.from_numpy(xs).to(dev)
    out = torch.empty_like(inp)
    check(lib().idf_expf_glibc(_lib.stream_ptr(), xs.size, ptr(inp), ptr(out)), "expf")
    got = out.cpu().numpy()
    ref = oracle.expf_many(xs)
    same = (got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref))
    assert same.all()


@pytest.mark.slow
def test_device_expf_exhaustive_checksum(tmp_path):
    """All 2^32 inputs: device checksum == host libm checksum (tests/native/expf_check.cpp)."""
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    exe = tmp_path / "expf_check"
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-fopenmp", "-I", os.path.join(PKG, "csrc"),
                    os.path.join(REPO, "tests", "native", "expf_check.cpp"), "-o", str(exe)],
                   check=True, capture_output=True)
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "16"))
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=600)
    assert "mismatches=0" in r.stdout, r.stdout
    host_sum = int(r.stdout.split("checksum=")[1])
    acc = torch.zeros(1, dtype=torch.int64, device="cuda")
    check(lib().idf_expf_checksum(_lib.stream_ptr(), 0, 1 << 32, ptr(acc)), "checksum")
    dev_sum = int(np.int64(acc.item()).view(np.uint64))
    assert dev_sum == host_sum


def test_decode_window_cdf_matches_plain_cdf():
    """The decoder's CDF with hoisted reciprocals == rans_cdf bit for bit (2^26 samples)."""
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    bad = torch.zeros(1, dtype=torch.int64, device="cuda")
    check(lib().idf_rans_cdf_selfcheck(_lib.stream_ptr(), 1 << 26, 12345, ptr(bad)), "selfcheck")
    assert int(bad.item()) == 0


def test_decode_slow_paths_match_oracle(oracle):
    """Scales outside the fast range (two-round exact search) and negative scales (the
    reference's serial binary search) mixed into streams with ordinary ones: final states,
    symbols and status equal the C oracle's decode (rans.pyx:69-110) of the same state and
    words.  Words and states are random (decode is a function of them whether or not an
    encoder produced them)."""
    g = np.random.default_rng(11)
    lens = g.integers(1, 400, 64)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    n = int(off[-1])
    mean = (g.integers(-512, 513, n) / 256).astype(np.float32)
    scale = (np.exp(6 * g.random(n) - 5)).astype(np.float32)
    kind = g.integers(0, 4, n)
    scale[kind == 1] = np.float32(2.0 ** -62)
    scale[kind == 2] = np.float32(2.0 ** 62)
    scale[kind == 3] = -np.float32(2.0 ** 40) * (1 + g.random((kind == 3).sum())).astype(np.float32)
    words = g.integers(0, 1 << 32, n, dtype=np.uint64).astype(np.uint32)
    init = (g.integers(1 << 32, 1 << 62, lens.size, dtype=np.uint64)).astype(np.uint64)
    nw = lens.astype(np.int64)
    rfs, rout, rst = oracle.decode_streams(off, off[:-1], nw, words, mean, scale, init)
    dfs, out, dst = _dec_streams(off, off[:-1], nw, words, mean, scale, init)
    ok = rst == 0
    assert ok.sum() >= lens.size // 2  # most streams decode without a reference error
    for k in np.flatnonzero(ok):
        a, e = off[k], off[k + 1]
        assert dfs[k] == rfs[k], k
        assert np.array_equal(out[a:e], rout[a:e]), k
        assert (dst[k] & ~32) == 0, (k, dst[k])  # at most IDF_STREAM_WORDS_LEFT
    hit = np.zeros(n, bool)
    for k in np.flatnonzero(ok):
        hit[off[k]:off[k + 1]] = True
    for kd in (1, 2, 3):  # every slow path ran inside an oracle-checked stream
        assert (hit & (kind == kd)).sum() > 100, kd


def test_decoder_part1_short_chain_exhaustive():
    """The decoder's short-chain logistic term == the reference arithmetic
    (round((M - 2048) / (1 + expf(-u))), IEEE division) for every non-NaN float u."""
    from idfcodec import _lib
    from idfcodec._lib import check, lib, ptr
    bad = torch.zeros(1, dtype=torch.int64, device="cuda")
    check(lib().idf_rans_part1_selfcheck(_lib.stream_ptr(), 0, 1 << 32, ptr(bad)), "part1")
    assert int(bad.item()) == 0


@pytest.mark.parametrize("wpb", ["2", "4", "1"])
def test_decode_stream_stopping_early_leaves_neighbours_exact(oracle, monkeypatch, wpb):
    """A stream whose decode stops on a zero scale (rans.pyx:36 raises ZeroDivisionError) ends
    its table producer early; the other streams of its block (IDF_DECODE_WPB streams per block:
    2 by default, 4, 1) decode on, equal to the oracle -- every block shape gives the same
    symbols, states and status."""
    monkeypatch.setenv("IDF_DECODE_WPB", wpb)
    g = np.random.default_rng(12)
    lens = np.array([300, 700, 130, 900, 64, 65, 1000, 5], np.int64)
    off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    n = int(off[-1])
    mean = (g.integers(-256, 257, n) / 256).astype(np.float32)
    scale = (np.exp(10 * g.random(n) - 5) / 256).astype(np.float32)
    x = (np.round((mean + scale * (10 * g.random(n) - 5)) * 256) / 256).astype(np.float32)
    fs, words, nw, st = _enc_streams(off, x, mean, scale)
    scale_d = scale.copy()
    stop = {1: 5, 3: 400, 6: 64}  # stream -> decode step (the chain runs backwards) hit by scale 0
    for k, t in stop.items():
        scale_d[off[k + 1] - 1 - t] = 0.0
    dfs, out, dst = _dec_streams(off, off[:-1], nw, words, mean, scale_d, fs)
    for k in range(lens.size):
        a, e = off[k], off[k + 1]
        if k in stop:
            assert dst[k] & 1, (k, dst[k])  # IDF_STREAM_SCALE_ZERO
            t = stop[k]
            assert np.array_equal(out[e - t:e], x[e - t:e]), k  # the symbols before the stop
        else:
            assert dst[k] == 0 and dfs[k] == 1 << 32, k
            assert np.array_equal(out[a:e], x[a:e]), k


@pytest.mark.timeout(600)
def test_reference_scale_50m_symbols(oracle):
    """rans/test.py at its own scale: ONE encode() and ONE decode() call of 50M symbols through
    the reference's Python API (lists in, lists out, decode's reversed conventions), with
    test.py's input distribution.  Encode is bit-identical to the C oracle (final state and
    every word); decode restores the message exactly and returns the initial state.  The
    decode keeps its block-boundary tables in LDS: no per-symbol device workspace."""
    import time
    from idfcodec._lib import lib
    from rans.rans import decode, encode
    n = 50_000_000
    g = np.random.default_rng(50)
    mean = (g.integers(-256, 257, n) / 256).astype(np.float32)
    scale = (np.exp(10 * g.random(n) - 5) / 256).astype(np.float32)
    msg = (np.round((mean + scale * (10 * g.random(n) - 5)) * 256) / 256).astype(np.float32)
    ml, sl, xl = mean.tolist(), scale.tolist(), msg.tolist()
    assert lib().idf_rans_decode_workspace_bytes(n) <= 64 * 1024
    t0 = time.time()
    st, buf = encode(1 << 32, n, xl, ml, sl)
    t1 = time.time()
    rst, rwords = oracle.encode(1 << 32, msg, mean, scale)
    assert st == rst and len(buf) == rwords.size
    assert np.array_equal(np.asarray(buf, dtype=np.uint32), rwords)
    del rwords
    t2 = time.time()
    st2, rec = decode(st, buf[::-1], n, ml[::-1], sl[::-1])
    t3 = time.time()
    assert st2 == 1 << 32
    assert np.array_equal(np.asarray(rec[::-1], dtype=np.float32), msg)
    print(f"50M symbols: encode {t1 - t0:.1f} s, decode {t3 - t2:.1f} s (host lists included), "
          f"{len(buf)} words; decode workspace {lib().idf_rans_decode_workspace_bytes(n)} B")
