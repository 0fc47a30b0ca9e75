"""The oracle pinned against the reference's own outputs (tests/golden, made by
tests/golden/make_golden.py from the reference's compiled coder and modules)."""
import numpy as np
import pytest
import torch
import yaml

CASES = ["kat1", "rand1", "rand96", "rand1863", "rand3072", "rand6144", "narrow", "edge_window",
         "out_of_window"]


@pytest.mark.parametrize("case", CASES)
def test_rans_oracle_encode_matches_reference(golden, oracle, case):
    d = golden("rans_kat.npz")
    st, w = oracle.encode(int(d[f"{case}/init_state"]), d[f"{case}/x"], d[f"{case}/mean"],
                          d[f"{case}/scale"])
    assert st == int(d[f"{case}/state"])
    assert np.array_equal(w, d[f"{case}/words"])


@pytest.mark.parametrize("case", CASES)
def test_rans_oracle_decode_matches_reference(golden, oracle, case):
    d = golden("rans_kat.npz")
    n = d[f"{case}/x"].size
    st, out = oracle.decode(int(d[f"{case}/state"]), d[f"{case}/words"], n, d[f"{case}/mean"],
                            d[f"{case}/scale"])
    assert st == int(d[f"{case}/dec_state"])
    assert np.array_equal(out, d[f"{case}/dec_x"])


def test_kat1_recorded_values(golden, oracle):
    """SURVEY App. C, recorded from the reference coder."""
    d = golden("rans_kat.npz")
    st, w = oracle.encode(1 << 32, d["kat1/x"], d["kat1/mean"], d["kat1/scale"])
    assert st == 28772813360 and w.size == 1102
    assert int(w.astype(np.uint64).sum()) % (1 << 32) == 2555577472
    assert w[:3].tolist() == [3753566951, 880733091, 2516695742]
    assert w[-3:].tolist() == [184250203, 2599675978, 2804102162]


def test_chained_and_empty(golden, oracle):
    d = golden("rans_kat.npz")
    x, m, s = d["kat1/x"], d["kat1/mean"], d["kat1/scale"]
    st, w0 = oracle.encode(1 << 32, x[:10], m[:10], s[:10])
    assert st == int(d["chain/state0"]) and np.array_equal(w0, d["chain/words0"])
    st2, w1 = oracle.encode(st, x[10:20], m[10:20], s[10:20])
    assert st2 == int(d["chain/state1"]) and np.array_equal(w1, d["chain/words1"])
    st, w = oracle.encode(1 << 32, [], [], [])
    assert st == int(d["empty/state"]) and w.size == int(d["empty/nwords"]) == 0


def test_rans_oracle_scale_zero_raises(oracle):
    with pytest.raises(ZeroDivisionError):
        oracle.encode(1 << 32, [0.0], [0.0], [0.0])


def test_streams_equal_single_calls(golden, oracle):
    d = golden("rans_kat.npz")
    x, m, s = d["kat1/x"], d["kat1/mean"], d["kat1/scale"]
    off = np.array([0, 100, 1000, 1001, 4096], np.int64)
    fs, words, nw, status = oracle.encode_streams(off, x, m, s)
    assert (status == 0).all()
    for k in range(4):
        st, w = oracle.encode(1 << 32, x[off[k]:off[k + 1]], m[off[k]:off[k + 1]], s[off[k]:off[k + 1]])
        assert fs[k] == st and np.array_equal(words[off[k]:off[k] + nw[k]], w)
    woff = off[:-1]
    fs2, out, st2 = oracle.decode_streams(off, woff, nw, words, m, s, fs)
    assert (fs2 == 1 << 32).all() and np.array_equal(out, x)


def _flow_case(golden, name):
    d = golden(f"flow_{name}.npz")
    cfg = yaml.safe_load(bytes(d["cfg_yaml"]).decode())
    sd = {k[3:]: torch.from_numpy(d[k]) for k in d.files if k.startswith("sd/")}
    return d, cfg, sd


@pytest.mark.parametrize("name", ["t1_idflows_2lvl", "t2_idflows_3lvl_leaky", "t3_cond_convcond",
                                  "t4_cond_s1_odd"])
def test_flow_oracle_matches_reference(golden, name):
    import flow_oracle as FO
    d, cfg, sd = _flow_case(golden, name)
    o = FO.FlowOracle(cfg, sd)
    x = torch.from_numpy(d["input"])
    cond = torch.from_numpy(d["cond"]) if "cond" in d.files else None
    lat, me, ls = o.forward(x, cond)
    for i in range(len(lat)):
        torch.testing.assert_close(lat[i], torch.from_numpy(d[f"latent{i}"]), rtol=0, atol=0)
        torch.testing.assert_close(me[i], torch.from_numpy(d[f"mean{i}"]), rtol=1e-6, atol=1e-6)
        torch.testing.assert_close(ls[i], torch.from_numpy(d[f"logscale{i}"]), rtol=1e-6, atol=1e-6)
    g = o.generated_from_latents([torch.from_numpy(d[f"latent{i}"]) for i in range(len(lat))])
    torch.testing.assert_close(g, torch.from_numpy(d["generated"]), rtol=0, atol=0)
    torch.testing.assert_close(o.log_likelihood(lat, me, ls), torch.from_numpy(d["log_prob"]),
                               rtol=1e-5, atol=1e-6)
    # hierarchical decoder given the true latents reproduces the input exactly
    L = [torch.from_numpy(d[f"latent{i}"]) for i in range(len(lat))]
    xd, _ = o.decode_levels(x.shape[0], lambda l, m, s: L[l], cond)
    assert torch.equal(xd, x)


def test_dequant_grid():
    """trainer.py:101 dequant == (k + [k>=128]) / 256 for every uint8 value."""
    import flow_oracle as FO
    k = torch.arange(256, dtype=torch.uint8)
    ref = FO.dequant(k)
    mine = (k.float() + (k >= 128).float()) / 256
    assert torch.equal(ref, mine)
