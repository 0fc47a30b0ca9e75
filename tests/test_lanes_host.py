"""Host logic of the ImageCodec decode lanes (no GPU): how a batch splits into lanes."""
from idfcodec.codec import ImageCodec


def test_lane_split():
    c = ImageCodec(engine=None, lanes=2)
    assert c._n_lanes(256) == 2
    assert c._n_lanes(15) == 1          # halves below LANE_MIN images
    assert c._n_lanes(17) == 1          # odd batch: no equal split
    assert c._n_lanes(16) == 2
    c.lanes = 4
    assert c._n_lanes(256) == 4
    assert c._n_lanes(18) == 2          # 18 % 4 != 0, 18 / 3 < LANE_MIN
    assert c._n_lanes(24) == 3
    c.lanes = 1
    assert c._n_lanes(256) == 1
    c.lanes = 0
    assert c._n_lanes(256) == 1


def test_lane_sizes(monkeypatch):
    c = ImageCodec(engine=None, lanes=2)
    monkeypatch.delenv("IDF_LANE_SPLIT", raising=False)
    assert c._lane_sizes(256, 2) == [128, 128]
    assert c._lane_sizes(24, 3) == [8, 8, 8]
    monkeypatch.setenv("IDF_LANE_SPLIT", "0.4375")
    assert c._lane_sizes(256, 2) == [112, 144]
    assert c._lane_sizes(16, 2) == [8, 8]      # clamped to LANE_MIN images per lane
    assert c._lane_sizes(24, 3) == [8, 8, 8]   # the split applies to 2 lanes only


def test_bench_rans_roofline_accounting():
    """bench.py's rANS line: algorithmic bytes (12 B/symbol + 4 B/word + 16 B/stream) over the
    summed launch time, ns per symbol of a stream's chain."""
    import os
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench

    class Ev:
        def __init__(self, t):
            self.t = t

        def elapsed_time(self, other):
            return other.t - self.t

    class Bs:
        def total_words(self):
            return 1000

    # two decode launches of 2 ms each: 100 streams x 3000 symbols
    trace = [("decode", 300000, 100, Ev(0.0), Ev(2.0)), ("decode", 300000, 100, Ev(5.0), Ev(7.0)),
             ("encode", 600000, 200, Ev(9.0), Ev(10.0))]
    r = bench.rans_roofline(trace, Bs(), steps=1)
    d = r["decode"]
    assert d["launch_ms_per_step"] == 4.0
    assert abs(d["ns_per_symbol"] - 4.0e6 / 6000) < 0.1
    byts = 12.0 * 600000 + 4.0 * 1000 + 16.0 * 200
    assert abs(d["achieved"] - round(byts / 4e-3 / 1e9, 2)) < 1e-6
    assert abs(r["encode"]["frac"] - round(r["encode"]["achieved"] / bench.PEAK_HBM_GBS, 5)) < 1e-9
