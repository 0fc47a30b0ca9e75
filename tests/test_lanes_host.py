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
