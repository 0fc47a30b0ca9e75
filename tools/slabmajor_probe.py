"""Timing-only probe of the slab-major premise (DESIGN "where round 3 leaves the hot kernel"):
the split-f16 Winograd convs at L0 c=496 (B=256, 32x32) reading their input with the DenseBlock
stride (ld 544: a slab's 64 B per pixel, 2176 B apart) and with ld 16 (consecutive pixels'
64-B pieces adjacent, as a [slab][pixel][16] layout would make them; the values read are
wrong -- timing only).  IDF_WQ=1 times wq, IDF_WQ=0 wx3."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "finalproject-losslessimagecompression_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from idfcodec import _lib  # noqa: E402
from idfcodec._lib import check, lib, ptr  # noqa: E402
from idfcodec.packing import round_up, wino_weights_x3  # noqa: E402


def main():
    B, hw, c = 256, 32, 496
    P = B * hw * hw
    dev = torch.device("cuda")
    s = _lib.stream_ptr()
    g_alloc, g_pad = 48, 44
    ldw = round_up(c, 16)
    UX, ysc = wino_weights_x3(np.random.default_rng(0).normal(0, 0.01, (g_alloc, 9, ldw)), ldw // 16)
    UX = torch.from_numpy(UX.view(np.int16)).to(dev)
    b3 = torch.zeros(g_alloc, device=dev)
    vt = torch.zeros(9 * g_alloc, device=dev)
    flag = torch.zeros(1, dtype=torch.int32, device=dev)
    out = torch.empty(P * 48, device=dev)
    res = {}
    for ld in (544, 16):
        X = torch.randn(P * ld + 64, device=dev) * 0.1
        wsn = lib().idf_conv3x3_wino_workspace(B, hw, hw, c, g_pad)
        ws = torch.empty(max(wsn, 1), device=dev)

        def run():
            check(lib().idf_conv3x3_wx3(s, B, hw, hw, c, ptr(X), ld, ptr(UX), g_alloc // 16, ysc,
                                        ptr(b3), ptr(vt), g_alloc, ptr(b3), g_pad, ptr(out), 48, 0,
                                        0.0, ptr(flag), 0, ptr(ws), wsn), "wx3")
        run()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            run()
        b.record()
        torch.cuda.synchronize()
        res[ld] = a.elapsed_time(b) / 10 * 1e3
        del X
    kind = "wq" if os.environ.get("IDF_WQ") == "1" else "wx3"
    print(f"{kind}: L0 c={c} ld 544 {res[544]:.1f} us | ld 16 (slab-major access) {res[16]:.1f} us",
          flush=True)


if __name__ == "__main__":
    main()
