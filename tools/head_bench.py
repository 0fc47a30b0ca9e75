"""Timing of the DenseBlock head GEMM shapes (imagenet64, B=256): the streaming head kernel
(N <= 16) against the tiled GEMM (N = 20 -> BN = 32 tiles), us per launch and HBM GB/s of the
P x K fp32 stream."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "finalproject-losslessimagecompression_amd"))
import torch  # noqa: E402

from idfcodec import _lib  # noqa: E402
from idfcodec._lib import check, lib, ptr  # noqa: E402


def main():
    s = _lib.stream_ptr()
    for name, P, K in (("L0", 262144, 540), ("L1", 65536, 548), ("L2", 16384, 564)):
        lda = 576
        a = torch.randn(P, lda, device="cuda")
        w = torch.randn(32, 576, device="cuda") * 0.05
        b = torch.zeros(32, device="cuda")
        o = torch.empty(P, 32, device="cuda")
        for N in (3, 12, 20):
            def run():
                check(lib().idf_conv1x1_f32(s, P, K, N, ptr(a), lda, ptr(w), 576, 32, ptr(b), ptr(o),
                                            32, 1, P, 1, None), "gemm")
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 100
            print(f"{name} P={P} K={K} N={N:2d}: {us:7.1f} us  {P * K * 4 / (us * 1e-6) / 1e9:6.0f} GB/s",
                  flush=True)


if __name__ == "__main__":
    main()
