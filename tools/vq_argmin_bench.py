"""Timing of the VQ argmin (idf_vq_argmin_ws) at the residual configs' shapes: rows x codes x
dim, one-pass (no workspace) and sliced.  Prints us per launch and fp32 MFMA TFLOP/s
(2 P K D per launch; peak 157.3)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "finalproject-losslessimagecompression_amd"))
import torch  # noqa: E402

from idfcodec import _lib  # noqa: E402
from idfcodec._lib import check, lib, ptr  # noqa: E402

SHAPES = [("config4 B=8", 8192, 8192, 512), ("config5 B=32", 19872, 8192, 512),
          ("config3 B=1024", 65536, 16384, 512)]


def main():
    s = _lib.stream_ptr()
    for name, P, K, D in SHAPES:
        x = torch.tanh(torch.randn(P, D, device="cuda"))
        e = torch.randn(K, D, device="cuda") * 0.5
        en = torch.empty(K, device="cuda")
        check(lib().idf_vq_norms(s, K, D, ptr(e), D, ptr(en)), "norms")
        idx = torch.empty(P, dtype=torch.int32, device="cuda")
        nws = int(lib().idf_vq_argmin_workspace_bytes(P, K))
        ws = torch.empty(max(nws, 1), dtype=torch.uint8, device="cuda")
        for label, n in (("one-pass", 0), ("sliced", nws)):
            def run():
                check(lib().idf_vq_argmin_ws(s, P, D, ptr(x), D, ptr(e), D, K, ptr(en), ptr(idx),
                                             ptr(ws), n), "argmin")
            run()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 5
            a.record()
            for _ in range(reps):
                run()
            b.record()
            torch.cuda.synchronize()
            ms = a.elapsed_time(b) / reps
            tf = 2.0 * P * K * D / (ms * 1e-3) / 1e12
            print(f"{name:16s} P={P:6d} K={K:6d} {label:9s} {ms * 1e3:9.1f} us  {tf:6.1f} TF/s "
                  f"({tf / 157.3:.2f} of f32 MFMA peak)", flush=True)


if __name__ == "__main__":
    main()
