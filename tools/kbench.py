"""Kernel microbenchmark of the folded 3x3 conv at the imagenet64 shapes (B=256): the LDS
halo-tiled kernel (idf_conv3x3_halo) and the implicit-GEMM kernel (idf_conv3x3_fold_f32),
per level and layer width.  Prints achieved TFLOP/s (unpadded FLOPs).
Env filters: KB_ONLY=wino,wx3,dx3,halo,gemm,bf16,dxb  KB_LEVELS=0,1,2  KB_LAYERS=0,3,6,9,11  KB_REPS=10."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "finalproject-losslessimagecompression_amd"))

import torch  # noqa: E402

from idfcodec import _lib  # noqa: E402
from idfcodec._lib import check, lib, ptr  # noqa: E402
from idfcodec.packing import round_up  # noqa: E402


def time_it(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    B = int(os.environ.get("KB_B", "256"))
    dev = torch.device("cuda")
    s = _lib.stream_ptr()
    g_pad, g_alloc, g_real = 44, 48, 43
    only = os.environ.get("KB_ONLY", "wino,wx3,dx3,halo,gemm,bf16").split(",")
    layers = [int(v) for v in os.environ.get("KB_LAYERS", "0,3,6,9,11").split(",")]
    levels = [int(v) for v in os.environ.get("KB_LEVELS", "0,1,2").split(",")]
    reps = int(os.environ.get("KB_REPS", "10"))
    tot = {k: [0.0, 0.0] for k in only}
    import numpy as np
    from idfcodec.packing import wino_weights
    for lvl, (hw, a) in enumerate(((32, 9), (16, 18), (8, 36))):
        if lvl not in levels:
            continue
        P = B * hw * hw
        for layer in layers:
            c_pad = round_up(a, 4) + layer * g_pad
            c_real = a + layer * 512 // 12
            ld = round_up(c_pad + g_pad, 16)
            feat = torch.randn(P * ld, device=dev)
            ldw = round_up(c_pad, 16)
            w = torch.randn(g_alloc * 9 * ldw, device=dev) * 0.01
            b3 = torch.zeros(g_alloc, device=dev)
            vt = torch.zeros(9 * g_alloc, device=dev)
            wsn = lib().idf_conv3x3_halo_workspace(B, hw, hw, c_pad, g_pad)
            ws = torch.empty(max(wsn, 1), device=dev)
            fl = 2.0 * P * 9 * c_real * g_real

            def halo():
                check(lib().idf_conv3x3_halo(s, B, hw, hw, c_pad, ptr(feat), ld, ptr(w), ldw, g_alloc,
                                             ptr(b3), ptr(vt), g_alloc, ptr(b3), g_pad,
                                             ptr(feat) + c_pad * 4, ld, 0, 0.0, ptr(ws), wsn), "halo")

            U = torch.from_numpy(wino_weights(np.random.default_rng(0).normal(
                0, 0.01, (g_alloc, 9, ldw)), ldw // 16)).to(dev)
            wwn = lib().idf_conv3x3_wino_workspace(B, hw, hw, c_pad, g_pad)
            wws = torch.empty(max(wwn, 1), device=dev)

            def wino():
                check(lib().idf_conv3x3_wino(s, B, hw, hw, c_pad, ptr(feat), ld, ptr(U), g_alloc // 16,
                                             ptr(b3), ptr(vt), g_alloc, ptr(b3), g_pad,
                                             ptr(feat) + c_pad * 4, ld, 0, 0.0, ptr(wws), wwn), "wino")

            from idfcodec.packing import wino_weights_x3
            UX, ysc = wino_weights_x3(np.random.default_rng(0).normal(
                0, 0.01, (g_alloc, 9, ldw)), ldw // 16)
            UX = torch.from_numpy(UX.view(np.int16)).to(dev)
            flag = torch.zeros(1, dtype=torch.int32, device=dev)

            def wx3():
                check(lib().idf_conv3x3_wx3(s, B, hw, hw, c_pad, ptr(feat), ld, ptr(UX), g_alloc // 16,
                                            ysc, ptr(b3), ptr(vt), g_alloc, ptr(b3), g_pad,
                                            ptr(feat) + c_pad * 4, ld, 0, 0.0, ptr(flag), 0, ptr(wws),
                                            wwn), "wx3")

            from idfcodec.packing import dx3_weights
            WD, dsc = dx3_weights(np.random.default_rng(0).normal(0, 0.01, (g_alloc, 9, ldw)), c_pad)
            WD = torch.from_numpy(WD.view(np.int16)).to(dev)
            xs = None
            dws, dwn = None, 0
            if "dx3" in only:
                nsx = (c_pad + g_pad + 15) // 16
                xs = torch.empty(nsx * 2 * P * 16, dtype=torch.int16, device=dev)
                check(lib().idf_dx3_split_cols(s, P, 0, c_pad, ptr(feat), ld, ptr(xs), nsx, ptr(flag),
                                               None, 0), "split")
                dwn = int(lib().idf_conv3x3_dx3_workspace(B, hw, hw, c_pad, g_pad))
                if dwn > 0:  # split K: zeroed counters (each launch leaves them zero)
                    dws = torch.zeros(dwn // 4, dtype=torch.int32, device=dev)

            def dx3():
                check(lib().idf_conv3x3_dx3(s, B, hw, hw, c_pad, ptr(xs), nsx, ptr(WD), g_alloc // 16,
                                            dsc, ptr(b3), ptr(vt), g_alloc, ptr(b3), g_pad,
                                            ptr(feat) + c_pad * 4, ld, 0, 0.0, ptr(flag), ptr(dws),
                                            dwn, None), "dx3")

            # KB_ONLY=dx3r4: round 4's dx3 kernel (tools/ab_lib/dx3_r4/libdx3old.so, built from
            # that commit's conv3_dx3.hip) on the same box, same data -- its old ABI
            old = None
            if "dx3r4" in only:
                import ctypes
                old = ctypes.CDLL(os.path.join(REPO, "tools", "ab_lib", "dx3_r4", "libdx3old.so"))
                P_, i32_, i64_, f32_ = ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64, ctypes.c_float
                old.idf_conv3x3_dx3.argtypes = [P_, i32_, i32_, i32_, i32_, P_, i32_, P_, i32_, f32_,
                                                P_, P_, i32_, P_, i32_, P_, i64_, i32_, f32_, P_]
                if xs is None:
                    nsx = (c_pad + g_pad + 15) // 16
                    xs = torch.empty(nsx * 2 * P * 16, dtype=torch.int16, device=dev)
                    check(lib().idf_dx3_split_cols(s, P, 0, c_pad, ptr(feat), ld, ptr(xs), nsx,
                                                   ptr(flag), None, 0), "split")

            def dx3r4():
                check(old.idf_conv3x3_dx3(s, B, hw, hw, c_pad, ptr(xs), nsx, ptr(WD), g_alloc // 16,
                                          dsc, ptr(b3), ptr(vt), g_alloc, ptr(b3), g_pad,
                                          ptr(feat) + c_pad * 4, ld, 0, 0.0, ptr(flag)), "dx3r4")

            from idfcodec.packing import bf16_weights
            WB = torch.from_numpy(bf16_weights(np.random.default_rng(1).normal(
                0, 0.01, (g_alloc, 9, ldw)).astype(np.float32), c_pad).view(np.int16)).to(dev)
            bwn = lib().idf_conv3x3_bf16_workspace(B, hw, hw, c_pad, g_pad)
            bws = torch.empty(max(bwn, 1), device=dev)

            ld16 = (ld + 7) // 8 * 8
            f16 = torch.zeros(P * ld16, dtype=torch.int16, device=dev)
            n16 = (c_pad + g_pad + 7) // 8 * 8 - c_pad

            def bf16():
                check(lib().idf_conv3x3_bf16(s, B, hw, hw, c_pad, ptr(f16), ld16, ptr(WB), g_alloc,
                                             ptr(b3), ptr(vt), g_alloc, ptr(b3), g_pad,
                                             ptr(feat) + c_pad * 4, ld, ptr(f16) + c_pad * 2, ld16,
                                             n16, 0, 0.0, ptr(bws), bwn), "bf16")

            from idfcodec.packing import dxb_weights
            WDB = torch.from_numpy(dxb_weights(np.random.default_rng(1).normal(
                0, 0.01, (g_alloc, 9, ldw)).astype(np.float32), c_pad).view(np.int16)).to(dev)
            nsb = (c_pad + g_pad + 15) // 16
            fb = None
            xwn, xws = 0, None
            if "dxb" in only:
                fb = torch.zeros(nsb * P * 16, dtype=torch.int16, device=dev)
                check(lib().idf_dxb_cols(s, P, 0, c_pad, ptr(feat), ld, ptr(fb), nsb, None, 0),
                      "to bf16")
                xwn = int(lib().idf_conv3x3_dx3_workspace(B, hw, hw, c_pad, g_pad))
                if xwn > 0:
                    xws = torch.zeros(xwn // 4, dtype=torch.int32, device=dev)

            def dxb():
                check(lib().idf_conv3x3_dxb(s, B, hw, hw, c_pad, ptr(fb), nsb, ptr(WDB),
                                            g_alloc // 16, ptr(b3), ptr(vt), g_alloc, ptr(b3), g_pad,
                                            ptr(feat) + c_pad * 4, ld, 0, 0.0, ptr(xws), xwn, None),
                      "dxb")

            def gemm():
                check(lib().idf_conv3x3_fold_f32(s, B, hw, hw, c_pad, ptr(feat), ld, ptr(w), ldw,
                                                 g_alloc, ptr(b3), ptr(vt), g_alloc, ptr(b3), g_pad,
                                                 ptr(feat) + c_pad * 4, ld, 0, 0.0), "gemm")
            line = f"L{lvl} hw={hw:2d} c={c_pad:4d} P={P:7d}"
            for name, fn in (("wino", wino), ("wx3", wx3), ("dx3", dx3), ("dx3r4", dx3r4),
                             ("halo", halo), ("gemm", gemm), ("bf16", bf16), ("dxb", dxb)):
                if name not in only:
                    continue
                ms = time_it(fn, reps)
                tot[name][0] += ms
                tot[name][1] += fl
                line += f"  {name} {ms*1e3:8.1f} us {fl/ms/1e9:6.1f} TF/s"
            print(line, flush=True)
    for k, (ms, fl) in tot.items():
        if ms > 0:
            print(f"{k}: sampled total {ms:.2f} ms  {fl/ms/1e9:.1f} TF/s")


if __name__ == "__main__":
    main()
