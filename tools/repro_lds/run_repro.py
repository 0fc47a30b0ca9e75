"""Reproducer run (GPU): the four LDS-table head-init forms of head_init_variants.hip, each
launched repeatedly on one non-blocking stream while another non-blocking stream runs the
imagenet64 level-0 fused DenseBlock (dx3 layers: one 149.5 KiB-LDS block per CU, LDS-DMA,
ds_read_b128 and MFMA; a 4 KiB head-init block fits beside it) -- the co-residency of two decode
lanes -- and alone.  Every output is compared bit for bit with the product head init
(idf_dx3_head_init, global weights) run alone.  Prints, per variant and condition, the launches
with differences, the differing pixels and their runs (length, 16-pixel alignment).
usage: python tools/repro_lds/run_repro.py [reps]"""
import ctypes
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "finalproject-losslessimagecompression_amd"))
from idfcodec import _lib, configs, synthetic  # noqa: E402
from idfcodec._lib import IdfHeadOut, ptr  # noqa: E402

reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
K = 24  # variant launches per rep
rl = ctypes.CDLL(os.path.join(REPO, "tools", "repro_lds", "librepro_lds.so"))
rl.repro_head_init.restype = ctypes.c_int
rl.repro_head_init.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int32,
                               ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int32,
                               ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]
L = _lib.lib()

# the head init's problem: config 5's 27 x 23 patches at B = 64, C0 = 64 inputs, 16 outputs
P, C0, NH = 64 * 27 * 23, 64, 16
g = torch.Generator().manual_seed(7)
x = (torch.randint(-64, 64, (P, C0), generator=g).float() / 256).cuda()
w = (torch.randn(NH, C0, generator=g) * 0.05).cuda()
bias = (torch.randn(NH, generator=g) * 0.1).cuda()
ref = torch.zeros(P, 16, device="cuda")
_lib.check(L.idf_dx3_head_init(_lib.stream_ptr(), P, C0, ptr(x), C0, ptr(w), C0, ptr(bias), NH,
                               ptr(ref)), "head init")
torch.cuda.synchronize()

# the contention: imagenet64 level 0's first coupling block (fused head, dx3 layers), B = 64
model = synthetic.build_model(configs.get("imagenet64")).cuda()
eng = model.engine()
Lv = eng.levels[0]
blk = eng.couple[0][0]
assert blk.desc.fuse_head == 1 and blk.desc.dx3 == 1
Bc = 64
Pc = Bc * Lv.h * Lv.w
k0 = blk.geom.k_in[0]
ws = eng.workspace(Bc, 1)
xc = (torch.randint(-64, 64, (Pc, k0), generator=g).float() / 256).cuda()
xc[:, Lv.a:] = 0.0
outc = torch.zeros(Pc, 16, device="cuda")


def run_block(stream):
    with torch.cuda.stream(stream):
        ws["feat"].view(-1, eng.ld_feat)[:Pc, :k0] = xc
        h = IdfHeadOut()
        h.mode, h.out, h.ld_out = _lib.EPI_STORE, ptr(outc), 16
        blk.run(_lib.stream_ptr(), Bc, Lv.h, Lv.w, ptr(ws["feat"]), eng.ld_feat, ptr(ws["tmp"]),
                eng.tmp_pitch(ws, Pc), h)


sA, sB = _lib.new_stream(), _lib.new_stream()
outs = torch.empty(K, P, 16, device="cuda")


def runs_of(mask):
    """(length, start % 16) of each run of consecutive differing pixels"""
    idx = mask.nonzero().flatten().tolist()
    res, i = [], 0
    while i < len(idx):
        j = i
        while j + 1 < len(idx) and idx[j + 1] == idx[j] + 1:
            j += 1
        res.append((j - i + 1, idx[i] % 16))
        i = j + 1
    return res


print(f"head init P {P} C0 {C0} n_head {NH}; contention: imagenet64 L0 coupling block B {Bc}, "
      f"{reps} reps x {K} launches per variant and condition", flush=True)
t0 = time.time()
for variant in (2, 4, 1, 3):
    for contended in (False, True):
        bad_launch, bad_pix, runs, inside = 0, 0, [], []
        for r in range(reps):
            outs.zero_()
            torch.cuda.synchronize()
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
            ev[0].record(torch.cuda.current_stream())
            torch.cuda.current_stream().synchronize()
            if contended:  # two block runs: the head inits all fall inside its dx3 layers
                run_block(sA)
                run_block(sA)
                ev[1].record(sA)
            with torch.cuda.stream(sB):
                ev[2].record(sB)
                for k in range(K):
                    rc = rl.repro_head_init(variant, _lib.stream_ptr(), P, C0, ptr(x), C0, ptr(w), C0,
                                            ptr(bias), NH, ptr(outs[k]))
                    assert rc == 0, rc
                ev[3].record(sB)
            torch.cuda.synchronize()
            if contended:  # the variant's launches ended before the block did: they ran beside it
                inside.append(ev[0].elapsed_time(ev[3]) < ev[0].elapsed_time(ev[1]))
            d = (outs != ref.unsqueeze(0)).any(2)  # [K, P]
            nb = d.any(1)
            bad_launch += int(nb.sum())
            bad_pix += int(d.sum())
            for k in nb.nonzero().flatten().tolist():
                if len(runs) < 12:
                    runs += runs_of(d[k])[:4]
        print(f"variant {variant} {'beside the dx3 block' if contended else 'alone':>20}: "
              f"{bad_launch} / {reps * K} launches differ, {bad_pix} pixels; runs (len, start%16) "
              f"{runs[:12]}" + (f"; variant launches ended inside the block's run in "
                                f"{sum(inside)} / {len(inside)} reps" if contended else ""), flush=True)
print(f"done in {time.time() - t0:.1f} s", flush=True)
