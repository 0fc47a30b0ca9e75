"""Debug: one dense block of a config run on two HIP streams at once (each its own workspace)
vs the same block run alone: bitwise equal head outputs?
usage: python tools/dbg_block_conc.py <config> [level] [coupling|prior] [reps]"""
import os
import sys
import torch
sys.path.insert(0, "finalproject-losslessimagecompression_amd")
from idfcodec import _lib, synthetic
from idfcodec._lib import ptr, IdfHeadOut

name = sys.argv[1] if len(sys.argv) > 1 else "resflow-patches-vqvae"
lvl = int(sys.argv[2]) if len(sys.argv) > 2 else 0
which = sys.argv[3] if len(sys.argv) > 3 else "coupling"
reps = int(sys.argv[4]) if len(sys.argv) > 4 else 20
codec, fl, vq, size = synthetic.build_residual(name)
eng = fl.engine()
Lv = eng.levels[lvl]
blk = eng.couple[lvl][0] if which == "coupling" else eng.prior[lvl]
B = int(os.environ.get("DBG_B", "64"))
P = B * Lv.h * Lv.w
g = torch.Generator().manual_seed(5)
k0 = blk.geom.k_in[0]
print(name, "level", lvl, which, "B", B, "HxW", Lv.h, Lv.w, "k_in", list(blk.geom.k_in),
      "n_head", blk.geom.n_head, "fuse", blk.desc.fuse_head, "dx3", blk.desc.dx3, flush=True)
nh = blk.geom.n_head


def setup(slot):
    ws = eng.workspace(B, slot)
    x = (torch.randint(-64, 64, (P, k0), generator=g).float() / 256).cuda()
    if which == "coupling":
        a = Lv.a
        x[:, a:] = 0.0  # the pad columns past a_ch
    ws["feat"].view(-1, eng.ld_feat)[:P, :k0] = x
    out = torch.zeros(P, 16, device="cuda")
    return ws, x, out


def run(ws, x, out, s):
    ws["feat"].view(-1, eng.ld_feat)[:P, :k0] = x
    h = IdfHeadOut()
    h.mode = _lib.EPI_STORE
    h.out = ptr(out)
    h.ld_out = 16
    blk.run(s, B, Lv.h, Lv.w, ptr(ws["feat"]), eng.ld_feat, ptr(ws["tmp"]),
            eng.tmp_pitch(ws, P), h)


sets = [setup(1), setup(2)]
refs = []
for ws, x, out in sets:
    run(ws, x, out, _lib.stream_ptr())
    torch.cuda.synchronize()
    refs.append(out.clone())
    run(ws, x, out, _lib.stream_ptr())
    torch.cuda.synchronize()
    assert torch.equal(out, refs[-1]), "not deterministic alone"
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
nbad = [0, 0]
for r in range(reps):
    for i, (ws, x, out) in enumerate(sets):
        out.zero_()
    torch.cuda.synchronize()
    for i, (ws, x, out) in enumerate(sets):
        with torch.cuda.stream(streams[i]):
            run(ws, x, out, _lib.stream_ptr())
    torch.cuda.synchronize()
    for i, (ws, x, out) in enumerate(sets):
        d = (out != refs[i]).any(1)
        if d.any():
            nbad[i] += 1
            pix = d.nonzero().flatten()
            if nbad[i] <= 3:
                p0 = pix[0].item()
                print(f"rep {r} stream {i}: {pix.numel()} pixels differ, first {pix[:6].tolist()}"
                      f" (image {p0 // (Lv.h * Lv.w)}, y {p0 % (Lv.h * Lv.w) // Lv.w},"
                      f" x {p0 % Lv.w}); got {out[p0, :nh].tolist()} want {refs[i][p0, :nh].tolist()}",
                      flush=True)
print("runs with differences per stream:", nbad, "of", reps, flush=True)

import ctypes
from idfcodec._lib import lib as _l
try:
    buf = (ctypes.c_uint32 * 8)()
    _l().idf_dx3_debug_read(buf)
    print("head-init check: LDS table bad words", buf[0], buf[1], "; pixels whose LDS sums differ",
          buf[5], "max pixel", buf[6], flush=True)
except AttributeError:
    pass
