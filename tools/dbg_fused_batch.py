"""Debug: is a residual config's flow batch invariant (B patches at once vs two halves), and
does the inverse (teacher-forced latents) reproduce the input for each half?
usage: python tools/dbg_fused_batch.py <config name>"""
import sys
import torch
sys.path.insert(0, "finalproject-losslessimagecompression_amd")
from idfcodec import synthetic

name = sys.argv[1] if len(sys.argv) > 1 else "resflows_smallpatch_split"
codec, fl, vq, size = synthetic.build_residual(name)
src = (256, 256) if name == "resflows_smallpatch_split" else (215, 178)
x = synthetic.images(2, H=src[0], W=src[1], seed=23).cuda()
# the patches the residual codec hands the flow (residual.py encode)
img = codec._edge(x, codec.H, codec.W) if tuple(x.shape[2:]) != (codec.H, codec.W) else x
data = codec._dequant(img)
idx = vq.indices(data)
rec = vq.reconstruct(idx)
res = codec._pointwise(2, data, rec)
res_p, _ = codec.patch.forward(res, None)
cond = None
if codec.conditional:
    cond, _ = codec.patch.forward(rec, None)
    cond = cond.contiguous()
eng = fl.engine()
N = res_p.shape[0]
print(name, "patches", tuple(res_p.shape), "conv", eng.conv_mode, flush=True)


def fwd(lo, hi, slot):
    ws = eng.load_nchw(res_p[lo:hi], slot=slot)
    ws = eng.forward_pm(hi - lo, cond=None if cond is None else cond[lo:hi], slot=slot)
    torch.cuda.synchronize()
    return {k: ws[k].clone() for k in ("lat", "mean", "logscale")}


full = fwd(0, N, 0)
h = N // 2
parts = [fwd(0, h, 1), fwd(h, N, 2)]
offs_f = eng.sym_offsets(N)
offs_h = [eng.sym_offsets(h), eng.sym_offsets(N - h)]
for key in ("lat", "mean", "logscale"):
    for l in range(len(eng.levels)):
        Lv = eng.levels[l]
        per = Lv.n_sym if hasattr(Lv, "n_sym") else None
        f = full[key][offs_f[l]:offs_f[l + 1]].view(N, -1)
        p0 = parts[0][key][offs_h[0][l]:offs_h[0][l + 1]].view(h, -1)
        p1 = parts[1][key][offs_h[1][l]:offs_h[1][l + 1]].view(N - h, -1)
        g = torch.cat([p0, p1])
        bad = (f != g).any(1).nonzero().flatten()
        print(f"{key} level {l}: images differing {bad.numel()}",
              bad[:8].tolist(), flush=True)

# teacher-forced inverse: the full batch's latents, decoded as one batch, as two halves one
# after the other, and as two halves on two streams at once
lat_full = full["lat"]


import os
PRIORS = os.environ.get("DBG_PRIORS", "1") == "1"
if os.environ.get("DBG_KEEP") == "1":
    for blks in eng.couple + [[b] for b in eng.prior]:
        for b in blks:
            b.desc.keep_feat = 1
    print("keep_feat = 1", flush=True)


def inv(lo, hi, slot):
    n = hi - lo
    offs = eng.sym_offsets(n)

    def dec(l, ws):
        src = lat_full[offs_f[l]:offs_f[l + 1]].view(N, -1)[lo:hi].reshape(-1)
        ws["lat"][offs[l]:offs[l + 1]].copy_(src)
    return eng.inverse_pm_steps(n, dec, cond=None if cond is None else cond[lo:hi], slot=slot,
                                priors=PRIORS)


def run_gen(g):
    while True:
        try:
            next(g)
        except StopIteration as d:
            return d.value


def check(tag, lo, hi, ws):
    n = hi - lo
    out = eng.image_nchw(ws, n)
    torch.cuda.synchronize()
    bad = (out != res_p[lo:hi]).flatten(1).any(1).nonzero().flatten()
    print(f"inverse {tag} [{lo},{hi}): patches differing {bad.numel()}", (bad + lo)[:8].tolist(),
          flush=True)
    for b in bad[:3].tolist():
        d = (out[b] - res_p[lo + b]).flatten()
        nz = d.nonzero().flatten()
        print(f"   patch {lo + b}: {nz.numel()} values differ, max |d| {d.abs().max().item():.6g},"
              f" d*256 {(d[nz[:6]] * 256).tolist()}", flush=True)


check("one batch", 0, N, run_gen(inv(0, N, 0)))
check("half seq", 0, h, run_gen(inv(0, h, 1)))
check("half seq", h, N, run_gen(inv(h, N, 2)))
streams = [torch.cuda.Stream(), torch.cuda.Stream()]
# forward halves on two streams at once vs the sequential forward
for rep in range(3):
    outs = [None, None]
    gens = []
    for i, (lo, hi) in enumerate(((0, h), (h, N))):
        with torch.cuda.stream(streams[i]):
            eng.load_nchw(res_p[lo:hi], slot=1 + i)
            gens.append(eng.forward_pm_steps(hi - lo, cond=None if cond is None else cond[lo:hi],
                                             slot=1 + i))
    live = [0, 1]
    while live:
        for i in list(live):
            with torch.cuda.stream(streams[i]):
                try:
                    next(gens[i])
                except StopIteration as d:
                    outs[i] = d.value
                    live.remove(i)
    torch.cuda.synchronize()
    for key in ("lat", "mean", "logscale"):
        for l in range(len(eng.levels)):
            f = full[key][offs_f[l]:offs_f[l + 1]].view(N, -1)
            g = torch.cat([outs[0][key][offs_h[0][l]:offs_h[0][l + 1]].view(h, -1),
                           outs[1][key][offs_h[1][l]:offs_h[1][l + 1]].view(N - h, -1)])
            bad = (f != g).any(1).nonzero().flatten()
            if bad.numel():
                print(f"forward conc{rep} {key} level {l}: images differing {bad.numel()}",
                      bad[:8].tolist(), flush=True)
SOLO = os.environ.get("DBG_SOLO") == "1"
junk = torch.randn(4096, 4096, device="cuda")
for rep in range(3):
    gens = []
    if SOLO:  # lane 0 alone beside an unrelated GEMM stream
        with torch.cuda.stream(streams[1]):
            for _ in range(40):
                junk = (junk @ junk).clamp_(-1, 1)
        with torch.cuda.stream(streams[0]):
            r = run_gen(inv(0, h, 1))
        torch.cuda.synchronize()
        check(f"solo{rep}", 0, h, r)
        continue
    for i, (lo, hi) in enumerate(((0, h), (h, N))):
        with torch.cuda.stream(streams[i]):
            gens.append(inv(lo, hi, 1 + i))
    live = [0, 1]
    res = [None, None]
    while live:
        for i in list(live):
            with torch.cuda.stream(streams[i]):
                try:
                    next(gens[i])
                except StopIteration as d:
                    res[i] = d.value
                    live.remove(i)
    torch.cuda.synchronize()
    check(f"half conc{rep}", 0, h, res[0])
    check(f"half conc{rep}", h, N, res[1])

import ctypes
from idfcodec._lib import lib as _l
try:
    fn = _l().idf_dx3_debug_read
    buf = (ctypes.c_uint32 * 8)()
    fn(buf)
    print("head-init LDS check: bad words", buf[0], buf[1], "first idx", buf[2], buf[3],
          "value", hex(buf[4]), flush=True)
except AttributeError:
    pass
