"""Throughput of the residual configs' codec (BASELINE configs[2..4]) on one or more GPUs.

Default: resflow-cond-imagenet64 (configs[2]), batch 1024 synthetic 64x64x3 uint8, seeded
weights (the configs' checkpoints are absent).  One step = ResidualCodec.encode then
decode of the batch, inputs resident in HBM.  Prints one JSON line: Mpx/s (encode+decode),
the encode / decode split, the VQ-VAE share of each, bits per pixel (flow streams + index
code) and the exactness of the round trip.  The flow's DenseLayer convs run in the config's
precision (bf16 MFMA for resflow-cond-imagenet64, as BASELINE configs[2] names; --precision
overrides).  Config 5's images are generated at their 215x178 source size and go through
the dataloader's replication pad (trainer.py:62) inside the codec.

Multi-GPU (configs[3]/[4] are 8-GPU configs): launched under torch.distributed.run, each rank
codes a contiguous slice of the global batch (no data-path collective) and the per-rank
bitstreams are gathered to rank 0 over RCCL (idfcodec.dist.gather_residual) inside the
timed encode; every rank then decodes its own shard.  Times are the max over ranks and the
pixel count is the whole batch (weak scaling when --batch is per rank, the default).

  python tools/bench_residual.py [--config NAME] [--batch B] [--steps K] [--warmup W]
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \\
      tools/bench_residual.py --config resflows_smallpatch_split
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "finalproject-losslessimagecompression_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

# images per GPU: config 3's B=1024 (BASELINE configs[2]); configs 4/5 sized to a few
# thousand flow patches per GPU (1024 8x8 patches per 256x256 image, 64 27x23 per image)
DEFAULT_BATCH = {"resflow-cond-imagenet64": 1024, "resflows_smallpatch_split": 8,
                 "resflow-patches-vqvae": 32}


PEAK_TFLOPS = {"bf16": 2500.0, "dxb": 2500.0, "x3": 2500.0, "dx3": 2500.0, "dx3w16": 2500.0,
               "f32": 157.3}  # MI355X_MICROARCH.md dense peaks


def flow_conv_roofline(codec, fl, img):
    """The flow's DenseLayer 3x3 convs (the residual configs' dominant kernel family) timed
    live: one encode after the timed steps, side-stream rANS off, HIP events around every
    conv launch on its own stream (idf_dense_block_f32_timed).  Algorithmic FLOPs per launch
    = 2*P*9*c*g of the unpadded layer; peak = the dense MFMA peak of the arithmetic the
    launches ran (bf16 / split-f16 on f16 MFMA / f32 MFMA)."""
    import ctypes
    from idfcodec import _lib
    eng = fl.engine()
    ic = codec._codec()
    L = _lib.lib()
    timer = L.idf_timer_create(65536)
    for b in eng._blocks:
        b.timer = timer
    prev = ic.overlap_encode
    ic.overlap_encode = False
    try:
        codec.encode(img)
        torch.cuda.synchronize()
        tot, cnt, fl_ = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
        _lib.check(L.idf_timer_summary(timer, _lib.TAG_CONV3X3, ctypes.byref(tot),
                                       ctypes.byref(cnt), ctypes.byref(fl_)), "timer")
    finally:
        ic.overlap_encode = prev
        for b in eng._blocks:
            b.timer = None
        L.idf_timer_destroy(timer)
    from idfcodec.engine import SPLIT_F16
    split = eng.wino and eng.conv_mode in SPLIT_F16
    mode = eng.conv_mode if eng.precision == "bf16" else (eng.conv_mode if split else "f32")
    nd = [(l, len(b.dx3_w)) for l in range(eng.nsplit) for b in eng.couple[l] + [eng.prior[l]]]
    dx3_levels = sorted({eng.levels[l].h for l, n in nd if n and eng.dx3_layers(l, eng.prior[l].geom)})
    kern = {"bf16": "conv3_bf16_kernel (bf16 MFMA, f32 accumulate)",
            "dxb": "conv3_dx3_kernel<..., true> (direct conv, one bf16 product per tap on bf16 "
                   "MFMA, f32 accumulate, packed tiles)",
            "x3": "conv3_wino_kernel<..., true, ...> (Winograd, split-f16 products on f16 MFMA)",
            "f32": "conv3_wino_kernel (Winograd, f32 MFMA)"}.get(
        mode, "conv3_dx3_kernel (direct split-f16 products on f16 MFMA, packed tiles) at levels "
              f"of height {dx3_levels}, conv3_wino_kernel<..., true, ...> elsewhere")
    n = max(cnt.value, 1)
    achieved = fl_.value / (tot.value * 1e-3) / 1e12 if tot.value > 0 else 0.0
    peak = PEAK_TFLOPS[mode]
    return {"kernel": "DenseLayer 3x3 conv, 1x1 folded in: " + kern, "bound": "mfma",
            "launches": cnt.value, "avg_launch_ms": round(tot.value / n, 5),
            "conv_ms_per_encode": round(tot.value, 3),
            "algorithmic_gflop_per_launch": round(fl_.value / n / 1e9, 4),
            "achieved": round(achieved, 3), "peak": peak, "unit": "TFLOP/s",
            "frac": round(achieved / peak, 4), "conv_mode": mode}


VQ_PEAK = {"conv_taps": ("f32 MFMA", 157.3), "argmin": ("f32 MFMA", 157.3),
           "conv_taps_x3": ("f16 MFMA (split-f16 products)", 2500.0),
           "resblock3x3_x3": ("f16 MFMA (split-f16 products)", 2500.0),
           "resblock3x3_f32": ("f32 MFMA", 157.3),
           "argmin_x3": ("f16 MFMA (split-f16 products)", 2500.0)}
VQ_KERNEL = {"conv_taps": "conv_taps_kernel (strided / transposed VQ-VAE convs as tap GEMMs)",
             "conv_taps_x3": "conv_taps_kernel<..., X3=true> (the tap GEMMs with split-f16 "
                             "products on v_mfma_f32_16x16x16_f16, VQ conv mode x3t)",
             "argmin": "vq_argmin_kernel (+vq_argmin_merge_kernel): fused distance + running "
                       "min over the codebook, 2*D*K FLOP per latent",
             "argmin_x3": "vq_argmin_kernel<true> (+merge): the codebook search with split-f16 "
                          "x.e products on v_mfma_f32_16x16x16_f16, 2*D*K FLOP per latent",
             "resblock3x3_x3": "conv3_wino_kernel<..., true, ...> via idf_conv3x3_wx3_res "
                               "(ResBlock 3x3, split-f16 Winograd, residual fused)",
             "resblock3x3_f32": "conv3_wino_kernel via idf_conv3x3_wino_res (exact f32)"}


def vq_roofline(codec, img):
    """The VQ-VAE's kernels timed live over one encode + decode after the timed steps: HIP
    events around every conv and argmin launch on its stream (VQEngine.timer).  Per kind:
    launches, milliseconds per encode + decode, algorithmic FLOPs (2 x taps x cin x cout per
    computed output; the Winograd ResBlock convs priced as the direct 3x3 they compute; argmin
    2 x D x K per latent) over the summed launch time, against the dense peak of the kind's
    arithmetic."""
    vqe = codec.vqvae.engine()
    vqe.timer = []
    try:
        codec.decode(codec.encode(img), verify=False)
        torch.cuda.synchronize()
        recs = vqe.timer
    finally:
        vqe.timer = None
    out = {}
    for kind in sorted({r[0] for r in recs}):
        rs = [r for r in recs if r[0] == kind]
        ms = sum(a.elapsed_time(b) for _, _, a, b in rs)
        fl = sum(r[1] for r in rs)
        what, peak = VQ_PEAK[kind]
        tf = fl / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
        out[kind] = {"kernel": VQ_KERNEL[kind], "launches": len(rs), "ms": round(ms, 3),
                     "gflop": round(fl / 1e9, 3), "achieved": round(tf, 3), "peak": peak,
                     "peak_of": what, "unit": "TFLOP/s", "frac": round(tf / peak, 4)}
    tot = sum(v["ms"] for v in out.values())
    dom = max(out, key=lambda k: out[k]["ms"]) if out else None
    return {"per_kind": out, "vq_kernel_ms_per_encode_decode": round(tot, 3),
            "dominant": dom, "bound": "mfma",
            "sampled": "every VQ-VAE conv / argmin launch of one encode + decode after the "
                       "timed steps"}


def phase_split(phases, steps):
    """Mean ms per phase of the timed steps from ResidualCodec's (name, event) marks."""
    acc = {}
    for marks in phases:
        for (_, a), (name, b) in zip(marks, marks[1:]):
            acc[name] = acc.get(name, 0.0) + a.elapsed_time(b)
    return {k: round(v / steps, 3) for k, v in acc.items()}


def run(config: str, batch: int | None = None, steps: int = 10, warmup: int = 2,
        precision: str | None = None) -> dict | None:
    """One residual config's encode+decode throughput on this rank's GPU (the process group,
    if any, already initialised).  Returns the result dict on rank 0, None elsewhere."""
    world = dist.get_world_size() if dist.is_initialized() else 1
    rank = dist.get_rank() if dist.is_initialized() else 0
    dev = torch.device("cuda", torch.cuda.current_device())
    from idfcodec import configs, synthetic
    from idfcodec.dist import all_reduce, gather_residual
    codec, fl, vq, (H, W) = synthetic.build_residual(config, device=dev, precision=precision)
    pb, pr = configs.PAD.get(config, (0, 0))
    Hs, Ws = H - pb, W - pr
    per = batch or DEFAULT_BATCH.get(config, 8)
    full = synthetic.images(per * world, H=Hs, W=Ws, seed=2)
    img = full[rank * per:(rank + 1) * per].to(dev)

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    def vq_time():
        data = codec._dequant(codec._edge(img, H, W))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        idx = vq.indices(data)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        vq.reconstruct(idx)
        torch.cuda.synchronize()
        return t1 - t0, time.perf_counter() - t1

    for _ in range(warmup):
        out, info = codec.decode(codec.encode(img))
    sync()
    te = td = 0.0
    merged = None
    enc_marks, dec_marks = [], []
    n_exact = 0
    for _ in range(steps):
        sync()
        t0 = time.perf_counter()
        codec.phases = []
        rbs = codec.encode(img)
        if world > 1:
            merged = gather_residual(rbs)
        torch.cuda.synchronize()
        enc_marks.append(codec.phases)
        t1 = time.perf_counter()
        codec.phases = []
        out, info = codec.decode(rbs, verify=False)
        torch.cuda.synchronize()
        dec_marks.append(codec.phases)
        codec.phases = None
        t2 = time.perf_counter()
        te += t1 - t0
        td += t2 - t1
        n_exact += int(torch.equal(out, img))  # every timed step's round trip (after its timing)
    exact = n_exact == steps
    t_idx, t_rec = vq_time()
    roof = flow_conv_roofline(codec, fl, img)
    vroof = vq_roofline(codec, img)
    enc_split, dec_split = phase_split(enc_marks, steps), phase_split(dec_marks, steps)
    if world > 1:
        t = torch.tensor([te, td, t_idx, t_rec, 0.0 if exact else 1.0], device=dev)
        all_reduce(t, dist.ReduceOp.MAX)
        te, td, t_idx, t_rec = (float(v) for v in t[:4])
        exact = float(t[4]) == 0.0
    res = None
    if rank == 0:
        bs = merged if merged is not None else rbs
        px = per * world * Hs * Ws
        res = {
            "metric": f"encode+decode Mpixels/s ({config}, bit-exact round trip)",
            "value": round(px * steps / (te + td) / 1e6, 4), "unit": "Mpx/s", "n_gpus": world,
            "batch_per_gpu": per, "image": [3, Hs, Ws], "coded_image": [3, H, W],
            "steps": steps, "warmup": warmup, "round_trip_exact_steps": f"{n_exact}/{steps}",
            "encode_ms": round(te / steps * 1e3, 2),
            "decode_ms": round(td / steps * 1e3, 2),
            "encode_mpx_s": round(px * steps / te / 1e6, 4),
            "decode_mpx_s": round(px * steps / td / 1e6, 4),
            "vq_indices_ms": round(t_idx * 1e3, 2), "vq_reconstruct_ms": round(t_rec * 1e3, 2),
            "bpp": round(3 * bs.bpd(), 4), "index_bits_share": round(
                1 - bs.flow.bits() / bs.bits(), 4),
            "round_trip_exact": exact, "scaling": "weak",
            "vq_conv": rbs.vq_conv, "roofline": roof, "vq_roofline": vroof,
            "encode_split_ms": enc_split, "decode_split_ms": dec_split,
            "split_note": ("device time between phase marks on the codec's stream, mean over "
                           "the timed steps (the flow phase includes its side-stream rANS "
                           "joins; host-side waits such as the VQ range-guard read sit in the "
                           "phase that issues them)"),
            "dtype": ("bf16 flow convs (f32 accumulate), f32 heads/VQ-VAE/CDF"
                      if fl.engine().precision == "bf16" else "f32"),
            "data": "synthetic uint8, seeded weights"}
    del codec, fl, vq, img, full
    torch.cuda.empty_cache()
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="resflow-cond-imagenet64")
    ap.add_argument("--batch", type=int, default=None, help="images per GPU")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--precision", default=None, choices=[None, "f32", "bf16"])
    a = ap.parse_args()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    res = run(a.config, a.batch, a.steps, a.warmup, a.precision)
    if res is not None:
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
