"""Throughput of the residual configs' codec (BASELINE configs[2..4]) on one GPU.

Default: resflow-cond-imagenet64 (configs[2]), batch 1024 synthetic 64x64x3 uint8, seeded
weights (the configs' checkpoints are absent).  One step = ResidualCodec.encode then
decode of the batch, inputs resident in HBM.  Prints one JSON line: Mpx/s (encode+decode),
the encode / decode split, the VQ-VAE share of each, bits per pixel (flow streams + index
code) and the exactness of the round trip.  The flow's DenseLayer convs run in the config's
precision (bf16 MFMA for resflow-cond-imagenet64, as BASELINE configs[2] names; --precision
overrides).

  python tools/bench_residual.py [--config NAME] [--batch B] [--steps K] [--warmup W]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="resflow-cond-imagenet64")
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--precision", default=None, choices=[None, "f32", "bf16"])
    a = ap.parse_args()
    from idfcodec import synthetic
    codec, fl, vq, (H, W) = synthetic.build_residual(a.config, precision=a.precision)
    img = synthetic.images(a.batch, H=H, W=W, seed=2).cuda()

    def vq_time(B):
        data = codec._dequant(img[:B])
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        idx = vq.indices(data)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        vq.reconstruct(idx)
        torch.cuda.synchronize()
        return t1 - t0, time.perf_counter() - t1

    for _ in range(a.warmup):
        out, info = codec.decode(codec.encode(img))
    torch.cuda.synchronize()
    te = td = 0.0
    for _ in range(a.steps):
        t0 = time.perf_counter()
        rbs = codec.encode(img)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        out, info = codec.decode(rbs, verify=False)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        te += t1 - t0
        td += t2 - t1
    exact = bool(torch.equal(out, img))
    t_idx, t_rec = vq_time(a.batch)
    px = a.batch * H * W
    print(json.dumps({
        "metric": f"encode+decode Mpixels/s ({a.config}, bit-exact round trip)",
        "value": round(px * a.steps / (te + td) / 1e6, 4), "unit": "Mpx/s", "n_gpus": 1,
        "batch": a.batch, "steps": a.steps, "encode_ms": round(te / a.steps * 1e3, 2),
        "decode_ms": round(td / a.steps * 1e3, 2),
        "vq_indices_ms": round(t_idx * 1e3, 2), "vq_reconstruct_ms": round(t_rec * 1e3, 2),
        "bpp": round(3 * rbs.bpd(), 4), "index_bits_share": round(
            1 - rbs.flow.bits() / rbs.bits(), 4),
        "round_trip_exact": exact,
        "dtype": ("bf16 flow convs (f32 accumulate), f32 heads/VQ-VAE/CDF"
                  if fl.engine().precision == "bf16" else "f32"),
        "data": "synthetic uint8, seeded weights"}),
        flush=True)


if __name__ == "__main__":
    main()
