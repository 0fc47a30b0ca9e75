"""bench.py -- encode+decode throughput of the MI355X IDF + rANS lossless codec.

Workload (BASELINE.json configs[1]): configs/imagenet64.yaml, batch 256 of
synthetic 64x64x3 uint8 images per GPU, fp32 flow + HIP rANS, synthetic seeded
weights (no checkpoints exist).  One step = encode (dequant -> IDF
forward + priors -> per-(image, level) rANS streams -> compaction) followed by
decode (priors -> rANS decode -> IDF inverse -> uint8) of that batch.  With N > 1
GPUs (one process per GPU, RCCL over xGMI) each rank codes its own 256-image shard
of the global batch and the step also assembles the single-batch bitstream on
rank 0 (gather_bitstream: a header gather + point-to-point sends) and hands each
rank its shard of it back for decode (scatter_bitstream) -- the file is what is
decoded.  Inputs are resident in HBM before the timed region.  Weak scaling:
value = all ranks' pixels / max-over-ranks time.

`python bench.py --gpus N` with N > 1 and no RANK in the environment starts N
ranks itself (torch.distributed.run, before anything touches the GPU) and exits
with their status.

Prints ONE JSON line on rank 0.  Extra keys: encode/decode split, bpp, exact
round trip, the roofline of the dominant kernel (timed live with HIP events in a
separate encode pass after the timed steps), the rANS chains, the residual configs
3-5 (BASELINE configs[2..4]: encode/decode Mpx/s and exactness, one short run each)
and the CPU baseline (the oracle: torch-fp32 flow + C rANS on this host's cores).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "finalproject-losslessimagecompression_amd")
sys.path.insert(0, PKG)
# hardware queues per process: the pipelined steps use six HIP streams (the encode's and its
# rANS side stream, the decode's and its two lanes, the default), so with 4 queues some share
# one and run in order -- measured faster than 8 or 16 queues with the round-4 decode (19.17-
# 19.32 vs 18.32-18.73 Mpx/s, 5 same-box pairs over two boxes: profiles/r04/hwq/).  Set before
# anything initialises HIP.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "4")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

PEAK_F32_TFLOPS = 157.3  # MI355X_MICROARCH.md: fp32 matrix (f32-in MFMA) = vector peak
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E
PEAK_F16_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/F16 dense MFMA peak
B_PER_GPU = 256
PX_PER_IMG = 64 * 64


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=B_PER_GPU)
    ap.add_argument("--cpu-baseline-images", type=int, default=64)
    ap.add_argument("--cpu-baseline-runs", type=int, default=3)
    ap.add_argument("--cpu-baseline-images-per-proc", type=int, default=16)
    ap.add_argument("--cpu-baseline-split", default=None,
                    help="PROCSxTHREADS for the CPU-baseline pool (default: one thread per "
                         "usable CPU)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--pipeline", type=int, default=1,
                    help="1: step k's decode runs beside step k+1's encode (two HIP streams, "
                         "separate engine workspaces; every timed step still encodes and "
                         "decodes one whole batch, pipeline fill and drain inside the timed "
                         "region); 0: each step's encode and decode back to back")
    ap.add_argument("--no-residual", action="store_true",
                    help="skip the residual configs 3-5 extras")
    ap.add_argument("--launch-probe", action="store_true",
                    help="ranks report their rank / world size and exit (tests the launcher)")
    return ap.parse_args()


def launch(args) -> int:
    """N ranks of this script under torch.distributed.run (one process per GPU).  The
    parent never touches the GPU and never execs: it waits and returns the ranks' status."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1", "--master-port",
           str(port), os.path.abspath(__file__), *sys.argv[1:]]
    return subprocess.call(cmd)


# the sources whose compiled kernels a committed PMC traffic capture describes
CONV_SOURCES = ("conv3_dx3.hip", "conv3_wino.hip", "wino_common.h", "idf_codec_internal.h")


def conv_source_hash() -> str:
    """sha256 over the conv kernels' sources (CONV_SOURCES, in order): tools/pmc_bench.sh stores
    it with a capture (source_hash.txt) and pmc_traffic reports a capture's traffic only while
    the built sources are still the ones it measured."""
    import hashlib
    h = hashlib.sha256()
    for name in CONV_SOURCES:
        with open(os.path.join(REPO, "finalproject-losslessimagecompression_amd", "csrc", name),
                  "rb") as f:
            h.update(name.encode() + b"\0" + f.read())
    return h.hexdigest()


def pmc_traffic(kernels, n_last: int, extra: str = "conv3_wino_reduce_kernel"):
    """HBM bytes per launch of the DenseLayer conv from the newest committed PMC passes
    (profiles/<round>/pmc_bench/{fetch,write}.csv[.gz], written by tools/pmc_bench.sh over this
    bench), over the same launches as roofline.achieved: the process's last n_last dispatches
    whose name contains one of `kernels` (the sampled encode pass ends the run) plus the `extra`
    dispatches among them (the 8x8 split-K reduce, whose time roofline_pass also counts).
    Bytes = 2 x FETCH_SIZE (the gfx950 correction for 16-B-per-lane streaming reads,
    MI355X_MICROARCH.md "HBM") + WRITE_SIZE, KiB -> bytes.  (None, why) when no capture exists
    or the newest one was taken from other kernel sources (its source_hash.txt differs from
    conv_source_hash())."""
    import csv
    import glob
    fetch = sorted(glob.glob(os.path.join(REPO, "profiles", "*", "pmc_bench", "fetch.csv*")))
    if not fetch or n_last <= 0:
        return None, None
    d = os.path.dirname(fetch[-1])
    hp = os.path.join(d, "source_hash.txt")
    want = conv_source_hash()
    have = open(hp).read().strip() if os.path.exists(hp) else None
    if have != want:
        return None, (f"{os.path.relpath(d, REPO)}: captured from other kernel sources "
                      f"(hash {have or 'unrecorded'} != built {want[:16]}); not reported")

    def total(name):
        import gzip
        path = os.path.join(d, name)
        opener = open
        if os.path.exists(path + ".gz"):
            path, opener = path + ".gz", gzip.open
        if not os.path.exists(path):
            return None
        with opener(path, "rt", newline="") as fh:
            rows = sorted(csv.DictReader(fh), key=lambda r: int(r["Dispatch_Id"]))
        main = [r for r in rows if any(k in r["Kernel_Name"] for k in kernels)]
        if len(main) < n_last:
            return None
        d0 = int(main[-n_last]["Dispatch_Id"])
        sel = main[-n_last:] + [r for r in rows if extra and extra in r["Kernel_Name"]
                                and int(r["Dispatch_Id"]) >= d0]
        return sum(float(r["Counter_Value"]) for r in sel)
    f, w = total("fetch.csv"), total("write.csv")
    if f is None or w is None:
        return None, None
    return (2.0 * f + w) * 1024.0 / n_last, f"{os.path.relpath(d, REPO)} (sources {want[:16]})"

def rans_roofline(trace, bs, steps):
    """rANS encode / decode (prep + serial pass per launch pair), timed with HIP events on
    the launch stream over the timed steps, against the HBM roofline.  Algorithmic bytes:
    encode reads x, mean, scale (12 B/symbol) and writes the words (4 B each) plus a state
    and a word count per stream (16 B); decode reads mean, scale (8 B/symbol), the words and
    the states and writes x (4 B/symbol) plus a final state per stream.  The serial chains
    (one rANS state per stream, rans.pyx's reference order) make both latency-bound:
    ns_per_symbol is the chain's time per symbol (launch time / symbols per stream)."""
    out = {}
    words = bs.total_words()
    for kind in ("encode", "decode"):
        recs = [r for r in trace if r[0] == kind]
        if not recs:
            continue
        ms = sum(a.elapsed_time(b) for _, _, _, a, b in recs)
        nsym = sum(r[1] for r in recs)
        chain = sum(r[1] / max(r[2], 1) for r in recs)
        nstr = sum(r[2] for r in recs)
        byts = 12.0 * nsym + 4.0 * words * steps + 16.0 * nstr
        gbs = byts / (ms * 1e-3) / 1e9
        # launch_ms: summed launch durations (decode lanes overlap, so it can exceed the
        # wall time the decode adds to a step)
        out[kind] = {"launch_ms_per_step": round(ms / steps, 4),
                     "msym_s": round(nsym / (ms * 1e-3) / 1e6, 2),
                     "ns_per_symbol": round(ms * 1e6 / chain, 1),
                     "bound": "latency (serial state chain per stream)",
                     "achieved": round(gbs, 2), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": round(gbs / PEAK_HBM_GBS, 5)}
    return out


def conv_kernel_name(eng):
    from idfcodec import engine
    if eng.wino and eng.conv_mode == "dx3":
        return ("conv3_dx3_kernel<3, ...> at every level (16 x 16 tiles of the 32x32 and 16x16 "
                "images; the 8x8 images packed 2 x 2 a tile, split K in 4 chunks summed by the "
                "tile's last block): DenseLayer 3x3 conv with the 1x1 folded in, direct form, "
                "split-f16 products over the block's split feature copy (x = xh + xl written once "
                "by the producer, halos by LDS-DMA; xh.wh + xl.wh + xh.wl on "
                "v_mfma_f32_16x16x32_f16, f32 accumulation), the DenseBlock head's share added in "
                "the epilogue; the 16x16 and 8x8 levels' DenseBlocks each as ONE launch "
                "(conv3_dx3_block_kernel<3, ...>: a workgroup per tile looping over the 12 "
                "layers, the 8x8 split-K chunks summed in the block, the head's sums in "
                "registers) -- bit for bit the per-layer launches")
    if eng.wino and eng.conv_mode == "x3":
        return ("conv3_wino_kernel<3, 448, true, false> (+conv3_wino_reduce_kernel at 8x8): "
                "DenseLayer 3x3 conv with the 1x1 folded in, Winograd F(2x2,3x3), split-f16 "
                "products (f32 operands as f16 hi/lo pairs, 3 x v_mfma_f32_16x16x16_f16, f32 "
                "accumulation)")
    if eng.wino:
        return ("conv3_wino_kernel<3> (+conv3_wino_reduce_kernel at 8x8): DenseLayer 3x3 conv "
                "with the 1x1 folded in, Winograd F(2x2,3x3), f32 MFMA")
    if eng.fold and engine.HALO:
        return ("conv3_halo_kernel<3> (+conv3_reduce_kernel at 8x8): DenseLayer 3x3 conv with "
                "the 1x1 folded in, LDS halo tiles, f32 MFMA")
    if eng.fold:
        return "gemm_f32_kernel<BM,48,4,1,MODE_CONV3,EPI_ACT_FOLD> (folded 3x3 conv, implicit GEMM)"
    return "gemm_f32_kernel<BM,48,4,1,MODE_CONV3,EPI_ACT> (3x3 conv, implicit GEMM)"


def wino_exec_ratio(eng):
    """MFMA FLOPs executed per algorithmic (direct-conv) FLOP of the 3x3 conv, FLOP-weighted over
    the levels.  Winograd F(2x2,3x3) issues 16 products per 2x2 outputs instead of 36 (x3: as
    three K=16 f16 MFMA passes); dx3 issues 14 K=32 MFMAs per 16 channels x 16 pixels x 16
    outputs where the three split products need 13.5 (the ninth tap's lo product pairs with
    zeros); both over 16-padded outputs (43 real growth channels -> 48).  1.0 for the direct
    f32 kernels."""
    if not eng.wino:
        return 1.0
    pad = 48.0 / 43.0
    wino = 16.0 / 36.0 * pad
    if eng.conv_mode == "f32":
        return wino
    direct = 3.0 * 14.0 / 13.5 * pad
    num = den = 0.0
    for l, L in enumerate(eng.levels):
        for b in eng.couple[l] + [eng.prior[l]]:
            g, nd = b.geom, eng.dx3_layers(l, b.geom)
            for i, gr in enumerate(g.growth):  # the layer's 3x3 FLOPs per pixel ~ c_in x g
                f = L.h * L.w * (g.a + sum(g.growth[:i])) * gr
                num += f * (direct if i < nd else 3.0 * wino)
                den += f
    return num / den


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_oracle(model_cfg):
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import flow_oracle as FO
    from idfcodec import synthetic
    model = synthetic.build_model(model_cfg)
    sd = {k: v.detach() for k, v in model.state_dict().items()}
    return FO.FlowOracle(model_cfg, sd)


def _cpu_chunk(o, img):
    """encode then decode one batch with the oracle: (t_enc, t_dec, exact)."""
    import numpy as np
    import flow_oracle as FO
    import rans_oracle as RO
    n_img = img.shape[0]
    t0 = time.perf_counter()
    x = FO.dequant(img)
    lat, me, ls = o.forward(x)
    flat = lambda ts: np.concatenate([t.reshape(-1).numpy() for t in ts])  # noqa: E731
    L = flat(lat)
    M = flat(me)
    S = flat([torch.exp(t) for t in ls])
    sizes = [t[0].numel() for t in lat]
    off = [0]
    for n in sizes:
        off += [off[-1] + n * (b + 1) for b in range(n_img)]
    off = np.asarray(off, np.int64)
    fs, words, nw, st = RO.encode_streams(off, L, M, S)
    t_enc = time.perf_counter() - t0

    def dec(l, m, s):
        k0 = l * n_img
        sl = slice(k0, k0 + n_img)
        o_l = off[k0:k0 + n_img + 1] - off[k0]
        m_np = m.reshape(-1).numpy()
        s_np = torch.exp(s).reshape(-1).numpy()
        w_off = off[k0:k0 + n_img]
        fs2, out, st2 = RO.decode_streams(o_l, w_off, nw[sl], words, m_np, s_np, fs[sl])
        return torch.from_numpy(out).view(m.shape)

    t1 = time.perf_counter()
    xd, _ = o.decode_levels(n_img, dec)
    t_dec = time.perf_counter() - t1
    return t_enc, t_dec, bool(torch.equal(xd, x))


def bpp_vs_oracle(model_cfg, img_u8, bs, B, n=16):
    """BASELINE's "bpp vs reference": the first n images of this rank's batch coded by the
    oracle (the torch-fp32 flow pinned bit for bit to the reference's modules + the C rANS
    pinned to the reference's rans.cpp) and by the device, in the reference's accounting
    (trainer.py:326-327: 64 bits per stream's final state + 32 per word, over the sub-pixels).
    The device side counts the same images' streams of the timed steps' last bitstream (level-
    major, image-minor: stream (l, b) = l * B + b).  Any difference comes from Round flips of
    the fp32 flows (tests/test_gpu_flow.py bounds them)."""
    import numpy as np
    o = _cpu_oracle(model_cfg)  # (puts oracle/ on the path)
    import flow_oracle as FO
    import rans_oracle as RO
    x = FO.dequant(img_u8[:n].cpu())
    lat, me, ls = o.forward(x)
    flat = lambda ts: np.concatenate([t.reshape(-1).numpy() for t in ts])  # noqa: E731
    sizes = [t[0].numel() for t in lat]
    off = [0]
    for m in sizes:
        off += [off[-1] + m * (b + 1) for b in range(n)]
    _, _, nw, st = RO.encode_streams(np.asarray(off, np.int64), flat(lat), flat(me),
                                     flat([torch.exp(t) for t in ls]))
    nsub = n * 3 * PX_PER_IMG
    bits_o = 64 * len(nw) + 32 * int(np.asarray(nw, np.int64).sum())
    hn = bs.nwords_host()
    k = [lv * B + b for lv in range(len(sizes)) for b in range(n)]
    bits_g = 64 * len(k) + 32 * int(hn[k].sum())
    return {"images": n, "bpp_oracle": round(3.0 * bits_o / nsub, 5),
            "bpp_device": round(3.0 * bits_g / nsub, 5),
            "bpp_difference": round(3.0 * (bits_g - bits_o) / nsub, 6),
            "bits_oracle": bits_o, "bits_device": bits_g,
            "oracle_status_ok": bool((np.asarray(st) == 0).all()),
            "oracle": ("oracle/flow_oracle.py (torch fp32, pinned to the reference modules) + "
                       "oracle/rans_oracle.c (pinned to the reference's rans.cpp), on the "
                       "bench's own first images")}


def _cpu_run(o, img, chunk):
    te = td = 0.0
    ok = True
    for c0 in range(0, img.shape[0], chunk):
        a, b, e = _cpu_chunk(o, img[c0:c0 + chunk])
        te, td, ok = te + a, td + b, ok and e
    return te, td, ok


def _cpu_worker(conn, cpus, threads, n_img, chunk, seed):
    """One process of the CPU-baseline pool: pinned to `cpus`, `threads` torch/OpenMP threads,
    its own n_img synthetic images.  Never touches the GPU.  Protocol: sends "ready" after
    the warm-up, then for every "run" message replies (t_enc, t_dec, exact, cpu_s, wall_s)."""
    os.environ.update(OMP_NUM_THREADS=str(threads), HIP_VISIBLE_DEVICES="",
                      CUDA_VISIBLE_DEVICES="", ROCR_VISIBLE_DEVICES="")
    try:
        os.sched_setaffinity(0, cpus)
    except (AttributeError, OSError):
        pass
    torch.set_num_threads(threads)
    from idfcodec import configs, synthetic
    o = _cpu_oracle(configs.get("imagenet64"))
    img = synthetic.images(n_img, seed=seed)
    _cpu_chunk(o, img[:1])  # warm-up (oneDNN primitives, the C coder's library)
    conn.send("ready")
    while True:
        msg = conn.recv()
        if msg != "run":
            break
        c0, w0 = time.process_time(), time.perf_counter()
        te, td, ok = _cpu_run(o, img, chunk)
        conn.send((te, td, ok, time.process_time() - c0, time.perf_counter() - w0))
    conn.close()


def _cgroup_cpus():
    """The cgroup v2 CPU quota in CPUs (cpu.max), or None when unlimited / unreadable."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        return None


def usable_cpus():
    """(affine CPUs, cgroup quota in CPUs or None, CPUs of time the process can use)."""
    affinity = sorted(os.sched_getaffinity(0))
    quota = _cgroup_cpus()
    usable = len(affinity)
    if quota is not None:
        usable = max(1, min(usable, int(quota + 1e-6)))
    return affinity, quota, usable


class CpuPool:
    """The CPU baseline's worker pool, started at the top of main() before anything touches
    the GPU (the workers are spawned processes: no process is started once HIP is live).
    It covers every CPU the process may run on: sched_getaffinity, capped by the cgroup's CPU
    quota when there is one (a GPU box grants 16 CPUs of time over 256 affine CPUs --
    profiles/r03/host_cpu_probe.txt: 64 busy processes get 16.4 CPUs), split into processes x
    threads, each process on its own CPUs and its own images.  The timed legs run after the
    GPU timing (the workers only wait on a pipe meanwhile)."""

    def __init__(self, n_img_per_proc, chunk=16, split=None):
        import multiprocessing as mp
        self.affinity, self.quota, usable = usable_cpus()
        self.usable = usable
        if split:
            procs, threads = (int(v) for v in split.lower().split("x"))
        else:
            threads = 1  # one thread per process: no OpenMP barriers, best CPU throughput
            procs = usable
        self.procs, self.threads = procs, threads
        self.n_img, self.chunk = n_img_per_proc, min(chunk, n_img_per_proc)
        ctx = mp.get_context("spawn")
        self.conns, self.workers = [], []
        for i in range(procs):
            cpus = self.affinity[(i * threads) % len(self.affinity):][:threads] or self.affinity
            a, b = ctx.Pipe()
            w = ctx.Process(target=_cpu_worker, args=(b, cpus, threads, n_img_per_proc,
                                                      self.chunk, 100 + i), daemon=True)
            w.start()
            self.conns.append(a)
            self.workers.append(w)
        self.ready = False

    def wait_ready(self, timeout=900):
        for c in self.conns:
            if not c.poll(timeout) or c.recv() != "ready":
                raise RuntimeError("CPU baseline worker failed to start")
        self.ready = True

    def run(self):
        """One timed pass: every worker codes its images; returns (wall, per-worker results)."""
        t0 = time.perf_counter()
        for c in self.conns:
            c.send("run")
        res = [c.recv() for c in self.conns]
        return time.perf_counter() - t0, res

    def close(self):
        for c in self.conns:
            try:
                c.send("stop")
            except OSError:
                pass
        for w in self.workers:
            w.join(timeout=30)
            if w.is_alive():
                w.terminate()


def cpu_baseline_pool(pool, runs):
    """The oracle on all of the host's usable CPUs: torch-fp32 flow (oracle/flow_oracle.py) +
    C rANS (oracle/rans_oracle.c), encode then decode, every pool process on its own images in
    batches of pool.chunk; the median of `runs` timed passes (after each worker's warm-up).
    cores = CPUs the pool ran on; effective_cpus = the CPU time it got / wall time."""
    import statistics
    if not pool.ready:
        pool.wait_ready()
    passes = [pool.run() for _ in range(max(1, runs))]
    walls = [w for w, _ in passes]
    med = statistics.median(walls)
    wall, res = passes[walls.index(sorted(walls)[len(walls) // 2])]
    px = pool.procs * pool.n_img * PX_PER_IMG
    exact = all(r[2] for _, rs in passes for r in rs)
    cpu_s = sum(r[3] for r in res)
    # the encode / decode split of the median pass: its wall time apportioned by the workers'
    # summed encode and decode times (every worker encodes then decodes each of its batches,
    # as the reference times rans_en_time / rans_de_time separately, trainer.py:310-320)
    te, td = sum(r[0] for r in res), sum(r[1] for r in res)
    enc_wall = wall * te / max(te + td, 1e-12)
    dec_wall = wall * td / max(te + td, 1e-12)
    return {"value": round(px / med / 1e6, 5), "unit": "Mpx/s",
            "encode_mpx_s": round(px / enc_wall / 1e6, 5),
            "decode_mpx_s": round(px / dec_wall / 1e6, 5),
            "encode_decode_split": ("median pass wall time x (summed per-worker encode | decode "
                                    "time) / (summed encode + decode time)"),
            "cores": pool.procs * pool.threads, "kind": "port",
            "split": f"{pool.procs} processes x {pool.threads} threads",
            "affinity_cpus": len(pool.affinity), "cgroup_cpu_quota": pool.quota,
            "effective_cpus": round(cpu_s / wall, 2),
            "cpu_model": _cpu_model(), "runs": len(passes),
            "runs_mpx_s": [round(px / w / 1e6, 5) for w in walls],
            "sample": (f"{pool.procs} x {pool.n_img} synthetic 64x64 images (one slice per "
                       f"process, batches of {pool.chunk}), imagenet64 model, encode+decode "
                       f"(torch-fp32 flow oracle + C rANS oracle), wall time of the whole "
                       f"pool, median of {len(passes)} passes; median pass "
                       f"{wall:.2f}s, round trips exact={exact}")}


def cpu_baseline(model_cfg, n_img, runs, chunk=16):
    """The oracle in THIS process with its torch threads (16 on a GPU box: OMP_NUM_THREADS):
    the round-2 figure, kept as the single-process comparison next to the pool's.  Median of
    `runs` timed runs after one warm-up."""
    import statistics
    o = _cpu_oracle(model_cfg)
    from idfcodec import synthetic
    img = synthetic.images(n_img, seed=7)
    threads = torch.get_num_threads()
    _cpu_chunk(o, img[:1])
    res = [_cpu_run(o, img, chunk) for _ in range(max(1, runs))]
    tot = [a + b for a, b, _ in res]
    med = statistics.median(tot)
    px = n_img * PX_PER_IMG
    return {"value": round(px / med / 1e6, 5), "threads": threads,
            "runs_mpx_s": [round(px / t / 1e6, 5) for t in tot],
            "sample": f"{n_img} images in batches of {chunk}, one process, {threads} threads"}


def conv_algorithmic_bytes(eng, B):
    """(launches, algorithmic HBM bytes) of one encode's DenseLayer convs -- the launches
    roofline_pass times: per layer the c input channels read and g outputs written, fp32, per
    pixel, plus its weights (9 direct taps or 16 Winograd positions x c x g f16 hi/lo pairs,
    4 B); a fused DenseBlock (engine.fused_block: every layer in one launch) is one launch
    carrying its layers' bytes."""
    n = byt = 0
    for l, L in enumerate(eng.levels):
        P = B * L.h * L.w
        # IDFlows' top prior sees zeros: computed once per model, not per encode
        cached = L.prior_x_zero and not eng.conditional
        for blk in list(eng.couple[l]) + ([] if cached else [eng.prior[l]]):
            geom = blk.geom
            c = geom.a
            nd = eng.dx3_layers(l, geom)
            fused = eng.fused_block(l, blk)
            n += 1 if fused else 0
            for i, g in enumerate(geom.growth):
                # weights per (c, g): 16 Winograd positions or 9 direct taps, f16 (hi, lo) pairs
                npos = 9 if i < nd else 16
                n += 0 if fused else 1
                byt += 4 * P * (c + g) + npos * c * g * 4
                c += g
    return n, byt


def roofline_pass(codec, eng, timer, img):
    """The dominant kernel timed live: one encode of the batch after the timed steps, with the
    side-stream rANS encode and the encode lanes off (every conv launch has the chip to
    itself) and HIP events
    around every DenseLayer conv launch of every coupling and prior (idf_dense_block_f32_timed
    brackets each launch on the stream it is issued on).  Returns (achieved TF/s,
    average launch ms, launches, algorithmic FLOPs per launch)."""
    import ctypes
    from idfcodec import _lib
    for b in eng._blocks:
        b.timer = timer
    prev, prev_lanes = codec.overlap_encode, codec.enc_lanes
    codec.overlap_encode = False
    codec.enc_lanes = 1  # one full-batch launch per conv, nothing beside it
    _lib.lib().idf_timer_reset(timer)
    try:
        codec.encode(img)
        torch.cuda.synchronize()
    finally:
        codec.overlap_encode, codec.enc_lanes = prev, prev_lanes
        for b in eng._blocks:
            b.timer = None
    tot, cnt, fl = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double()
    _lib.check(_lib.lib().idf_timer_summary(timer, _lib.TAG_CONV3X3, ctypes.byref(tot),
                                            ctypes.byref(cnt), ctypes.byref(fl)), "timer")
    n = max(cnt.value, 1)
    tflops = fl.value / (tot.value * 1e-3) / 1e12 if tot.value > 0 else 0.0
    return tflops, tot.value / n, cnt.value, fl.value / n


def residual_extras(args):
    """BASELINE configs[2..4] (the residual VQ-VAE + flow codecs): 10 timed steps after 2
    warm-up each on this rank's GPU (sharded per rank when N > 1, bitstreams gathered to rank 0
    in the timed encode), with the flow convs' and the VQ-VAE kernels' rooflines and the
    encode / decode phase split, reported beside the headline."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import bench_residual
    out = {}
    for name in ("resflow-cond-imagenet64", "resflows_smallpatch_split", "resflow-patches-vqvae"):
        try:
            r = bench_residual.run(name, steps=10, warmup=2)
        except Exception as e:  # reported, never hides the headline
            r = {"error": repr(e)}
            if dist.is_initialized():
                raise
        if r is not None:
            out[name] = {k: r[k] for k in ("value", "encode_mpx_s", "decode_mpx_s", "encode_ms",
                                           "decode_ms", "batch_per_gpu", "image", "bpp",
                                           "round_trip_exact", "dtype", "n_gpus",
                                           "vq_indices_ms", "vq_reconstruct_ms", "vq_conv",
                                           "roofline", "vq_roofline", "encode_split_ms",
                                           "decode_split_ms", "steps", "warmup",
                                           "round_trip_exact_steps") if k in r} \
                if "error" not in r else r
    return out


def main():
    args = parse()
    if args.gpus > 1 and "RANK" not in os.environ:
        return launch(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.launch_probe:  # no GPU work: the launcher test
        print(json.dumps({"rank": rank, "world": world, "local_rank": local}), flush=True)
        return 0
    if world != args.gpus:
        raise SystemExit(f"bench.py --gpus {args.gpus} but WORLD_SIZE={world}")
    # the CPU baseline's pool starts here, before anything touches the GPU; its timed passes
    # run after the GPU timing
    pool = None
    if not args.no_cpu_baseline and world == 1:
        pool = CpuPool(args.cpu_baseline_images_per_proc, split=args.cpu_baseline_split)
    # IDF_DIST_BACKEND=gloo IDF_SHARE_GPU=1: every rank on cuda:0, collectives staged through
    # host memory -- a one-GPU rehearsal of the N-rank path (the real run is RCCL, one GPU each)
    backend = os.environ.get("IDF_DIST_BACKEND", "nccl")
    if os.environ.get("IDF_SHARE_GPU") == "1":
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        assert dist.get_world_size() == args.gpus, "process group size != --gpus"

    from idfcodec import _lib, configs, synthetic
    from idfcodec.dist import (all_reduce, broadcast_state, gather_bitstream, scatter_bitstream,
                               shard_range)

    cfg = configs.get("imagenet64")
    model = synthetic.build_model(cfg).to(dev)
    if world > 1:
        broadcast_state(model)  # replicated weights: one broadcast from rank 0
    codec = model.codec()
    eng = model.engine()
    B = args.batch
    lo, hi = shard_range(B * world, rank, world)
    img = synthetic.images(B * world, seed=2)[lo:hi].to(dev)  # this rank's shard
    # every timed step's round trip: a device-side count of the steps whose decoded batch equals
    # the input, enqueued on the decode's stream right after it (no host sync in the timed
    # region; read once after it) -- the reference checks every batch, trainer.py:320
    exact_steps = []  # one 0-d device bool per decoded batch

    def count_exact(out):
        exact_steps.append(torch.all(out == img))

    def step():
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e2 = torch.cuda.Event(enable_timing=True)
        e0.record()
        bs = codec.encode(img)
        full = None
        if world > 1:
            full = gather_bitstream(bs, dst=0)  # the single-batch file on rank 0
            bs, _ = scatter_bitstream(full, src=0, device=dev)  # decode what the file holds
        e1.record()
        out, info = codec.decode(bs, verify=False)
        e2.record()
        count_exact(out)
        return bs, full, out, (e0, e1, e2)

    # Pipelined steps: the encode of batch k+1 (stream E, engine workspace ENC_SLOT) runs
    # beside the decode of batch k (stream D, the decode lanes' workspaces): the decode's
    # serial rANS chains, which its own lanes cannot hide, overlap the next encode's convs.
    # Each batch's decode waits on an event recorded after its encode (and, N > 1, after its
    # gather -> scatter); the bitstreams stay referenced until the loop ends.
    enc_stream = dec_stream = None
    if args.pipeline:
        enc_stream, dec_stream = _lib.new_stream(dev), _lib.new_stream(dev)

    def encode_part():
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(enc_stream):
            a.record()
            bs = codec.encode(img, slot=codec.ENC_SLOT)
            full = None
            if world > 1:
                full = gather_bitstream(bs, dst=0)
                bs, _ = scatter_bitstream(full, src=0, device=dev)
            b.record()
        return bs, full, (a, b)

    def decode_part(bs, after):
        a = torch.cuda.Event(enable_timing=True)
        b = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(dec_stream):
            dec_stream.wait_event(after)
            a.record()
            out, _ = codec.decode(bs, verify=False)
            b.record()
            count_exact(out)
        return out, (a, b)

    def run_steps(n):
        res = [step() for _ in range(n)]
        return res[-1][0], res[-1][1], res[-1][2], [((e0, e1), (e1, e2)) for *_, (e0, e1, e2) in res]

    def run_steps_pipelined(n):
        keep, evs = [], []
        bs, full, ee = encode_part()
        keep.append((bs, full, ee))
        out = None
        for k in range(n):
            prev_bs, prev_full, prev_ee = keep[-1]
            out, de = decode_part(prev_bs, prev_ee[1])  # batch k's decode ...
            evs.append((prev_ee, de))
            if k + 1 < n:
                keep.append(encode_part())  # ... beside batch k+1's encode
        last_bs, last_full, _ = keep[-1]
        return last_bs, last_full, out, evs

    if args.pipeline:
        run_steps = run_steps_pipelined  # noqa: F811

    if args.warmup:
        run_steps(args.warmup)
    if pool is not None:
        pool.wait_ready()  # the workers' start-up never overlaps the timed steps
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    codec.coder.trace = []  # HIP events around the rANS launches of the timed steps
    exact_steps.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bs, full, out, evs = run_steps(args.steps)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    step_ok = torch.stack(exact_steps).to(torch.int64)
    if world > 1:
        all_reduce(step_ok, dist.ReduceOp.MIN)  # a step is exact when every rank's shard is
    n_exact, n_checked = int(step_ok.sum().item()), int(step_ok.numel())
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        all_reduce(t, dist.ReduceOp.MAX)
    elapsed = float(t.item())
    rans = rans_roofline(codec.coder.trace, bs, args.steps)
    codec.coder.trace = None
    # per batch: the encode's and the decode's own stream time (pipelined: while overlapping)
    enc_ms = sum(e[0].elapsed_time(e[1]) for e, _ in evs) / len(evs)
    dec_ms = sum(d[0].elapsed_time(d[1]) for _, d in evs) / len(evs)
    serial = None
    if args.pipeline:
        # the same steps back to back (untimed for `value`): what one batch costs alone
        pe = []
        for _ in range(4):
            pe.append(step())
        torch.cuda.synchronize()
        se = sum(a.elapsed_time(b) for *_, (a, b, c) in pe) / len(pe)
        sd = sum(b.elapsed_time(c) for *_, (a, b, c) in pe) / len(pe)
        serial = {"encode_ms": round(se, 3), "decode_ms": round(sd, 3),
                  "ms_per_step": round(se + sd, 3),
                  "mpx_s": round(world * B * PX_PER_IMG / (se + sd) / 1e3, 4)}

    # exactness of the last timed step on every rank (and, N > 1, of the whole gathered
    # single-batch bitstream decoded on rank 0 alone, below)
    ok = torch.tensor([1 if torch.equal(out, img) else 0], dtype=torch.int64, device=dev)
    if world > 1:
        all_reduce(ok, dist.ReduceOp.MIN)
    exact = bool(ok.item())
    full_exact = None
    if world > 1 and rank == 0:
        whole = synthetic.images(B * world, seed=2).to(dev)
        img_full, info = codec.decode(full)
        full_exact = bool(info["ok"]) and bool(torch.equal(img_full, whole))
        del whole, img_full
    bits = full.bits() if full is not None else bs.bits()
    bpp = 3.0 * bits / (3 * B * world * PX_PER_IMG)
    bpp_ref = None
    if rank == 0 and not args.no_cpu_baseline:
        try:
            bpp_ref = bpp_vs_oracle(cfg, img, bs, B)
        except Exception as e:  # reported, never hides the headline
            bpp_ref = {"error": repr(e)}

    timer = _lib.lib().idf_timer_create(8192)
    c3_tflops, c3_avg_ms, c3_n, c3_flops = roofline_pass(codec, eng, timer, img)
    _lib.lib().idf_timer_destroy(timer)

    flops = eng.flops_per_image()["total"]
    # both range-check variants of the kernels: roofline_pass times every DenseLayer conv launch
    knames = {"dx3": ("conv3_dx3_kernel<3,", "conv3_dx3_block_kernel<3,",
                      "conv3_wino_kernel<3, 448, true,"),
              "x3": ("conv3_wino_kernel<3, 448, true,",),
              "f32": ("conv3_wino_kernel<3, 448, false",)}[eng.conv_mode] if eng.wino else ()
    traffic, traffic_src = pmc_traffic(knames, c3_n) if eng.wino else (None, None)
    n_algo, b_algo = conv_algorithmic_bytes(eng, B)
    algo_bytes = b_algo / n_algo if n_algo == c3_n and n_algo else None
    # the split-f16 kernels' products run on f16 MFMA: price them against the f16 dense peak
    peak = PEAK_F16_TFLOPS if (eng.wino and eng.conv_mode in ("x3", "dx3")) else PEAK_F32_TFLOPS
    flops_exec = eng.flops_per_image(fold=eng.fold)["total"]
    fold, conv_mode, kdesc, exec_ratio = eng.fold, eng.conv_mode, conv_kernel_name(eng), \
        wino_exec_ratio(eng)
    step_ms = elapsed / args.steps * 1e3
    px_total = world * B * PX_PER_IMG * args.steps
    value = px_total / elapsed / 1e6

    residual = None
    if not args.no_residual:
        del codec, eng, model, img, out, bs, full
        torch.cuda.empty_cache()
        residual = residual_extras(args)

    result = None
    if rank == 0:
        cpu = None
        if pool is not None:
            try:
                cpu = cpu_baseline_pool(pool, args.cpu_baseline_runs)
            except Exception as e:  # the baseline is reported, never the product
                cpu = {"value": None, "error": repr(e)}
            finally:
                pool.close()
            try:
                cpu["single_process"] = cpu_baseline(cfg, args.cpu_baseline_images,
                                                     args.cpu_baseline_runs)
            except Exception as e:
                cpu["single_process"] = {"value": None, "error": repr(e)}
            # north_star's target is stated on the ENCODE rate (>= 100x the reference CPU
            # encode Mpx/s at 1 GPU): the GPU encode back to back (one batch alone on the
            # chip) and inside the pipelined steps, over the pool's encode rate
            ce = cpu.get("encode_mpx_s") if isinstance(cpu, dict) else None
            if ce:
                gpu_enc = {"pipelined": B * PX_PER_IMG / enc_ms / 1e3}
                if serial:
                    gpu_enc["back_to_back"] = B * PX_PER_IMG / serial["encode_ms"] / 1e3
                cpu["gpu_over_cpu_encode"] = {k: round(v / ce, 1) for k, v in gpu_enc.items()}
                cpu["gpu_over_cpu"] = round(value / cpu["value"], 1) if cpu.get("value") else None
        result = {
            "metric": "encode+decode Mpixels/s (imagenet64, bit-exact round trip)",
            "value": round(value, 4),
            "unit": "Mpx/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(step_ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic uint8 images (seeded), synthetic seeded weights",
            "config": {"workload": "configs/imagenet64.yaml, batch 256 x 64x64x3 uint8 per GPU, "
                                   "fp32 flow + HIP rANS (BASELINE configs[1])",
                       "global_batch": world * B, "parallelism": f"dp{world} (batch shards)",
                       "streams_per_gpu": 3 * B,
                       "multi_gpu_step": ("encode shard -> gather_bitstream to rank 0 -> "
                                          "scatter_bitstream -> decode shard"
                                          if world > 1 else "encode -> decode")},
            "encode_mpx_s": round(B * PX_PER_IMG / enc_ms / 1e3, 4),
            "decode_mpx_s": round(B * PX_PER_IMG / dec_ms / 1e3, 4),
            "encode_ms": round(enc_ms, 3),
            "decode_ms": round(dec_ms, 3),
            "pipelined": bool(args.pipeline),
            "step_overlap": ("step k's decode runs beside step k+1's encode on a second HIP "
                             "stream (encode_ms / decode_ms: each part's own stream time while "
                             "overlapping); every timed step encodes and decodes one whole "
                             "batch, pipeline fill and drain inside the timed region"
                             if args.pipeline else None),
            "serial": serial,
            "bpp": round(bpp, 4),
            "bits_per_subpixel": round(bpp / 3, 4),
            "bpp_vs_reference": bpp_ref,
            "round_trip_exact": exact and n_exact == n_checked,
            "round_trip_exact_steps": f"{n_exact}/{n_checked}",
            "round_trip_check": ("every timed step's decoded batch compared with its input on "
                                 "the device (torch.all(out == img), enqueued after the decode; "
                                 "N > 1: every rank's shard), read after the timed region"),
            "gathered_bitstream_exact": full_exact,
            "flow_tflops_per_direction": round(B * flops / 1e12, 4),
            "flow_tflops_executed_per_direction": round(B * flops_exec / 1e12, 4),
            "fold_1x1_into_3x3": fold,
            "roofline": {
                "kernel": kdesc,
                "flops_per_launch": "2*P*9*c*g (P = B*h*w pixels, c/g unpadded in/out "
                                    "channels of the layer; a fused DenseBlock launch sums "
                                    "its layers)",
                "algorithmic_gflop_per_launch": round(c3_flops / 1e9, 3),
                "sampled": ("every DenseLayer conv launch (8 couplings + prior, every level) of "
                            "one encode after the timed steps, side-stream rANS encode off"),
                "launches": c3_n,
                "bound": "mfma",
                "achieved": round(c3_tflops, 3),
                "peak": peak,
                "unit": "TFLOP/s",
                "frac": round(c3_tflops / peak, 4),
                "conv_mode": conv_mode,
                "traffic": traffic,
                "traffic_unit": "B/launch (HBM, PMC)",
                "traffic_source": traffic_src,
                "algorithmic_bytes_per_launch": algo_bytes,
                "traffic_over_algorithmic": (round(traffic / algo_bytes, 3)
                                             if traffic and algo_bytes else None),
                "avg_launch_ms": round(c3_avg_ms, 5),
                "mfma_executed_tflops": round(c3_tflops * exec_ratio, 3),
                "mfma_executed_frac": round(c3_tflops * exec_ratio / peak, 4),
            },
            "rans": rans,
            "residual_configs": residual,
            "cpu_baseline": cpu,
        }
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
