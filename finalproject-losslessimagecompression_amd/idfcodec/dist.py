"""Batch sharding across ranks, the bitstream gather/scatter and the weight broadcast
(the reference itself is single-device, trainer.py:204,262).

Images are independent, so each rank (one process per GPU) codes a contiguous slice
of the batch with no data-path collective.  The exchanges are:

  * broadcast_state: the model's weights, once, from rank 0 (one flat buffer per dtype,
    241 MB fp32 for imagenet64 -- one large transfer instead of 1 404 small ones);
  * gather_streams (encode side): every shard's per-stream (final state, word count) and
    its word buffer go to the destination rank only -- a gather of a fixed 2-int64
    header, then point-to-point sends of the exact byte counts (grouped
    isend/irecv = ncclSend/ncclRecv over xGMI under backend "nccl"), so rank 0 receives
    the payload once instead of every rank receiving world x the payload;
  * scatter_streams (decode side): the mirror -- the source rank cuts the single-batch
    bitstream into each rank's image shard (level-major, local-image-minor, the order the
    rank's decoder expects) and sends each rank its streams.

Stream order: a B-image Bitstream holds stream (l, b) at index l*B + b.  A rank's shard of
images [lo, hi) holds (l, b - lo) at l*(hi-lo) + (b-lo).  interleave_levels maps the
rank-order concatenation of shards to the single-batch order; shard_streams the reverse.
The reorders run as one vectorised segment gather on whatever device holds the words.
With backend "nccl" every tensor must live on the rank's GPU; the CPU tests use gloo.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous slice [lo, hi) of n items for `rank` (the first n % world ranks get one more)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


# ------------------------------------------------------------------ stream reorders
def segment_gather(words: torch.Tensor, nwords: torch.Tensor, order: torch.Tensor,
                   total: int | None = None):
    """Concatenate the word runs of streams `order` (indices into nwords) in that order.
    words holds the runs of all streams back to back (push order).  Returns
    (nwords[order], words of those runs).  total: the output length if known (saves a
    device->host sync)."""
    nwords = nwords.to(torch.int64)
    start = torch.cumsum(nwords, 0) - nwords
    lens = nwords[order]
    if total is None:
        total = int(lens.sum().item()) if lens.numel() else 0
    if total == 0:
        return lens, words[:0]
    src = start[order]
    dst = torch.cumsum(lens, 0) - lens
    seg = torch.repeat_interleave(torch.arange(order.numel(), device=words.device), lens,
                                  output_size=total)
    pos = torch.arange(total, device=words.device, dtype=torch.int64)
    return lens, words[src[seg] + (pos - dst[seg])]


def _rank_counts(n_images: int, world: int):
    return [shard_range(n_images, r, world) for r in range(world)]


def interleave_levels(states, nwords, words, world: int, n_levels: int,
                      per_rank_images: int | list[int], total: int | None = None):
    """Reorder rank-major gathered streams (rank, level, local image) into the single-batch
    order (level, global image) of idfcodec.codec.Bitstream.  per_rank_images: one count for
    equal shards, or the list of each rank's image count."""
    counts = ([per_rank_images] * world if isinstance(per_rank_images, int)
              else list(per_rank_images))
    if len(counts) != world:
        raise ValueError("per_rank_images must list one image count per rank")
    base, bases = 0, []
    for c in counts:
        bases.append(base)
        base += n_levels * c
    if base != states.numel():
        raise ValueError(f"{states.numel()} streams gathered, {base} expected")
    idx = []
    for l in range(n_levels):
        for r in range(world):
            b0 = bases[r] + l * counts[r]
            idx.extend(range(b0, b0 + counts[r]))
    order = torch.tensor(idx, dtype=torch.int64, device=states.device)
    nw, w = segment_gather(words, nwords, order.to(words.device), total)
    return states[order], nw.to(nwords.dtype), w


def shard_streams(states, nwords, words, n_levels: int, n_images: int, lo: int, hi: int):
    """The streams of images [lo, hi) of a single-batch bitstream, in the shard's own order
    (level-major, local-image-minor)."""
    idx = [l * n_images + b for l in range(n_levels) for b in range(lo, hi)]
    order = torch.tensor(idx, dtype=torch.int64, device=states.device)
    nw, w = segment_gather(words, nwords, order.to(words.device))
    return states[order], nw.to(nwords.dtype), w


# ------------------------------------------------------------------ collectives
# Backend "nccl" (RCCL over xGMI) moves device tensors directly.  Backend "gloo" moves host
# tensors only: there a device tensor is staged through host memory, so the same code runs
# the bench's N-rank path on one GPU (IDF_DIST_BACKEND=gloo, a rehearsal of the RCCL run).
def _staged(t, group) -> bool:
    return t.is_cuda and dist.get_backend(group) == dist.Backend.GLOO


def _p2p(ops):
    """ops: (is_send, tensor, peer, group) tuples or None; runs them as one batch."""
    ops = [o for o in ops if o is not None]
    if not ops:
        return
    p2p, back = [], []
    for is_send, t, peer, group in ops:
        if _staged(t, group):
            h = t.cpu() if is_send else torch.empty(t.shape, dtype=t.dtype)
            if not is_send:
                back.append((t, h))
            t = h
        p2p.append(dist.P2POp(dist.isend if is_send else dist.irecv, t, peer, group))
    for req in dist.batch_isend_irecv(p2p):
        req.wait()
    for t, h in back:
        t.copy_(h)


def _send(t, peer, group):
    return (True, t, peer, group) if t.numel() else None


def _recv(t, peer, group):
    return (False, t, peer, group) if t.numel() else None


def _broadcast(t, src, group):
    if _staged(t, group):
        h = t.cpu()
        dist.broadcast(h, src=src, group=group)
        t.copy_(h)
    else:
        dist.broadcast(t, src=src, group=group)


def all_reduce(t, op=dist.ReduceOp.SUM, group=None):
    """dist.all_reduce, staged through host memory under gloo."""
    if _staged(t, group):
        h = t.cpu()
        dist.all_reduce(h, op=op, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, op=op, group=group)


def _gather_hdr(hdr, dst, group):
    """A fixed-size int64 header from every rank to dst: the list of headers on dst, else None."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    if _staged(hdr, group):
        h = hdr.cpu()
        hs = [torch.empty_like(h) for _ in range(world)] if rank == dst else None
        dist.gather(h, hs, dst=dst, group=group)
        return hs
    hs = [torch.empty_like(hdr) for _ in range(world)] if rank == dst else None
    dist.gather(hdr, hs, dst=dst, group=group)
    return hs


def gather_streams(states: torch.Tensor, nwords: torch.Tensor, words: torch.Tensor, dst: int = 0,
                   group=None):
    """Gather every rank's (states[int64 n_s], nwords[int64 n_s], words[int32 total]) to `dst`.

    Shards may differ in size.  Returns, on `dst`, (states, nwords, words) concatenated in
    rank order; None elsewhere.  Traffic: a 16-byte header per rank through a gather, then
    each shard's metadata and words sent once, point to point, to dst."""
    rank = dist.get_rank(group)
    dev = words.device
    hdr = torch.tensor([states.numel(), words.numel()], dtype=torch.int64, device=dev)
    hdrs = _gather_hdr(hdr, dst, group)
    meta = torch.cat([states.view(torch.int64), nwords.to(torch.int64)])
    if rank != dst:
        _p2p([_send(meta, dst, group), _send(words.contiguous(), dst, group)])
        return None
    sizes = torch.stack(hdrs).cpu().tolist()  # the one host sync: every shard's sizes
    ns_tot = sum(s[0] for s in sizes)
    nw_tot = sum(s[1] for s in sizes)
    st_out = torch.empty(ns_tot, dtype=torch.int64, device=dev)
    nw_out = torch.empty(ns_tot, dtype=torch.int64, device=dev)
    w_out = torch.empty(nw_tot, dtype=words.dtype, device=dev)
    metas, ops = [], []
    so = wo = 0
    for r, (ns, nw) in enumerate(sizes):
        if r == rank:
            st_out[so:so + ns] = states.view(torch.int64)
            nw_out[so:so + ns] = nwords.to(torch.int64)
            w_out[wo:wo + nw] = words
        else:
            m = torch.empty(2 * ns, dtype=torch.int64, device=dev)
            metas.append((m, so, ns))
            ops += [_recv(m, r, group), _recv(w_out[wo:wo + nw], r, group)]
        so += ns
        wo += nw
    _p2p(ops)
    for m, so, ns in metas:
        st_out[so:so + ns] = m[:ns]
        nw_out[so:so + ns] = m[ns:]
    return st_out, nw_out, w_out


def scatter_streams(states, nwords, words, n_levels: int, n_images: int, src: int = 0,
                    group=None, device=None):
    """Decode-side mirror of gather_streams: `src` holds a single-batch bitstream of
    n_images images (states / nwords / words; other ranks pass None and their device);
    every rank receives the streams of its image shard shard_range(n_images, rank, world)
    in shard order.  Returns (states, nwords, words, (lo, hi)) on every rank."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = words.device if rank == src else torch.device(device or "cpu")
    hdr = torch.tensor([n_levels, n_images], dtype=torch.int64, device=dev)
    _broadcast(hdr, src, group)
    n_levels, n_images = (int(v) for v in hdr.cpu().tolist())
    ranges = _rank_counts(n_images, world)
    lo, hi = ranges[rank]
    if rank == src:
        mine = None
        meta_ops, word_ops, keep = [], [], []
        for r, (a, b) in enumerate(ranges):
            st, nw, w = shard_streams(states, nwords, words, n_levels, n_images, a, b)
            if r == rank:
                mine = (st, nw.to(torch.int64), w)
                continue
            meta = torch.cat([st.view(torch.int64), nw.to(torch.int64)])
            w = w.contiguous()
            keep += [meta, w]
            meta_ops.append(_send(meta, r, group))
            word_ops.append(_send(w, r, group))
        # metadata first: receivers size their word buffers from it
        _p2p(meta_ops)
        _p2p(word_ops)
        return (*mine, (lo, hi))
    ns = n_levels * (hi - lo)
    meta = torch.empty(2 * ns, dtype=torch.int64, device=dev)
    _p2p([_recv(meta, src, group)])
    st, nw = meta[:ns].clone(), meta[ns:].clone()
    total = int(nw.sum().item()) if ns else 0
    w = torch.empty(total, dtype=torch.int32, device=dev)
    _p2p([_recv(w, src, group)])
    return st, nw, w, (lo, hi)


def broadcast_state(module: torch.nn.Module, src: int = 0, group=None):
    """Make every rank's parameters and buffers equal to `src`'s: one broadcast of a flat
    buffer per dtype (the imagenet64 flow is 241 MB fp32 -- a few large xGMI transfers,
    not one collective per tensor).  Call before building the FlowEngine (it packs the
    weights once)."""
    tensors = [t for t in module.state_dict().values() if t.numel()]
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    for (dt, dv), ts in sorted(by_dtype.items(), key=lambda kv: str(kv[0])):
        flat = torch.cat([t.detach().reshape(-1) for t in ts])
        _broadcast(flat, src, group)
        o = 0
        with torch.no_grad():
            for t in ts:
                n = t.numel()
                t.copy_(flat[o:o + n].view_as(t))
                o += n


def gather_padded(t: torch.Tensor, dst: int = 0, group=None):
    """Gather a variable-length 1-D tensor from every rank to `dst` (rank order); None elsewhere."""
    rank = dist.get_rank(group)
    dev = t.device
    hdr = torch.tensor([t.numel()], dtype=torch.int64, device=dev)
    hdrs = _gather_hdr(hdr, dst, group)
    if rank != dst:
        _p2p([_send(t.contiguous(), dst, group)])
        return None
    sizes = torch.cat(hdrs).cpu().tolist()
    out = torch.empty(sum(sizes), dtype=t.dtype, device=dev)
    ops, o = [], 0
    for r, n in enumerate(sizes):
        if r == rank:
            out[o:o + n] = t
        else:
            ops.append(_recv(out[o:o + n], r, group))
        o += n
    _p2p(ops)
    return out


def merge_residual(parts):
    """Concatenate equal-shaped ResidualBitstreams of consecutive image shards into the
    single-batch bitstream (flow streams re-ordered level-major / global-image-minor,
    index code runs concatenated)."""
    fl = [p.flow for p in parts]
    modes = {f.meta.get("conv", "f32") for f in fl}
    if len(modes) != 1:
        raise ValueError(f"shards coded with different conv modes {sorted(modes)}: re-encode "
                         "them in one mode (ImageCodec engine.set_conv_mode) before merging")
    st = torch.cat([f.states for f in fl])
    nw = torch.cat([f.nwords.to(torch.int64) for f in fl])
    w = torch.cat([f.words for f in fl])
    return _assemble(parts[0], len(parts), st, nw, w, torch.cat([p.idx_words for p in parts]))


def _assemble(first, world, st, nw, w, idx):
    from .codec import Bitstream
    from .residual import ResidualBitstream
    fl = first.flow
    st, nw, w = interleave_levels(st, nw, w, world, len(fl.level_shapes), fl.n_images)
    meta = {k: v for k, v in fl.meta.items() if k in ("n_subpixels", "conv")}
    if "n_subpixels" in meta:
        meta["n_subpixels"] = meta["n_subpixels"] * world
    flow = Bitstream(fl.n_images * world, fl.level_shapes, st, nw, w, None, meta)
    return ResidualBitstream(flow, idx, first.n_images * world, first.image_shape, first.grid,
                             first.embed_num, first.source_hw)


def agree_conv_mode(bs, group=None):
    """Every shard must have run the same conv arithmetic (a tripped split-f16 range guard on
    one rank re-encodes that shard with exact-f32 convs).  Raises ValueError otherwise."""
    from .codec import CONV_CODES
    code = CONV_CODES[bs.meta.get("conv", "f32")]
    both = torch.tensor([code, -code], dtype=torch.int64, device=bs.words.device)
    all_reduce(both, dist.ReduceOp.MAX, group)
    hi, neg_lo = both.cpu().tolist()
    if hi != -neg_lo:
        raise ValueError("shards coded with different conv modes: re-encode the x3 shards "
                         "with engine.set_conv_mode('f32') and gather again")


def gather_bitstream(bs, dst: int = 0, group=None):
    """The single-batch Bitstream of all ranks' equal image shards, on `dst` (None elsewhere):
    gather_streams + interleave_levels, the n_subpixels scaled to the whole batch."""
    from .codec import Bitstream
    world = dist.get_world_size(group)
    agree_conv_mode(bs, group)
    got = gather_streams(bs.states, bs.nwords, bs.words, dst=dst, group=group)
    if got is None:
        return None
    st, nw, w = got
    st, nw, w = interleave_levels(st, nw, w, world, len(bs.level_shapes), bs.n_images,
                                  total=w.numel())
    meta = {k: v for k, v in bs.meta.items() if k in ("n_subpixels", "conv")}
    if "n_subpixels" in meta:
        meta["n_subpixels"] = meta["n_subpixels"] * world
    return Bitstream(bs.n_images * world, bs.level_shapes, st, nw, w, None, meta)


def scatter_bitstream(bs, src: int = 0, group=None, device=None):
    """Each rank's shard of the single-batch Bitstream `bs` held by `src` (others pass None
    and their device): the decode-side mirror of gather_bitstream.  Returns (Bitstream of
    the rank's images, (lo, hi))."""
    from .codec import Bitstream
    rank = dist.get_rank(group)
    if rank == src:
        hdr_shapes = torch.tensor([v for s in bs.level_shapes for v in s] +
                                  [bs.meta.get("n_subpixels", 0) // max(bs.n_images, 1),
                                   _conv_code(bs)], dtype=torch.int64, device=bs.words.device)
        nlev = torch.tensor([len(bs.level_shapes)], dtype=torch.int64, device=bs.words.device)
    else:
        dev = torch.device(device or "cpu")
        nlev = torch.empty(1, dtype=torch.int64, device=dev)
    _broadcast(nlev, src, group)
    n_levels = int(nlev.item())
    if rank != src:
        hdr_shapes = torch.empty(3 * n_levels + 2, dtype=torch.int64, device=nlev.device)
    _broadcast(hdr_shapes, src, group)
    h = hdr_shapes.cpu().tolist()
    shapes = [tuple(h[3 * i: 3 * i + 3]) for i in range(n_levels)]
    sub_per_img, code = h[-2], h[-1]
    if rank == src:
        st, nw, w, (lo, hi) = scatter_streams(bs.states, bs.nwords, bs.words, n_levels,
                                              bs.n_images, src=src, group=group)
    else:
        st, nw, w, (lo, hi) = scatter_streams(None, None, None, n_levels, 0, src=src,
                                              group=group, device=nlev.device)
    from .codec import CONV_NAMES
    meta = {"n_subpixels": sub_per_img * (hi - lo), "conv": CONV_NAMES[code]}
    return Bitstream(hi - lo, shapes, st, nw, w, None, meta), (lo, hi)


def _conv_code(bs):
    from .codec import CONV_CODES
    return CONV_CODES[bs.meta.get("conv", "f32")]


def gather_residual(rbs, dst: int = 0, group=None):
    """Assemble the residual configs' per-shard ResidualBitstreams (idfcodec.residual) on `dst`
    (RCCL over xGMI with backend nccl): the flow streams via gather_streams, re-ordered to the
    single-batch order, and the image-aligned index code runs concatenated in rank order.
    Equal shards required.  Returns the merged bitstream on `dst`, None elsewhere."""
    world = dist.get_world_size(group)
    agree_conv_mode(rbs.flow, group)
    fl = rbs.flow
    got = gather_streams(fl.states, fl.nwords, fl.words, dst=dst, group=group)
    idx = gather_padded(rbs.idx_words, dst=dst, group=group)
    if got is None:
        return None
    return _assemble(rbs, world, *got, idx)
