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

import os
import weakref

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


# index tensors of the reorders, per (kind, shard layout, device): built once per batch shape,
# not on every step (a bench step re-uses the same world and batch)
_ORDERS: dict = {}


def _order(key, device, build):
    k = (key, str(device))
    t = _ORDERS.get(k)
    if t is None:
        if len(_ORDERS) >= 64:
            _ORDERS.clear()
        t = _ORDERS[k] = torch.tensor(build(), dtype=torch.int64, device=device)
    return t


def _interleave_idx(counts, n_levels):
    base, bases = 0, []
    for c in counts:
        bases.append(base)
        base += n_levels * c
    idx = []
    for l in range(n_levels):
        for r, c in enumerate(counts):
            b0 = bases[r] + l * c
            idx.extend(range(b0, b0 + c))
    return idx


def _to_device(h: torch.Tensor, device) -> torch.Tensor:
    """A host tensor on `device` without a stream sync (pinned staging, async copy)."""
    device = torch.device(device)
    if device.type == "cpu":
        return h
    return h.pin_memory().to(device, non_blocking=True)


def _interleave(states, nwords, words, world, n_levels, per_rank_images, total=None,
                host_nwords=None):
    counts = ([per_rank_images] * world if isinstance(per_rank_images, int)
              else list(per_rank_images))
    if len(counts) != world:
        raise ValueError("per_rank_images must list one image count per rank")
    if n_levels * sum(counts) != states.numel():
        raise ValueError(f"{states.numel()} streams gathered, {n_levels * sum(counts)} expected")
    key = ("interleave", tuple(counts), n_levels)
    order = _order(key, states.device, lambda: _interleave_idx(counts, n_levels))
    worder = order if words.device == states.device else _order(
        key, words.device, lambda: _interleave_idx(counts, n_levels))
    nw_h = None
    if host_nwords is not None:
        nw_h = host_nwords.to(torch.int64)[_order(key, "cpu", lambda: _interleave_idx(
            counts, n_levels))]
        if total is None:
            total = int(nw_h.sum())
    nw, w = segment_gather(words, nwords, worder, total)
    return states[order], nw.to(nwords.dtype), w, nw_h


def interleave_levels(states, nwords, words, world: int, n_levels: int,
                      per_rank_images: int | list[int], total: int | None = None):
    """Reorder rank-major gathered streams (rank, level, local image) into the single-batch
    order (level, global image) of idfcodec.codec.Bitstream.  per_rank_images: one count for
    equal shards, or the list of each rank's image count."""
    return _interleave(states, nwords, words, world, n_levels, per_rank_images, total)[:3]


def _shard_idx(n_levels, n_images, lo, hi):
    return [l * n_images + b for l in range(n_levels) for b in range(lo, hi)]


def _shard(states, nwords, words, n_levels, n_images, lo, hi, host_nwords=None):
    key = ("shard", n_levels, n_images, lo, hi)
    build = lambda: _shard_idx(n_levels, n_images, lo, hi)  # noqa: E731
    order = _order(key, states.device, build)
    worder = order if words.device == states.device else _order(key, words.device, build)
    nw_h, total = None, None
    if host_nwords is not None:
        nw_h = host_nwords.to(torch.int64)[_order(key, "cpu", build)]
        total = int(nw_h.sum())
    nw, w = segment_gather(words, nwords, worder, total)
    return states[order], nw.to(nwords.dtype), w, nw_h


def shard_streams(states, nwords, words, n_levels: int, n_images: int, lo: int, hi: int):
    """The streams of images [lo, hi) of a single-batch bitstream, in the shard's own order
    (level-major, local-image-minor)."""
    return _shard(states, nwords, words, n_levels, n_images, lo, hi)[:3]


# ------------------------------------------------------------------ collectives
# Backend "nccl" (RCCL over xGMI) moves device tensors directly.  Backend "gloo" moves host
# tensors only: there a device tensor is staged through host memory, so the same code runs
# the bench's N-rank path on one GPU (IDF_DIST_BACKEND=gloo, a rehearsal of the RCCL run).
#
# Sizes, word-count tables and header fields are host-resident at their producer (tensor
# shapes, the encoder's compaction, a file), so they travel on a gloo group over the same
# ranks: no exchange reads a device value back to size its buffers, and the timed step's
# stream never drains for one.  Only the payload (final states, words) moves over RCCL.
_HOST_GROUPS: dict = {}
# build the separate gloo group even when `group` is gloo itself, so the RCCL configuration's
# two-group traffic runs under gloo (tests; IDF_DIST_HOST_GROUP=separate for the bench rehearsal)
SEPARATE_HOST_GROUP = os.environ.get("IDF_DIST_HOST_GROUP") == "separate"


def host_group(group=None):
    """The gloo group over `group`'s ranks that carries host metadata (`group` itself under
    gloo).  Created on first use; for a sub-group of an RCCL world every rank of the world must
    call this once, together, before the first exchange (torch.distributed.new_group is
    collective over the world)."""
    if dist.get_backend(group) == dist.Backend.GLOO and not SEPARATE_HOST_GROUP:
        return group
    # keyed by the group's ranks and checked against the group object itself (a weak
    # reference): a destroyed group, or a re-initialised world, never hands out the gloo
    # group of its predecessor even if the new group object reuses the old one's id()
    pg = group if group is not None else dist.distributed_c10d._get_default_group()
    ranks = tuple(dist.get_process_group_ranks(pg))
    hit = _HOST_GROUPS.get(ranks)
    if hit is not None and hit[0]() is pg:
        return hit[1]
    g = dist.new_group(ranks=None if group is None else list(ranks), backend="gloo")
    _HOST_GROUPS[ranks] = (weakref.ref(pg), g)
    return g


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
    """A fixed-size host int64 header from every rank to dst over the host group: the list of
    headers on dst, else None."""
    hg = host_group(group)
    world = dist.get_world_size(hg)
    hs = [torch.empty_like(hdr) for _ in range(world)] if dist.get_rank(hg) == dst else None
    dist.gather(hdr, hs, dst=dst, group=hg)
    return hs


def _gather(states, nwords, words, dst, group, host_nwords):
    rank = dist.get_rank(group)
    hg = host_group(group)
    dev = words.device
    nw_h = (nwords.detach().to("cpu", torch.int64) if host_nwords is None
            else host_nwords.to(torch.int64))
    hdr = torch.tensor([states.numel(), words.numel()], dtype=torch.int64)
    hdrs = _gather_hdr(hdr, dst, group)
    if rank != dst:
        _p2p([_send(nw_h, dst, hg)])
        _p2p([_send(states.view(torch.int64).contiguous(), dst, group),
              _send(words.contiguous(), dst, group)])
        return None
    sizes = torch.stack(hdrs).tolist()  # host values: every shard's stream and word count
    ns_tot = sum(s[0] for s in sizes)
    nw_tot = sum(s[1] for s in sizes)
    parts, ops = [], []
    for r, (ns, _) in enumerate(sizes):
        if r == rank:
            parts.append(nw_h)
        else:
            parts.append(torch.empty(ns, dtype=torch.int64))
            ops.append(_recv(parts[-1], r, hg))
    _p2p(ops)
    nw_host = torch.cat(parts) if parts else torch.zeros(0, dtype=torch.int64)
    st_out = torch.empty(ns_tot, dtype=torch.int64, device=dev)
    w_out = torch.empty(nw_tot, dtype=words.dtype, device=dev)
    ops = []
    so = wo = 0
    for r, (ns, nw) in enumerate(sizes):
        if r == rank:
            st_out[so:so + ns] = states.view(torch.int64)
            w_out[wo:wo + nw] = words
        else:
            ops += [_recv(st_out[so:so + ns], r, group), _recv(w_out[wo:wo + nw], r, group)]
        so += ns
        wo += nw
    _p2p(ops)
    return st_out, _to_device(nw_host, dev), w_out, nw_host


def gather_streams(states: torch.Tensor, nwords: torch.Tensor, words: torch.Tensor, dst: int = 0,
                   group=None, host_nwords: torch.Tensor | None = None):
    """Gather every rank's (states[int64 n_s], nwords[int64 n_s], words[int32 total]) to `dst`.

    Shards may differ in size.  Returns, on `dst`, (states, nwords, words) concatenated in
    rank order; None elsewhere.  Traffic: a 16-byte header and the word-count table per rank
    on the host group, then each shard's final states and words sent once, point to point,
    to dst.  host_nwords: the host copy of nwords if the caller has one (else one read)."""
    got = _gather(states, nwords, words, dst, group, host_nwords)
    return None if got is None else got[:3]


def _scatter(states, nwords, words, n_levels, n_images, src, group, device, host_nwords):
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    hg = host_group(group)
    dev = words.device if rank == src else torch.device(device or "cpu")
    hdr = torch.tensor([n_levels, n_images], dtype=torch.int64)
    dist.broadcast(hdr, src=src, group=hg)
    n_levels, n_images = (int(v) for v in hdr.tolist())
    ranges = _rank_counts(n_images, world)
    lo, hi = ranges[rank]
    if rank == src:
        nw_all = (nwords.detach().to("cpu", torch.int64) if host_nwords is None
                  else host_nwords.to(torch.int64))
        mine, shards = None, []
        for r, (a, b) in enumerate(ranges):
            st, nw, w, nw_h = _shard(states, nwords, words, n_levels, n_images, a, b, nw_all)
            if r == rank:
                mine = (st, nw.to(torch.int64), w, nw_h)
            else:
                shards.append((r, st, w, nw_h))
        # word-count tables first, on the host group: receivers size their buffers from them
        _p2p([_send(nw_h, r, hg) for r, _, _, nw_h in shards])
        _p2p([op for r, st, w, _ in shards
              for op in (_send(st.view(torch.int64).contiguous(), r, group),
                         _send(w.contiguous(), r, group))])
        return (*mine, (lo, hi))
    ns = n_levels * (hi - lo)
    nw_h = torch.empty(ns, dtype=torch.int64)
    _p2p([_recv(nw_h, src, hg)])
    st = torch.empty(ns, dtype=torch.int64, device=dev)
    w = torch.empty(int(nw_h.sum()), dtype=torch.int32, device=dev)
    _p2p([_recv(st, src, group), _recv(w, src, group)])
    return st, _to_device(nw_h, dev), w, nw_h, (lo, hi)


def scatter_streams(states, nwords, words, n_levels: int, n_images: int, src: int = 0,
                    group=None, device=None, host_nwords: torch.Tensor | None = None):
    """Decode-side mirror of gather_streams: `src` holds a single-batch bitstream of
    n_images images (states / nwords / words; other ranks pass None and their device);
    every rank receives the streams of its image shard shard_range(n_images, rank, world)
    in shard order.  Returns (states, nwords, words, (lo, hi)) on every rank."""
    st, nw, w, _, rng = _scatter(states, nwords, words, n_levels, n_images, src, group, device,
                                 host_nwords)
    return st, nw, w, rng


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
    hdr = torch.tensor([t.numel()], dtype=torch.int64)
    hdrs = _gather_hdr(hdr, dst, group)
    if rank != dst:
        _p2p([_send(t.contiguous(), dst, group)])
        return None
    sizes = torch.cat(hdrs).tolist()
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
    if len({p.vq_conv for p in parts}) != 1:
        raise ValueError("shards' VQ decoders ran different conv modes: re-encode them with "
                         "one IDF_VQ_CONV before merging")
    if len(modes) != 1:
        raise ValueError(f"shards coded with different conv modes {sorted(modes)}: re-encode "
                         "them in one mode (ImageCodec engine.set_conv_mode) before merging")
    st = torch.cat([f.states for f in fl])
    nw = torch.cat([f.nwords.to(torch.int64) for f in fl])
    w = torch.cat([f.words for f in fl])
    return _assemble(parts[0], len(parts), st, nw, w, torch.cat([p.idx_words for p in parts]))


def _assemble(first, world, st, nw, w, idx, nw_host=None):
    from .codec import Bitstream
    from .residual import ResidualBitstream
    fl = first.flow
    st, nw, w, nw_h = _interleave(st, nw, w, world, len(fl.level_shapes), fl.n_images,
                                  host_nwords=nw_host)
    meta = {k: v for k, v in fl.meta.items() if k in ("n_subpixels", "conv")}
    if "n_subpixels" in meta:
        meta["n_subpixels"] = meta["n_subpixels"] * world
    flow = Bitstream(fl.n_images * world, fl.level_shapes, st, nw, w, None, meta, nw_h)
    return ResidualBitstream(flow, idx, first.n_images * world, first.image_shape, first.grid,
                             first.embed_num, first.source_hw, first.vq_conv)


def agree_shards(bs, group=None, vq_conv=None):
    """Before any point-to-point traffic, every rank checks -- on the host group, with one
    MAX all-reduce -- that all shards ran the same conv arithmetic (a tripped split-f16 range
    guard on one rank re-encodes that shard with exact-f32 convs), hold the same number of
    images (gather_bitstream / gather_residual need equal shards) and are compacted (a
    compact=False stream's words sit at scratch offsets, not back to back).  Every rank raises
    the same ValueError, so none is left blocked in a later exchange."""
    from .codec import CONV_CODES
    code = CONV_CODES.get(bs.meta.get("conv", "f32"), -1)
    scratch = int("scratch_offsets" in bs.meta)
    vq_modes = (None, "f32", "x3", "x3t")  # idfcodec.vq.VQ_CONV_MODES, and "no VQ"
    if vq_conv not in vq_modes:
        raise ValueError(f"unknown VQ conv mode {vq_conv!r}")
    vq = vq_modes.index(vq_conv)
    v = torch.tensor([code, -code, bs.n_images, -bs.n_images, scratch, vq, -vq],
                     dtype=torch.int64)
    dist.all_reduce(v, op=dist.ReduceOp.MAX, group=host_group(group))
    hi, neg_lo, n_hi, neg_n_lo, any_scratch, vq_hi, neg_vq_lo = v.tolist()
    if vq_hi != -neg_vq_lo:
        raise ValueError("shards' VQ decoders ran different conv modes (a tripped split-f16 "
                         "guard on one rank): re-encode with IDF_VQ_CONV=f32 and gather again")
    if any_scratch:
        raise ValueError("a shard's bitstream is not compacted (encode(compact=False)): "
                         "gather compacted bitstreams only")
    if hi != -neg_lo or hi < 0:
        raise ValueError("shards coded with different conv modes: re-encode the x3 shards "
                         "with engine.set_conv_mode('f32') and gather again")
    if n_hi != -neg_n_lo:
        raise ValueError("shards hold different image counts: gather_bitstream needs equal "
                         "shards (gather_streams + interleave_levels take ragged ones)")


agree_conv_mode = agree_shards


def gather_bitstream(bs, dst: int = 0, group=None):
    """The single-batch Bitstream of all ranks' equal image shards, on `dst` (None elsewhere):
    gather_streams + interleave_levels, the n_subpixels scaled to the whole batch."""
    from .codec import Bitstream
    world = dist.get_world_size(group)
    agree_shards(bs, group)
    got = _gather(bs.states, bs.nwords, bs.words, dst, group, bs.host_nwords)
    if got is None:
        return None
    st, nw, w, nw_h = _interleave(*got[:3], world, len(bs.level_shapes), bs.n_images,
                                  total=got[2].numel(), host_nwords=got[3])
    meta = {k: v for k, v in bs.meta.items() if k in ("n_subpixels", "conv")}
    if "n_subpixels" in meta:
        meta["n_subpixels"] = meta["n_subpixels"] * world
    return Bitstream(bs.n_images * world, bs.level_shapes, st, nw, w, None, meta, nw_h)


def scatter_bitstream(bs, src: int = 0, group=None, device=None):
    """Each rank's shard of the single-batch Bitstream `bs` held by `src` (others pass None
    and their device): the decode-side mirror of gather_bitstream.  Returns (Bitstream of
    the rank's images, (lo, hi)).  The header travels on the host group."""
    from .codec import CONV_NAMES, Bitstream
    rank = dist.get_rank(group)
    hg = host_group(group)
    if rank == src:
        if "scratch_offsets" in bs.meta:
            raise ValueError("scatter a compacted bitstream (encode(compact=True))")
        hdr_shapes = torch.tensor([v for s in bs.level_shapes for v in s] +
                                  [bs.meta.get("n_subpixels", 0) // max(bs.n_images, 1),
                                   _conv_code(bs)], dtype=torch.int64)
        nlev = torch.tensor([len(bs.level_shapes)], dtype=torch.int64)
    else:
        nlev = torch.empty(1, dtype=torch.int64)
    dist.broadcast(nlev, src=src, group=hg)
    n_levels = int(nlev[0])
    if rank != src:
        hdr_shapes = torch.empty(3 * n_levels + 2, dtype=torch.int64)
    dist.broadcast(hdr_shapes, src=src, group=hg)
    h = hdr_shapes.tolist()
    shapes = [tuple(h[3 * i: 3 * i + 3]) for i in range(n_levels)]
    sub_per_img, code = h[-2], h[-1]
    if rank == src:
        st, nw, w, nw_h, (lo, hi) = _scatter(bs.states, bs.nwords, bs.words, n_levels,
                                             bs.n_images, src, group, None, bs.host_nwords)
    else:
        st, nw, w, nw_h, (lo, hi) = _scatter(None, None, None, n_levels, 0, src, group,
                                             device, None)
    meta = {"n_subpixels": sub_per_img * (hi - lo), "conv": CONV_NAMES[code]}
    return Bitstream(hi - lo, shapes, st, nw, w, None, meta, nw_h), (lo, hi)


def _conv_code(bs):
    from .codec import CONV_CODES
    conv = bs.meta.get("conv", "f32")
    if conv not in CONV_CODES:
        raise ValueError(f"cannot scatter a bitstream with conv mode {conv!r}")
    return CONV_CODES[conv]


def gather_residual(rbs, dst: int = 0, group=None):
    """Assemble the residual configs' per-shard ResidualBitstreams (idfcodec.residual) on `dst`
    (RCCL over xGMI with backend nccl): the flow streams via gather_streams, re-ordered to the
    single-batch order, and the image-aligned index code runs concatenated in rank order.
    Equal shards required.  Returns the merged bitstream on `dst`, None elsewhere."""
    world = dist.get_world_size(group)
    fl = rbs.flow
    agree_shards(fl, group, rbs.vq_conv)
    got = _gather(fl.states, fl.nwords, fl.words, dst, group, fl.host_nwords)
    idx = gather_padded(rbs.idx_words, dst=dst, group=group)
    if got is None:
        return None
    return _assemble(rbs, world, *got[:3], idx, got[3])
