"""Batch sharding across ranks and the bitstream gather.

Images are independent, so each rank (one process per GPU) encodes a
contiguous slice of the batch with no data-path collective.  The one exchange
step is assembling the per-shard bitstreams on rank 0: an all_gather of the
small per-rank metadata (word counts) followed by a gather of the
variable-length word buffers, padded to the largest shard (payload ~1.3 B per
symbol, a few MB per batch: latency-bound, not xGMI-bandwidth-bound).  With
backend "nccl" this is RCCL over xGMI; the CPU tests run it over gloo.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


def shard_range(n: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous slice [lo, hi) of n items for `rank` (the first n % world ranks get one more)."""
    q, r = divmod(n, world)
    lo = rank * q + min(rank, r)
    return lo, lo + q + (1 if rank < r else 0)


def gather_streams(states: torch.Tensor, nwords: torch.Tensor, words: torch.Tensor, dst: int = 0,
                   group=None):
    """Gather every rank's (states[int64 n_s], nwords[int64 n_s], words[int32 total]) to `dst`.

    All ranks must hold the same number of streams (equal shards).  Returns, on
    `dst`, (states, nwords, words) concatenated in rank order; None elsewhere.
    Tensors must be on the device the process group communicates on."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = words.device
    n_local = torch.tensor([words.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(sizes, n_local, group=group)
    sizes = [int(s.item()) for s in sizes]
    cap = max(max(sizes), 1)
    padded = torch.zeros(cap, dtype=words.dtype, device=dev)
    padded[: words.numel()] = words
    meta = torch.cat([states.view(torch.int64), nwords.to(torch.int64)])
    if rank == dst:
        wbufs = [torch.empty(cap, dtype=words.dtype, device=dev) for _ in range(world)]
        mbufs = [torch.empty_like(meta) for _ in range(world)]
    else:
        wbufs = mbufs = None
    # gather == all_gather restricted to dst; all_gather keeps the code path
    # identical on backends without a native gather (RCCL exposes gather as p2p)
    if dist.get_backend(group) == "gloo":
        dist.gather(padded, wbufs, dst=dst, group=group)
        dist.gather(meta, mbufs, dst=dst, group=group)
    else:
        allw = [torch.empty(cap, dtype=words.dtype, device=dev) for _ in range(world)]
        allm = [torch.empty_like(meta) for _ in range(world)]
        dist.all_gather(allw, padded, group=group)
        dist.all_gather(allm, meta, group=group)
        if rank == dst:
            wbufs, mbufs = allw, allm
    if rank != dst:
        return None
    ns = states.numel()
    st = torch.cat([m[:ns] for m in mbufs])
    nw = torch.cat([m[ns:] for m in mbufs])
    w = torch.cat([b[:s] for b, s in zip(wbufs, sizes)])
    return st, nw, w


def interleave_levels(states, nwords, words, world: int, n_levels: int, per_rank_images: int):
    """Reorder rank-major gathered streams (rank, level, image) into the single-batch
    order (level, global image) used by idfcodec.codec.Bitstream."""
    ns_rank = n_levels * per_rank_images
    idx = []
    for l in range(n_levels):
        for r in range(world):
            base = r * ns_rank + l * per_rank_images
            idx.extend(range(base, base + per_rank_images))
    idx_t = torch.tensor(idx, dtype=torch.int64, device=states.device)
    off = torch.zeros_like(nwords)
    if nwords.numel() > 1:
        off[1:] = torch.cumsum(nwords, 0)[:-1]
    pieces = [words[int(off[i]): int(off[i]) + int(nwords[i])] for i in idx]
    w = torch.cat(pieces) if pieces else words[:0]
    return states[idx_t], nwords[idx_t], w


def gather_padded(t: torch.Tensor, dst: int = 0, group=None):
    """Gather a variable-length 1-D tensor from every rank to `dst` (rank order); None elsewhere."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    dev = t.device
    n_local = torch.tensor([t.numel()], dtype=torch.int64, device=dev)
    sizes = [torch.zeros_like(n_local) for _ in range(world)]
    dist.all_gather(sizes, n_local, group=group)
    sizes = [int(s.item()) for s in sizes]
    cap = max(max(sizes), 1)
    padded = torch.zeros(cap, dtype=t.dtype, device=dev)
    padded[: t.numel()] = t
    if dist.get_backend(group) == "gloo":
        bufs = [torch.empty(cap, dtype=t.dtype, device=dev) for _ in range(world)] if rank == dst else None
        dist.gather(padded, bufs, dst=dst, group=group)
    else:
        bufs = [torch.empty(cap, dtype=t.dtype, device=dev) for _ in range(world)]
        dist.all_gather(bufs, padded, group=group)
    if rank != dst:
        return None
    return torch.cat([b[:s] for b, s in zip(bufs, sizes)])


def merge_residual(parts):
    """Concatenate equal-shaped ResidualBitstreams of consecutive image shards into the
    single-batch bitstream (flow streams re-ordered level-major / global-image-minor,
    index code runs concatenated)."""
    from .codec import Bitstream
    from .residual import ResidualBitstream
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


def gather_residual(rbs, dst: int = 0, group=None):
    """Assemble the residual configs' per-shard ResidualBitstreams (idfcodec.residual) on `dst`
    (RCCL over xGMI with backend nccl): the flow streams via gather_streams, re-ordered to the
    single-batch order, and the image-aligned index code runs concatenated in rank order.
    Equal shards required.  Returns the merged bitstream on `dst`, None elsewhere."""
    world = dist.get_world_size(group)
    fl = rbs.flow
    # every shard must have run the same conv mode (a tripped split-f16 range guard on one
    # rank re-encodes that shard with exact-f32 convs): agree on it first
    mode = torch.tensor([1 if fl.meta.get("conv", "f32") == "x3" else 0], dtype=torch.int64,
                        device=fl.words.device)
    lo, hi = mode.clone(), mode.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    if int(lo.item()) != int(hi.item()):
        raise ValueError("shards coded with different conv modes: re-encode the x3 shards "
                         "with engine.set_conv_mode('f32') and gather again")
    got = gather_streams(fl.states, fl.nwords, fl.words, dst=dst, group=group)
    idx = gather_padded(rbs.idx_words, dst=dst, group=group)
    if got is None:
        return None
    return _assemble(rbs, world, *got, idx)
