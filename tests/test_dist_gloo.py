"""world_size-2 gloo rehearsal of the multi-GPU path (batch shards + bitstream gather)."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import ORACLE, PKG


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _fake_shard(rank, n_levels, per_rank):
    """Deterministic stand-in for one rank's encoded shard: oracle-encoded streams."""
    import sys
    sys.path.insert(0, ORACLE)
    import numpy as np
    import rans_oracle
    g = np.random.default_rng(100 + rank)
    n = 257
    ns = n_levels * per_rank
    mean = g.integers(-64, 64, n * ns).astype(np.float32) / 256
    scale = np.exp(g.normal(-3, 1, n * ns)).astype(np.float32)
    x = (np.round((mean + scale * g.normal(0, 1, n * ns)) * 256) / 256).astype(np.float32)
    off = np.arange(ns + 1, dtype=np.int64) * n
    fs, words, nw, st = rans_oracle.encode_streams(off, x, mean, scale)
    w = np.concatenate([words[off[k]:off[k] + nw[k]] for k in range(ns)])
    return (torch.from_numpy(fs.view(np.int64).copy()), torch.from_numpy(nw.copy()),
            torch.from_numpy(w.view(np.int32).copy()))


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from idfcodec.dist import gather_streams, interleave_levels, shard_range
    lo, hi = shard_range(10, rank, world)
    assert (lo, hi) == ((0, 5) if rank == 0 else (5, 10))
    st, nw, w = _fake_shard(rank, 3, 4)
    res = gather_streams(st, nw, w, dst=0)
    if rank == 0:
        st_all, nw_all, w_all = res
        st2, nw2, w2 = interleave_levels(st_all, nw_all, w_all, world, 3, 4)
        torch.save({"st": st_all, "nw": nw_all, "w": w_all, "st2": st2, "nw2": nw2, "w2": w2}, out)
    else:
        assert res is None
    dist.barrier()
    dist.destroy_process_group()


def test_gather_streams_two_ranks(tmp_path):
    out = str(tmp_path / "g.pt")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r = torch.load(out, weights_only=True)
    parts = [_fake_shard(k, 3, 4) for k in range(2)]
    assert torch.equal(r["st"], torch.cat([p[0] for p in parts]))
    assert torch.equal(r["nw"], torch.cat([p[1] for p in parts]))
    assert torch.equal(r["w"], torch.cat([p[2] for p in parts]))
    # level-major / global-image order: stream (l, r*4 + b)
    for l in range(3):
        for rnk in range(2):
            for b in range(4):
                j = l * 8 + rnk * 4 + b
                assert r["st2"][j] == parts[rnk][0][l * 4 + b]


def test_shard_range_covers():
    import sys
    sys.path.insert(0, PKG)
    from idfcodec.dist import shard_range
    for n in (0, 1, 7, 256):
        for world in (1, 2, 3, 8):
            rs = [shard_range(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))


def _res_worker(rank, world, port, out):
    import sys
    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from idfcodec.codec import Bitstream
    from idfcodec.dist import gather_residual
    from idfcodec.residual import ResidualBitstream
    st, nw, w = _fake_shard(rank, 2, 3)
    flow = Bitstream(3, [(6, 4, 4), (12, 2, 2)], st, nw, w, meta={"n_subpixels": 3 * 192})
    idx = torch.arange(5, dtype=torch.int32) + 100 * rank  # 5 words: 3 images x 1..2 words
    rbs = ResidualBitstream(flow, idx, 3, (3, 8, 8), (2, 2), 8192)
    res = gather_residual(rbs)
    if rank == 0:
        torch.save({"st": res.flow.states, "idx": res.idx_words, "n": res.n_images,
                    "ns": res.flow.meta["n_subpixels"]}, out)
    else:
        assert res is None
    dist.barrier()
    dist.destroy_process_group()


def test_gather_residual_two_ranks(tmp_path):
    """configs 4/5 (8 x MI355X, batch-sharded): the residual bitstreams of two ranks merge on
    rank 0 -- flow streams in single-batch order, index code runs in rank order."""
    out = str(tmp_path / "r.pt")
    mp.spawn(_res_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r = torch.load(out, weights_only=True)
    assert r["n"] == 6 and r["ns"] == 6 * 192
    assert torch.equal(r["idx"], torch.cat([torch.arange(5) + 100 * k for k in range(2)]).int())
    parts = [_fake_shard(k, 2, 3) for k in range(2)]
    for l in range(2):
        for rnk in range(2):
            for b in range(3):
                assert r["st"][l * 6 + rnk * 3 + b] == parts[rnk][0][l * 3 + b]
