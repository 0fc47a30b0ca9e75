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


def _res_worker(rank, world, port, out, vq_conv="f32"):
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
    rbs = ResidualBitstream(flow, idx, 3, (3, 8, 8), (2, 2), 8192, vq_conv=vq_conv)
    res = gather_residual(rbs)
    if rank == 0:
        assert res.vq_conv == vq_conv
        torch.save({"st": res.flow.states, "idx": res.idx_words, "n": res.n_images,
                    "ns": res.flow.meta["n_subpixels"]}, out)
    else:
        assert res is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("vq_conv", ["f32", "x3", "x3t"])
def test_gather_residual_two_ranks(tmp_path, vq_conv):
    """configs 4/5 (8 x MI355X, batch-sharded): the residual bitstreams of two ranks merge on
    rank 0 -- flow streams in single-batch order, index code runs in rank order -- for every
    VQ conv mode (round 6's default "x3t" included: the one-GPU N=2 rehearsal found it
    missing from agree_shards)."""
    out = str(tmp_path / "r.pt")
    mp.spawn(_res_worker, args=(2, _free_port(), out, vq_conv), nprocs=2, join=True)
    r = torch.load(out, weights_only=True)
    assert r["n"] == 6 and r["ns"] == 6 * 192
    assert torch.equal(r["idx"], torch.cat([torch.arange(5) + 100 * k for k in range(2)]).int())
    parts = [_fake_shard(k, 2, 3) for k in range(2)]
    for l in range(2):
        for rnk in range(2):
            for b in range(3):
                assert r["st"][l * 6 + rnk * 3 + b] == parts[rnk][0][l * 3 + b]


N_SYM = 131


def _stream_inputs(l, b):
    """Deterministic (x, mean, scale) of global stream (level l, image b)."""
    import numpy as np
    g = np.random.default_rng(1000 * l + b)
    mean = g.integers(-64, 64, N_SYM).astype(np.float32) / 256
    scale = np.exp(g.normal(-3, 1, N_SYM)).astype(np.float32)
    x = (np.round((mean + scale * g.normal(0, 1, N_SYM)) * 256) / 256).astype(np.float32)
    return x, mean, scale


def _encode(pairs):
    """oracle-encode the streams `pairs` [(l, b)] in order -> (states, nwords, words) torch."""
    import sys
    sys.path.insert(0, ORACLE)
    import numpy as np
    import rans_oracle
    ins = [_stream_inputs(l, b) for l, b in pairs]
    off = np.arange(len(pairs) + 1, dtype=np.int64) * N_SYM
    cat = lambda i: np.concatenate([t[i] for t in ins]) if ins else np.zeros(0, np.float32)  # noqa
    fs, words, nw, st = rans_oracle.encode_streams(off, cat(0), cat(1), cat(2))
    w = np.concatenate([words[off[k]:off[k] + nw[k]] for k in range(len(pairs))] or
                       [np.zeros(0, np.uint32)])
    return (torch.from_numpy(fs.view(np.int64).copy()), torch.from_numpy(nw.astype(np.int64)),
            torch.from_numpy(w.view(np.int32).copy()))


def _scatter_worker(rank, world, port, n_images, out):
    """rank 0 holds the single-batch bitstream; scatter -> every rank decodes its shard with
    the oracle (exact symbols, final state 2^32) -> re-encodes it -> gather back to rank 0."""
    import sys
    sys.path.insert(0, PKG)
    sys.path.insert(0, ORACLE)
    import numpy as np
    import rans_oracle
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from idfcodec.codec import Bitstream
    from idfcodec.dist import (gather_bitstream, gather_streams, interleave_levels,
                               scatter_bitstream, shard_range)
    L = 2
    shapes = [(1, 1, N_SYM)] * L
    full = None
    if rank == 0:
        st, nw, w = _encode([(l, b) for l in range(L) for b in range(n_images)])
        full = Bitstream(n_images, shapes, st, nw, w, None,
                         {"n_subpixels": n_images * 10, "conv": "x3"})
    mine, (lo, hi) = scatter_bitstream(full, src=0)
    assert (lo, hi) == shard_range(n_images, rank, world)
    assert mine.n_images == hi - lo and mine.meta["conv"] == "x3"
    assert mine.meta["n_subpixels"] == (hi - lo) * 10 and mine.level_shapes == shapes
    # decode every stream of the shard with the oracle
    pairs = [(l, b) for l in range(L) for b in range(lo, hi)]
    ns = len(pairs)
    wnp = mine.words.numpy().view(np.uint32)
    nwn = mine.nwords.numpy()
    woff = np.concatenate([[0], np.cumsum(nwn)[:-1]]).astype(np.int64) if ns else np.zeros(0, np.int64)
    off = np.arange(ns + 1, dtype=np.int64) * N_SYM
    ins = [_stream_inputs(l, b) for l, b in pairs]
    if ns:
        fs, xs, stt = rans_oracle.decode_streams(
            off, woff, nwn, wnp if wnp.size else np.zeros(1, np.uint32),
            np.concatenate([t[1] for t in ins]), np.concatenate([t[2] for t in ins]),
            mine.states.numpy().view(np.uint64))
        assert (fs == 1 << 32).all() and (stt == 0).all()
        assert np.array_equal(xs, np.concatenate([t[0] for t in ins]))
    # encode the shard again and gather it back
    st, nw, w = _encode(pairs)
    got = gather_streams(st, nw, w, dst=0)
    if n_images % world == 0:
        local = Bitstream(hi - lo, shapes, st, nw, w, None,
                          {"n_subpixels": (hi - lo) * 10, "conv": "x3"})
        whole = gather_bitstream(local, dst=0)
    if rank == 0:
        counts = [shard_range(n_images, r, world)[1] - shard_range(n_images, r, world)[0]
                  for r in range(world)]
        st2, nw2, w2 = interleave_levels(*got, world, L, counts)
        res = {"st": st2, "nw": nw2, "w": w2, "st0": full.states, "nw0": full.nwords,
               "w0": full.words}
        if n_images % world == 0:
            res.update(ws=whole.states, wnw=whole.nwords, ww=whole.words,
                       wn=torch.tensor(whole.n_images), wsub=torch.tensor(whole.meta["n_subpixels"]))
        torch.save(res, out)
    else:
        assert got is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_images", [(2, 6), (2, 5), (3, 7)])
def test_scatter_decode_gather_round_trip(tmp_path, world, n_images):
    """Decode side of 8(e): scatter the single-batch bitstream, decode every shard, re-encode,
    gather: the reassembled bitstream equals the original bit for bit (equal and ragged
    shards)."""
    out = str(tmp_path / "s.pt")
    mp.spawn(_scatter_worker, args=(world, _free_port(), n_images, out), nprocs=world, join=True)
    r = torch.load(out, weights_only=True)
    assert torch.equal(r["st"], r["st0"]) and torch.equal(r["nw"], r["nw0"].to(torch.int64))
    assert torch.equal(r["w"], r["w0"])
    if "ws" in r:
        assert torch.equal(r["ws"], r["st0"]) and torch.equal(r["ww"], r["w0"])
        assert int(r["wn"]) == n_images and int(r["wsub"]) == n_images * 10


def _host_group_worker(rank, world, port, out):
    """The RCCL configuration's traffic split on CPU: sizes / word-count tables / headers on a
    separate gloo group, payload on the main group.  Full round trip through
    gather_bitstream / scatter_bitstream; the host word-count tables ride along."""
    import sys
    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import idfcodec.dist as D
    from idfcodec.codec import Bitstream
    D.SEPARATE_HOST_GROUP = True
    L, per = 2, 3
    shapes = [(1, 1, N_SYM)] * L
    pairs = [(l, b) for l in range(L) for b in range(rank * per, (rank + 1) * per)]
    st, nw, w = _encode(pairs)
    local = Bitstream(per, shapes, st, nw, w, None, {"n_subpixels": per * 10, "conv": "f32"},
                      host_nwords=nw.clone())
    res = {}
    for step in range(2):  # the second step re-uses the cached index tensors and host group
        whole = D.gather_bitstream(local, dst=0)
        mine, (lo, hi) = D.scatter_bitstream(whole, src=0)
        assert D.host_group() is not None and len(D._HOST_GROUPS) == 1
        assert torch.equal(mine.host_nwords, mine.nwords.to(torch.int64))
        assert torch.equal(mine.states, st) and torch.equal(mine.words, w) and (lo, hi) == (
            rank * per, (rank + 1) * per)
        if rank == 0:
            assert torch.equal(whole.host_nwords, whole.nwords.to(torch.int64))
            res[f"st{step}"], res[f"w{step}"] = whole.states, whole.words
    if rank == 0:
        torch.save(res, out)
    dist.barrier()
    dist.destroy_process_group()


def test_host_metadata_group_round_trip(tmp_path):
    out = str(tmp_path / "h.pt")
    mp.spawn(_host_group_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r = torch.load(out, weights_only=True)
    st, nw, w = _encode([(l, b) for l in range(2) for b in range(6)])
    for step in range(2):
        assert torch.equal(r[f"st{step}"], st) and torch.equal(r[f"w{step}"], w)


def _agree_worker(rank, world, port, case, out):
    import sys
    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from idfcodec.codec import Bitstream
    from idfcodec.dist import gather_bitstream
    per = 3 if (case != "ragged" or rank == 0) else 2
    st, nw, w = _encode([(l, b) for l in range(2) for b in range(per)])
    meta = {"n_subpixels": per * 10, "conv": "x3" if (case == "mode" and rank == 1) else "f32"}
    if case == "scratch" and rank == 1:
        meta["scratch_offsets"] = torch.zeros(2 * per, dtype=torch.int64)
    bs = Bitstream(per, [(1, 1, N_SYM)] * 2, st, nw, w, None, meta)
    try:
        gather_bitstream(bs, dst=0)
        msg = "ok"
    except ValueError as e:
        msg = str(e)
    with open(out + f".{rank}", "w") as f:
        f.write(msg)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("case,match", [("ragged", "image counts"), ("scratch", "compacted"),
                                        ("mode", "conv modes")])
def test_gather_bitstream_refuses_on_every_rank(tmp_path, case, match):
    """ADVICE r2 (dist.py:330): unequal shards, an uncompacted stream or mixed conv modes are
    found by one host all-reduce before any point-to-point traffic, and every rank raises (no
    rank is left blocked in the exchange)."""
    out = str(tmp_path / "a")
    mp.spawn(_agree_worker, args=(2, _free_port(), case, out), nprocs=2, join=True)
    for r in range(2):
        with open(out + f".{r}") as f:
            assert match in f.read()


def _bcast_worker(rank, world, port, out):
    import sys
    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from idfcodec.dist import broadcast_state
    torch.manual_seed(rank)  # every rank starts from different weights
    m = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8))
    broadcast_state(m)
    torch.save({k: v for k, v in m.state_dict().items()}, out + f".{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_broadcast_state_two_ranks(tmp_path):
    out = str(tmp_path / "b.pt")
    mp.spawn(_bcast_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    a = torch.load(out + ".0", weights_only=True)
    b = torch.load(out + ".1", weights_only=True)
    torch.manual_seed(0)
    ref = torch.nn.Sequential(torch.nn.Conv2d(3, 8, 3), torch.nn.BatchNorm2d(8)).state_dict()
    for k in ref:
        assert torch.equal(a[k], b[k]) and torch.equal(a[k], ref[k]), k


def test_bench_launches_n_ranks():
    """`bench.py --gpus 2` starts 2 ranks itself (torch.distributed.run) without touching the
    GPU in the parent; --launch-probe makes each rank report and exit."""
    import json
    import subprocess
    import sys
    from conftest import REPO
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2",
                        "--launch-probe"], capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(d["rank"] for d in lines) == [0, 1]
    assert all(d["world"] == 2 for d in lines)
