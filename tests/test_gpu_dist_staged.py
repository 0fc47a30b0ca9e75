"""The multi-GPU exchanges (idfcodec.dist) on DEVICE tensors under gloo: two ranks on cuda:0,
every collective staged through host memory -- the path `IDF_DIST_BACKEND=gloo
IDF_SHARE_GPU=1 bench.py --gpus 2` rehearses on one GPU (the production path is RCCL, whose
device tensors need no staging).  Gather -> interleave, scatter, weight broadcast and the
MAX all-reduce must give the same bytes as the host-tensor path (tests/test_dist_gloo.py)."""
import os

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import PKG
from test_dist_gloo import _fake_shard, _free_port

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, out):
    import sys
    sys.path.insert(0, PKG)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from idfcodec.dist import (all_reduce, broadcast_state, gather_streams, interleave_levels,
                               scatter_streams)
    dev = torch.device("cuda", 0)
    L, per = 3, 4
    st, nw, w = (t.to(dev) for t in _fake_shard(rank, L, per))
    got = gather_streams(st, nw, w, dst=0)
    res = {}
    if rank == 0:
        assert all(t.is_cuda for t in got)
        st2, nw2, w2 = interleave_levels(*got, world, L, per)
        res.update(st=got[0].cpu(), nw=got[1].cpu(), w=got[2].cpu())
        # the single-batch file back out to both ranks
        mine = scatter_streams(st2, nw2, w2, L, world * per, src=0)
    else:
        assert got is None
        mine = scatter_streams(None, None, None, L, 0, src=0, device=dev)
    s_st, s_nw, s_w, (lo, hi) = mine
    assert s_w.is_cuda and (lo, hi) == (rank * per, (rank + 1) * per)
    res.update({f"sc_st{rank}": s_st.cpu(), f"sc_nw{rank}": s_nw.cpu(), f"sc_w{rank}": s_w.cpu()})
    torch.manual_seed(rank)
    m = torch.nn.Conv2d(3, 8, 3).to(dev)
    broadcast_state(m)
    res[f"w{rank}"] = m.weight.detach().cpu()
    t = torch.tensor([float(rank + 1)], device=dev)
    all_reduce(t, dist.ReduceOp.MAX)
    res[f"max{rank}"] = t.cpu()
    torch.save(res, out + f".{rank}")
    dist.barrier()
    dist.destroy_process_group()


def test_device_tensors_staged_under_gloo(tmp_path):
    out = str(tmp_path / "d.pt")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r0 = torch.load(out + ".0", weights_only=True)
    r1 = torch.load(out + ".1", weights_only=True)
    sh = [_fake_shard(r, 3, 4) for r in range(2)]
    # gather: rank-order concatenation of the shards, bit for bit
    assert torch.equal(r0["st"], torch.cat([s[0] for s in sh]))
    assert torch.equal(r0["nw"], torch.cat([s[1] for s in sh]).to(torch.int64))
    assert torch.equal(r0["w"], torch.cat([s[2] for s in sh]))
    # scatter of the interleaved file: each rank gets back exactly its own shard
    for r, rr in ((0, r0), (1, r1)):
        assert torch.equal(rr[f"sc_st{r}"], sh[r][0])
        assert torch.equal(rr[f"sc_nw{r}"], sh[r][1].to(torch.int64))
        assert torch.equal(rr[f"sc_w{r}"], sh[r][2])
    torch.manual_seed(0)
    ref = torch.nn.Conv2d(3, 8, 3).weight.detach()
    assert torch.equal(r0["w0"], ref) and torch.equal(r1["w1"], ref)
    assert float(r0["max0"]) == 2.0 and float(r1["max1"]) == 2.0
