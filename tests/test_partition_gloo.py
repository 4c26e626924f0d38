"""Multi-process (gloo, world_size 2 and 4) test of the edge partition + chunked all-reduce.

The per-shard aggregate is computed by the fp64 oracle on CPU (no GPU here);
on the GPU box the same code path runs libgta per chunk and RCCL all-reduces.
Checks: column cuts balance nnz, shards partition the edge set exactly, and
the all-reduced sum of shard aggregates equals the single-device aggregate.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, partition
from oracle import isa_ref


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _np_aggregate(g, x, w, out_view, plan):
    ip = g.indptr.numpy()
    ip0 = ip - ip[0]
    ix = g.indices.numpy()[ip[0]:ip[-1]]
    ww = None if w is None else w.numpy()[ip[0]:ip[-1]]
    out_view.copy_(torch.from_numpy(isa_ref.aggregate(ip0, ix, x.numpy(), "src", ww).astype(np.float32)))


def _worker(rank, world, port, n, e, F, H, n_chunks, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = G.synthetic(n, e, seed=4)
        gen = torch.Generator().manual_seed(9)
        x = torch.randn(n, F, generator=gen)
        w = torch.rand(g.nnz, H, generator=gen)
        shard = partition.make_shard(g, rank, world)
        xl = x[shard.c0:shard.c1].contiguous()
        wl = w[shard.edge_ids].contiguous()
        chunked = partition.ChunkedRows(shard.graph, n_chunks=n_chunks, chunk=0)
        y = torch.zeros(n, F)
        partition.distributed_aggregate(chunked, xl, wl, y, aggregate_fn=_np_aggregate)
        counts = torch.tensor([shard.graph.nnz], dtype=torch.int64)
        dist.all_reduce(counts)
        if rank == 0:
            ip, ix = g.numpy()
            ref = isa_ref.aggregate(ip, ix, x.numpy(), "src", w.numpy())
            bound = 1e-5 * isa_ref.aggregate_abs(ip, ix, x.numpy(), "src", w.numpy()) + 1e-6
            ok = bool(np.all(np.abs(y.numpy() - ref) <= bound))
            q.put((ok, int(counts.item()), g.nnz, float(np.abs(y.numpy() - ref).max())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n_chunks", [(2, 1), (2, 4), (4, 3)])
def test_distributed_aggregate_gloo(world, n_chunks):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, 500, 8000, 16, 4, n_chunks, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    ok, total, nnz, err = q.get(timeout=10)
    assert total == nnz, "shards must partition the edge set"
    assert ok, f"all-reduced shard aggregates differ from the single-device result (max err {err})"


def test_column_cuts_balance():
    g = G.synthetic(5000, 200000, seed=1)
    for world in (2, 4, 8):
        cuts = partition.column_cuts(g, world)
        assert cuts[0] == 0 and cuts[-1] == g.n_cols and torch.all(cuts[1:] >= cuts[:-1])
        sizes = [partition.make_shard(g, r, world, cuts).graph.nnz for r in range(world)]
        assert sum(sizes) == g.nnz
        assert max(sizes) <= 1.05 * g.nnz / world + 200
