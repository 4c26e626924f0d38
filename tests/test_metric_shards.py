"""The headline workload's inputs (metric.py) and its multi-GPU layouts, on the CPU.

* graph.CounterCSR / hash_normal: counter-hashed, so any row range or id subset is generated on its
  own, bitwise equal to the same part of the whole graph (what lets each rank of the multi-GPU
  bench build only its tile);
* metric.Shard on every rank of a grid: the tiles cover every edge once with the whole graph's
  alpha, and the row groups' partial aggregates, reduce-scattered chunk by chunk and reassembled
  from every rank's owned rows, equal the whole-graph fp64 oracle;
* bench.Aggregate.step under gloo (world 2 and 4, both modes) with the oracle standing in for the
  kernel: the exchange logic the RCCL run uses, end to end.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed, graph as G, metric
from oracle import isa_ref

N, E = 2000, 40000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_hash_is_pinned_and_exact():
    """lowbias32 (no int64 overflow anywhere) -- pinned values, so a change of the generator shows."""
    x = torch.tensor([0, 1, 2, 0xFFFFFFFF, 123456789], dtype=torch.int64)
    assert G.mix32(x).tolist() == [0, 1753845952, 3507691905, 1734902346, 2834422664]
    h = G.hash32(torch.arange(5, dtype=torch.int64), 0, 1)
    assert torch.equal(h, G.hash32(torch.arange(5, dtype=torch.int64), 0, 1))
    z = G.hash_normal(torch.arange(200000, dtype=torch.int64), 0, 2, torch.float64)
    assert abs(float(z.mean())) < 0.01 and abs(float(z.std()) - 1.0) < 0.01


def test_counter_csr_rows_are_slices_of_the_whole():
    csr = G.CounterCSR(N, E, seed=3)
    lip, src, gen = csr.rows(0, N, "cpu")
    assert int(lip[-1]) == E and src.numel() == E
    ip = lip.numpy()
    s = src.numpy()
    for r in range(0, N, 131):
        seg = s[ip[r]:ip[r + 1]]
        assert np.all(np.diff(seg) >= 0) and (seg.size == 0 or (seg.min() >= 0 and seg.max() < N))
    assert torch.equal(torch.sort(gen).values, torch.arange(E))
    for r0, r1 in ((0, 7), (500, 1333), (1999, 2000)):
        l2, s2, g2 = csr.rows(r0, r1, "cpu")
        e0, e1 = int(lip[r0]), int(lip[r1])
        assert torch.equal(l2, lip[r0:r1 + 1] - e0)
        assert torch.equal(s2, src[e0:e1]) and torch.equal(g2, gen[e0:e1])
    # degrees: lognormal, skewed, exact total
    deg = np.diff(ip)
    assert deg.sum() == E and deg.max() > 4 * deg.mean()


def test_alpha_is_a_per_row_softmax():
    whole = metric.Shard(N, E, 0, 1, 1, 1, "cpu")
    ip, _ = whole.graph.numpy()
    rows = np.repeat(np.arange(N), np.diff(ip))
    s = np.zeros((N, metric.HEADS))
    np.add.at(s, rows, whole.alpha.double().numpy())
    nz = np.diff(ip) > 0
    assert np.allclose(s[nz], 1.0, atol=1e-5)
    assert torch.equal(whole.x, metric.x_rows(torch.arange(N), "cpu"))


def _global_counts(pr, pc):
    """What the all-reduce of every rank's row-group column histogram returns."""
    csr = G.CounterCSR(N, E)
    rc = distributed.row_cuts_ip(torch.from_numpy(csr.indptr_np), pr)
    tot = torch.zeros(N, dtype=torch.int64)
    for i in range(pr):
        tot += torch.bincount(csr.rows(rc[i], rc[i + 1], "cpu")[1], minlength=N) * pc
    return lambda c: tot.clone()


@pytest.mark.parametrize("pr,pc,chunks,fracs", [(1, 2, 1, None), (2, 2, 2, None), (4, 2, 2, None), (3, 1, 2, None),
                                                (1, 4, 3, None), (4, 2, 2, (0.7, 0.3)), (2, 2, 3, (0.5, 0.3, 0.2)),
                                                (1, 2, 2, (0.9, 0.1))])
def test_grid_tiles_reassemble_to_the_whole_aggregate(pr, pc, chunks, fracs):
    """Every rank's tile aggregate, reduce-scattered chunk by chunk inside its row group, covers
    each row exactly once and equals the whole-graph oracle; equal and weighted chunk sizes
    (bench's default in edges mode: 70 / 30, the smaller chunk last)."""
    whole = metric.Shard(N, E, 0, 1, 1, 1, "cpu")
    ip, ix = whole.graph.numpy()
    ref = isa_ref.aggregate(ip, ix, whole.x.numpy(), "src", whole.alpha.numpy())
    world = pr * pc
    shards = [metric.Shard(N, E, r, pr, pc, chunks, "cpu", count_reduce=_global_counts(pr, pc), fracs=fracs)
              for r in range(world)]
    assert sum(s.graph.nnz for s in shards) == E
    partial = {}
    for r, s in enumerate(shards):
        sip, six = s.graph.numpy()
        partial[r] = isa_ref.aggregate(sip, six, s.x.numpy(), "src", s.alpha.numpy())
        # every tile edge carries the whole graph's alpha and source
        ge = s.grid.edge_ids.numpy()
        np.testing.assert_array_equal(whole.alpha.numpy()[ge], s.alpha.numpy())
        np.testing.assert_array_equal(ix[ge], six + s.grid.c0)
    full = np.full((N, metric.F), np.nan)
    for r, s in enumerate(shards):
        g = s.grid
        own = []
        for c in range(g.chunks):  # the reduce-scatter of chunk c inside row group i
            a, b = g.chunk_rows(c)
            tot = sum(partial[g.i * pc + jj][a:b] for jj in range(pc))
            p0, p1 = g.part(c)
            assert (b - a) == pc * (p1 - p0)  # one equal part per rank of the group
            own.append(tot[g.j * (p1 - p0):(g.j + 1) * (p1 - p0)])
        own = np.concatenate(own)
        rows = g.owned_rows(r).numpy()
        ok = rows >= 0
        assert np.all(np.isnan(full[rows[ok]]))  # every row owned once
        full[rows[ok]] = own[ok]
    assert not np.isnan(full).any()
    np.testing.assert_allclose(full, ref, rtol=0, atol=1e-12)


def test_default_grids():
    assert distributed.grid_shape(1) == (1, 1)
    assert [distributed.grid_shape(w) for w in (2, 4, 8)] == [(1, 2), (2, 2), (4, 2)]
    assert [distributed.grid_shape(w, "rows") for w in (2, 4, 8)] == [(2, 1), (4, 1), (8, 1)]


def _bench_worker(rank, world, port, mode, q, n=N, e=E, chunks=2):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import types

        import bench

        def launch(self, c):  # the oracle in place of the HIP kernel (no GPU here)
            a, b, gg = self.parts[c]
            ip = gg.indptr.numpy() - int(gg.indptr[0])
            ix = gg.indices.numpy()[int(gg.indptr[0]):int(gg.indptr[-1])]
            w = self.alpha.numpy()[int(gg.indptr[0]):int(gg.indptr[-1])]
            self.y[a:b] = torch.from_numpy(isa_ref.aggregate(ip, ix, self.x.numpy(), "src", w).astype(np.float32))

        bench.Aggregate.launch = launch
        bench.ops.BlockedPlan.auto_blocks = staticmethod(lambda g, f: 1)   # single-pass plan, no device plan
        bench.G.Graph.plan = lambda self, chunk=512: None
        args = types.SimpleNamespace(mode=mode, grid="auto", row_chunks=chunks, chunk_fracs="auto", n=n, e=e, blocks=0,
                                     impl="plan")
        shard, agg, m, pr, pc, n_chunks = bench.build(args, world, rank, torch.device("cpu"), "gloo", lambda s: None)
        if chunks == 0:  # bench's default: three weighted chunks in edges mode, two in rows mode
            assert n_chunks == (3 if (mode == "edges" and pc > 1) else 2)
        for _ in range(2):
            agg.step()
        g = shard.grid
        if mode == "rows":
            w_ = world * g.mk
            part = torch.cat([agg.y_full[c * w_ + rank * g.mk:c * w_ + (rank + 1) * g.mk] for c in range(g.chunks)])
            owned = torch.arange(g.chunks * g.mk) + g.r0
            owned = torch.where(owned < g.r1, owned, torch.full_like(owned, -1))
            # the gathered table holds every rank's rows at the padded positions
            full = torch.zeros(n, metric.F)
            for q_ in range(world):
                r0, r1 = shard.rcuts[q_], shard.rcuts[q_ + 1]
                rows = torch.cat([agg.y_full[c * w_ + q_ * g.mk:c * w_ + (q_ + 1) * g.mk] for c in range(g.chunks)])
                full[r0:r1] = rows[:r1 - r0]
            whole = metric.Shard(n, e, 0, 1, 1, 1, "cpu")
            ip, ix = whole.graph.numpy()
            ref = isa_ref.aggregate(ip, ix, whole.x.numpy(), "src", whole.alpha.numpy())
            gathered_err = float(np.abs(full.numpy() - ref).max())
        else:
            part, owned = agg.y_own, g.owned_rows(rank)
            gathered_err = 0.0
        ratio, err, n_rows = bench.oracle_parity(shard, part, owned, k=400)
        if mode == "edges":  # every owned row of this rank against the fp64 oracle, not a sample
            whole = metric.Shard(n, e, 0, 1, 1, 1, "cpu")
            ip, ix = whole.graph.numpy()
            ref = isa_ref.aggregate(ip, ix, whole.x.numpy(), "src", whole.alpha.numpy())
            ok = owned >= 0
            gathered_err = float(np.abs(part[ok].double().numpy() - ref[owned[ok].numpy()]).max()) if ok.any() else 0.0
        q.put((rank, (pr, pc), ratio, n_rows, gathered_err, int(shard.graph.nnz)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,mode,n,e,chunks", [(2, "edges", N, E, 2), (4, "edges", N, E, 2), (2, "rows", N, E, 2),
                                                  (3, "rows", N, E, 2), (8, "edges", N, E, 2), (8, "edges", 400, 9, 2),
                                                  (8, "edges", 8, 20, 2), (8, "edges", N, E, 0), (2, "edges", N, E, 0),
                                                  (8, "edges", 8, 20, 0)])
def test_bench_exchange_gloo(world, mode, n, e, chunks):
    """bench.py's N-rank step (gloo, oracle kernels): every rank's rows after the exchange match the
    fp64 oracle; in rows mode the gathered table is the whole Y.  World 8 runs the driver's 8-GPU
    layout, the 4 x 2 grid with one row-group sub-group per pair of ranks (distributed.row_groups),
    every rank's owned rows checked; the 9-edge graph leaves ranks with empty tiles; the 8-row graph
    gives row blocks of one row per rank, so the 70 / 30 chunking leaves an empty last chunk.  chunks = 0:
    bench's default count (three chunks of 55 / 30 / 15 % in edges mode)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, mode, q, n, e, chunks)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    out = [q.get(timeout=10) for _ in range(world)]
    for rank, grid, ratio, n_rows, gathered, nnz in out:
        assert grid == distributed.grid_shape(world, mode)
        assert ratio <= 1.0, (rank, ratio)
        assert gathered < 1e-5
    assert sum(o[5] for o in out) == (e if mode == "edges" else sum(o[5] for o in out))
    if e < world:
        assert any(o[5] == 0 for o in out)  # at least one rank held an empty tile


@pytest.mark.parametrize("pr,pc", [(1, 2), (2, 2), (4, 2)])
def test_column_counts_rebuild_a_tile_alone(pr, pc):
    """metric.column_counts (one process counting every edge's source, no process group) equals the
    all-reduced row-group histograms, so a rank's tile rebuilt alone -- bench's per-rank PMC child --
    has the same column cuts, edges and alpha as the tile the distributed run builds."""
    cc = metric.column_counts(N, E, "cpu", step=7777)
    assert torch.equal(cc * pc, _global_counts(pr, pc)(None))
    for r in range(pr * pc):
        a = metric.Shard(N, E, r, pr, pc, 2, "cpu", count_reduce=_global_counts(pr, pc), fracs=(0.7, 0.3))
        b = metric.Shard(N, E, r, pr, pc, 2, "cpu", col_counts=cc, fracs=(0.7, 0.3), keep_rows=False)
        assert (a.grid.c0, a.grid.c1) == (b.grid.c0, b.grid.c1)
        assert torch.equal(a.graph.indptr, b.graph.indptr) and torch.equal(a.graph.indices, b.graph.indices)
        assert torch.equal(a.alpha, b.alpha) and torch.equal(a.x, b.x)


@pytest.mark.parametrize("world,mode", [(8, "edges"), (4, "edges"), (2, "edges"), (4, "rows")])
def test_bench_builds_a_tile_alone_without_a_process_group(monkeypatch, world, mode):
    """bench.py's PMC child (and scripts/tile_chunks.py) rebuild one rank's tile in a process with
    no process group: bench.build with backend "none" and the whole-graph column histogram must not
    touch torch.distributed (the 4 x 2 grid's row sub-groups included), and must give the tile the
    distributed run builds."""
    import types

    import bench
    monkeypatch.setattr(bench.ops.BlockedPlan, "auto_blocks", staticmethod(lambda g, f, elem=4: 1))
    monkeypatch.setattr(bench.G.Graph, "plan", lambda self, chunk=512: None)
    assert not dist.is_initialized()
    args = types.SimpleNamespace(mode=mode, grid="auto", row_chunks=2, chunk_fracs="auto", n=N, e=E, blocks=0,
                                 impl="plan")
    cc = metric.column_counts(N, E, "cpu")
    pr, pc = distributed.grid_shape(world, mode)
    tot = 0
    for r in range(world):
        shard, agg, m, pr_, pc_, chunks = bench.build(args, world, r, torch.device("cpu"), "none", lambda s: None,
                                                      col_counts=cc)
        assert (pr_, pc_) == (pr, pc) and agg.group is None
        ref = metric.Shard(N, E, r, pr, pc, 2, "cpu", count_reduce=(_global_counts(pr, pc) if pc > 1 else None),
                           fracs=(0.7, 0.3) if (mode == "edges" and pc > 1) else None)
        if mode == "edges":
            assert torch.equal(shard.graph.indices, ref.graph.indices) and torch.equal(shard.alpha, ref.alpha)
        tot += shard.graph.nnz
    assert tot == E
