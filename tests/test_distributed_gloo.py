"""Multi-process (gloo) execution of whole golden layer streams on node-range shards.

Each rank runs the executor over its edge shard (distributed.py) with the
oracle-backed stand-in kernels (tests/fake_ops.py; no GPU here): gathers are
exchanged as partial aggregates (all-reduce under gloo, reduce-scatter under
RCCL) and dst-side scatters all-gather their node rows.  The row blocks of
every sink output, put back together, must equal the single-device fp64
oracle (oracle/exec_ref.py) on the same Cora-shaped graph.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

STREAMS = [(net, r) for net in ("GCN", "SGC", "GraphSAGE", "GIN", "GAT", "DGN", "PNA") for r in (False, True)
           if (net, r) != ("GCN", True)]  # the reference emits no GCN-trans stream


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, golden_dir, q, layout="cols", nets=None):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import json

        from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed, executor, graph as G, ir, workloads
        from gta_graph_tensor_acclelrator_for_general_gnn_amd.semantics import Semantics
        from oracle.exec_ref import execute_ref
        from tests import fake_ops
        from tests.test_ir_executor_cpu import compare
        executor.ops = fake_ops
        man = json.load(open(os.path.join(golden_dir, "manifest.json")))
        z = np.load(os.path.join(golden_dir, "cora_graph.npz"))
        ip, ix = z["indptr"], z["indices"]
        g = G.from_numpy(ip, ix)
        report = []
        if nets is None:
            recs = [[s for s in man["streams"] if "file" in s and s["dataset"] == "cora" and s["network"] == net
                     and s["reorder"] == reorder][0] for net, reorder in STREAMS]
        else:  # every golden stream of these networks (the round-5 ORDER-C gathers: all their fusions)
            recs = [s for s in man["streams"] if "file" in s and s["network"] in nets]
        for rec in recs:
            net, reorder = rec["network"], rec["reorder"]
            sem = Semantics.for_network(net, reorder)
            og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
            st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
            tensors = workloads.make_tensors(og, g, net, seed=3)
            if layout == "cols":
                shard = distributed.DistShard(g, rank, world)
            elif layout == "rows-empty":  # rank 1 owns no row; every source table is all-gathered
                cuts = [0, g.n_rows // 2, g.n_rows // 2] + [g.n_rows] * (world - 2)
                shard = distributed.RowShard(g, rank, world, cuts=cuts, replicate_inputs=False)
            else:  # "rows": model inputs replicated; "rows-allgather": every source table exchanged
                shard = distributed.RowShard(g, rank, world, replicate_inputs=layout == "rows")
            res, ex = distributed.run_stream(og, st, shard, tensors, sem)
            full = {k: ex.dist.full_rows(v) for k, v in res.outputs.items()}
            nnz = torch.tensor([shard.graph.nnz])
            dist.all_reduce(nnz)
            if rank == 0:
                ref = execute_ref(og, sem, ip, ix, {k: v.double().numpy() for k, v in tensors.items()})
                compare(full, ref, full.keys(), rtol=1e-4)
                assert int(nnz) == g.nnz
                report.append((rec["file"], ex.dist.bytes + ex.dist.replicated_bytes))
        if rank == 0:
            q.put(("ok", report))
    except Exception as e:  # report to the parent instead of hanging the other rank
        q.put(("fail", f"rank {rank}: {type(e).__name__}: {e}"))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,layout", [(2, "cols"), (3, "cols"), (2, "rows"), (3, "rows"), (2, "rows-allgather"),
                                          (3, "rows-empty")])
def test_layer_streams_distributed_gloo(golden_dir, world, layout):
    """layout "cols": source-column shards (reduce-scatter per gather); "rows": destination-row
    shards (all-gather per source table, fusions on); "rows-empty": a live group in which rank 1
    owns no row (repeated cut), so its distinct same-width source tables are all zero-element --
    each must still join every all-gather its peers run, and the values must match the oracle."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, golden_dir, q, layout)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    status, info = q.get(timeout=10)
    assert status == "ok", info
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert len(info) == len(STREAMS) and all(b > 0 for _, b in info)


GATHER_C_NETS = ("GCNT", "BIDIR", "EDGEC")


@pytest.mark.parametrize("world,layout", [(2, "cols"), (4, "cols"), (2, "rows"), (4, "rows-allgather"), (3, "rows-empty")])
def test_gather_c_streams_distributed_gloo(golden_dir, world, layout):
    """the ORDER-C gather exchange (distributed.Comm.reduce_cols: a reduce-scatter of the
    padded [world * m] column table for row shards, the unreduced y[:n_local] slice for column
    shards) on every reference-lowered gather-C golden stream (GCNT = the transposed GCN aggregate,
    BIDIR = in + out sums, EDGEC = an SF edge tensor gathered to its source; 22 streams, every
    fusion partition the reference emitted), world 2 / 3 / 4, both shard layouts; the re-assembled
    sink outputs equal the single-device fp64 oracle."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, golden_dir, q, layout, GATHER_C_NETS))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    status, info = q.get(timeout=10)
    assert status == "ok", info
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert len(info) == 22 and all(b > 0 for _, b in info), info


def test_row_shard_layout_single_process():
    """Row shards: contiguous CSR slices with padded column ids; the padded table gathers back to x."""
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed, graph as G
    g = G.synthetic(1000, 20000, seed=2)
    world = 3
    ip, ix = g.numpy()
    x = torch.randn(g.n_rows, 5)
    shards = [distributed.RowShard(g, r, world) for r in range(world)]
    m = shards[0].m
    full = torch.zeros(world * m, 5)
    for s in shards:
        full[s.rank * m: s.rank * m + s.n_local] = x[s.r0:s.r1]
    assert [s.r0 for s in shards] + [shards[-1].r1] == shards[0].cuts and shards[-1].r1 == g.n_rows
    for s in shards:
        sip, six = s.graph.numpy()
        assert s.graph.n_rows == s.n_local and s.graph.n_cols == world * m
        np.testing.assert_array_equal(sip, ip[s.r0:s.r1 + 1] - ip[s.r0])
        # every padded column id reads the global source row
        torch.testing.assert_close(full[torch.as_tensor(six).long()], x[torch.as_tensor(ix[s.e0:s.e1]).long()])
        same_row = np.diff(np.repeat(np.arange(s.n_local), np.diff(sip))) == 0
        assert np.all(np.diff(six.astype(np.int64))[same_row] >= 0)  # the remap keeps rows sorted
    assert sum(s.e1 - s.e0 for s in shards) == g.nnz
    # nnz balance: no shard holds more than its share plus one row
    assert max(s.e1 - s.e0 for s in shards) <= g.nnz / world + int(np.diff(ip).max())


def test_row_shards_with_empty_ranks(golden_dir):
    """More ranks than rows: the empty row shards run every network's stream (no process group;
    tests/fake_ops kernels) and return [0, F] blocks."""
    import json

    from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed, executor, graph as G, ir, workloads
    from gta_graph_tensor_acclelrator_for_general_gnn_amd.semantics import Semantics
    from tests import fake_ops
    old_ops, executor.ops = executor.ops, fake_ops
    try:
        man = json.load(open(os.path.join(golden_dir, "manifest.json")))
        g = G.from_numpy(np.array([0, 2, 2, 5]), np.array([1, 2, 0, 1, 2], dtype=np.int32))
        for net, reorder in STREAMS:
            rec = [s for s in man["streams"] if "file" in s and s["dataset"] == "cora" and s["network"] == net
                   and s["reorder"] == reorder][0]
            sem = Semantics.for_network(net, reorder)
            og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
            st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
            tensors = workloads.make_tensors(og, g, net, seed=3)
            for r in range(5):
                shard = distributed.RowShard(g, r, 5)
                res, _ = distributed.run_stream(og, st, shard, tensors, sem)
                assert all(v.shape[0] == shard.n_local for v in res.outputs.values()), (net, reorder, r)
    finally:
        executor.ops = old_ops


def test_shard_layout_single_process():
    """Padded destination rows, local column ids, and the edge set partition (no process group)."""
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed, graph as G
    g = G.synthetic(1000, 20000, seed=2)
    world = 3
    total = 0
    ip, ix = g.numpy()
    for r in range(world):
        s = distributed.DistShard(g, r, world)
        sip, six = s.graph.numpy()
        assert s.graph.n_rows == world * s.m and s.graph.n_cols == s.n_local
        assert six.min() >= 0 and six.max() < s.n_local
        eids = s.edge_ids.numpy()
        assert np.all(np.diff(eids) > 0)  # CSR order kept
        np.testing.assert_array_equal(ix[eids] - s.c0, six)
        rows = np.repeat(np.arange(len(ip) - 1), np.diff(ip))[eids]
        blk = np.searchsorted(np.array(s.cuts), rows, side="right") - 1
        prow = blk * s.m + rows - np.array(s.cuts)[blk]
        np.testing.assert_array_equal(np.repeat(np.arange(world * s.m), np.diff(sip)), prow)
        total += len(eids)
    assert total == g.nnz


@pytest.mark.parametrize("world,chunks", [(3, 4), (2, 1), (4, 3), (8, 8)])
def test_chunk_major_shard_layout(world, chunks):
    """bench.py's reduce-scatter layout: padded row k*W*mk + q*mk + j holds global row
    cuts[q] + k*mk + j; every chunk is one contiguous range with one part per rank; edges keep
    their CSR order; global_rows() inverts the map for each rank's reduced rows."""
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed, graph as G
    g = G.synthetic(1000, 20000, seed=2)
    ip, ix = g.numpy()
    rows_of = np.repeat(np.arange(len(ip) - 1), np.diff(ip))
    total = 0
    for r in range(world):
        s = distributed.DistShard(g, r, world, chunks=chunks)
        sip, six = s.graph.numpy()
        assert s.graph.n_rows == chunks * world * s.mk
        prow = np.repeat(np.arange(len(sip) - 1), np.diff(sip))
        k, rem = prow // (world * s.mk), prow % (world * s.mk)
        q, j = rem // s.mk, rem % s.mk
        eids = s.edge_ids.numpy()
        np.testing.assert_array_equal(np.array(s.cuts)[q] + k * s.mk + j, rows_of[eids])
        np.testing.assert_array_equal(ix[eids] - s.c0, six)
        for a, b in zip(sip[:-1], sip[1:]):
            assert np.all(np.diff(eids[a:b]) > 0)
        gr = s.global_rows(r).numpy()
        own = gr[gr >= 0]
        np.testing.assert_array_equal(own, np.arange(s.c0, s.c1))
        total += len(eids)
    assert total == g.nnz


def _grid_worker(rank, world, pr, pc, port, q, chunks=1):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed, graph as G
        from oracle import isa_ref
        g = G.synthetic(600, 12000, seed=8)
        gen = torch.Generator().manual_seed(3)
        x = torch.randn(600, 16, generator=gen)
        w = torch.rand(g.nnz, 4, generator=gen)
        s = distributed.GridShard(g, rank, pr, pc, chunks=chunks)
        groups = distributed.row_groups(pr, pc)
        sip, six = s.graph.numpy()
        y = torch.from_numpy(isa_ref.aggregate(sip, six, x[s.c0:s.c1].numpy(), "src",
                                               w[s.edge_ids].numpy()).astype(np.float32))
        own = []
        for c in range(s.chunks):  # one reduce-scatter per chunk (gloo stand-in: all-reduce + slice)
            a, b = s.chunk_rows(c)
            yc = y[a:b].contiguous()
            dist.all_reduce(yc, group=groups[s.i])
            own.append(yc[s.j * s.mk:(s.j + 1) * s.mk])
        own = torch.cat(own)
        assert own.shape[0] == s.out_rows()
        mmax = max(len(s.owned_rows(r)) for r in range(world))
        mine = torch.zeros(mmax, 16)
        mine[:own.shape[0]] = own
        parts = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(parts, mine)
        if rank == 0:
            full = np.zeros((600, 16))
            for r in range(world):
                rows = s.owned_rows(r).numpy()
                ok = rows >= 0
                full[rows[ok]] = parts[r][:len(rows)][ok].numpy()
            ip, ix = g.numpy()
            ref = isa_ref.aggregate(ip, ix, x.numpy(), "src", w.numpy())
            q.put(float(np.abs(full - ref).max() / np.abs(ref).max()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("pr,pc,chunks", [(2, 2, 1), (1, 2, 1), (3, 1, 1), (2, 2, 3), (1, 2, 2)])
def test_grid_tiles_reduce_scatter_gloo(pr, pc, chunks):
    """bench.py's 2-D layout: row-group partial sums (one reduce-scatter, or one per chunk of the
    chunk-major padded rows), reassembled from every rank's owned rows, equal the single-device
    aggregate."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = pr * pc
    procs = [ctx.Process(target=_grid_worker, args=(r, world, pr, pc, port, q, chunks)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=10) < 1e-5


def test_row_tile_grid_covers_every_edge_once():
    """--mode rows: N destination-row tiles (a 1-column grid) cover every edge exactly once and each
    rank owns its rows."""
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed, graph as G
    g = G.synthetic(500, 9000, seed=4)
    for world in (1, 2, 4, 8):
        assert distributed.grid_shape(world, "rows") == (world, 1)
        shards = [distributed.GridShard(g, r, world, 1) for r in range(world)]
        assert sum(s.graph.nnz for s in shards) == g.nnz
        owned = torch.cat([s.owned_rows(r) for r, s in enumerate(shards)])
        assert torch.equal(torch.sort(owned[owned >= 0]).values, torch.arange(g.n_rows))


def _src_rows_worker(rank, world, port, q):
    import datetime
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=datetime.timedelta(seconds=30))
    try:
        from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed, graph as G
        g = G.synthetic(12, 60, seed=4)
        cuts = [0, 6, 6, 12]  # rank 1 owns no row
        shard = distributed.RowShard(g, rank, world, cuts=cuts, replicate_inputs=False)
        comm = distributed.Comm(shard)
        assert comm.on
        tabs = [torch.arange(g.n_rows * 4, dtype=torch.float32).view(g.n_rows, 4) * (t + 1) for t in range(3)]
        for t, full_t in enumerate(tabs):  # three distinct same-width tables; rank 1's blocks are all [0, 4]
            mine = full_t[shard.r0:shard.r1].clone()
            got = comm.src_rows(mine)
            for qq in range(world):
                a, b = cuts[qq], cuts[qq + 1]
                torch.testing.assert_close(got[qq * shard.m: qq * shard.m + b - a], full_t[a:b])
            assert comm.src_rows(mine) is got  # a repeated table is not exchanged again
        q.put(("ok", rank))
    except Exception as e:
        q.put(("fail", f"rank {rank}: {type(e).__name__}: {e}"))
        raise
    finally:
        dist.destroy_process_group()


def test_src_rows_distinct_tables_on_an_empty_rank():
    """Comm.src_rows' cache must tell distinct zero-element blocks apart (their
    data_ptr is 0), or the empty rank skips an all-gather its peers run."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_src_rows_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    res = [q.get(timeout=10) for _ in range(3)]
    assert all(s == "ok" for s, _ in res), res
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_tensor_kind_uses_the_op_type_when_n_equals_e():
    """with N == E the row count cannot tell node from edge inputs; the op graph can."""
    from types import SimpleNamespace as NS

    from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed, graph as G
    og = NS(ops=[NS(type="scatter"), NS(type="applyedge"), NS(type="gather"), NS(type="applynode")])
    kind = lambda k, rows: distributed.tensor_kind(k, rows, 10, 10, og)  # noqa: E731
    assert [kind(f"ext:{i}:1", 10) for i in range(4)] == ["node", "edge", "edge", "node"]
    assert kind("x_edge", 10) == "edge" and kind("w:3", 10) == "w" and kind("ext:1:1", 1) == "w"
    assert distributed.tensor_kind("ext:1:1", 10, 10, 10) == "node"  # without the op graph: row count
    # a RowShard slices an applyedge input of an N == E graph as edges [e0, e1)
    ip = np.array([0, 0, 0, 3, 3, 4, 5, 5, 8, 9, 10])
    g = G.from_numpy(ip, np.arange(10, dtype=np.int32) % 10)
    s = distributed.RowShard(g, 1, 2)
    t = torch.arange(10, dtype=torch.float32).view(10, 1)
    out = s.local_tensors({"ext:1:1": t, "ext:0:0": t}, og)
    torch.testing.assert_close(out["ext:1:1"], t[s.e0:s.e1])
    torch.testing.assert_close(out["ext:0:0"], t[s.r0:s.r1])
