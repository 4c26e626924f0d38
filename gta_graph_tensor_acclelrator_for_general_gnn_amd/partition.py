"""Edge partition across GPUs + RCCL all-reduce of partial vertex aggregates.

The reference has no distributed backend; the partition unit is its column
axis j of the (T-row x 1-column) edge tiles (code/preprocessing.py:26-38,
interpreter TC = N, code/interpreter.py:828-829).  Rank p owns the edges whose
SOURCE column lies in [cut[p], cut[p+1]), cuts chosen from the prefix sum of
per-column nnz so every rank gets ~E/p edges.  Each rank keeps a destination-
sorted CSR of its edges with LOCAL column ids and only its slice of X, so its
gather table is 1/p of X.  The one exchange step is the sum of the partial
aggregates: Y = sum_p Y_p, an all-reduce (RCCL over xGMI under the "nccl"
backend), issued per destination-row chunk so it overlaps the next chunk's
aggregate.
"""
import torch

from .graph import Graph


def column_cuts(graph, world):
    """Source-column cut points [world+1] balancing nnz (prefix sum of per-column counts)."""
    return cuts_from_counts(torch.bincount(graph.indices.long(), minlength=graph.n_cols), world)


def cuts_from_counts(counts, world):
    """Cut points [world+1] of a per-column nnz histogram (the column sums of the reference's tile
    metadata, code/preprocessing.py:26-38) so every part holds ~nnz/world edges."""
    n_cols = counts.numel()
    nnz = float(counts.sum())
    csum = torch.cumsum(counts, 0)
    targets = torch.arange(1, world, device=csum.device, dtype=torch.float64) * (nnz / world)
    inner = torch.searchsorted(csum.to(torch.float64), targets, right=False) + 1
    cuts = torch.cat([torch.zeros(1, dtype=torch.int64, device=csum.device), inner.to(torch.int64),
                      torch.full((1,), n_cols, dtype=torch.int64, device=csum.device)])
    return torch.clamp(cuts, 0, n_cols).cpu()


class Shard:
    """One rank's edges: CSR over all destination rows, local source ids in [0, c1-c0)."""

    def __init__(self, graph, edge_mask, c0, c1):
        keep = edge_mask
        rows_of_edge = graph.row_of_edge()
        kept_rows = rows_of_edge[keep].long()
        counts = torch.bincount(kept_rows, minlength=graph.n_rows)
        indptr = torch.zeros(graph.n_rows + 1, dtype=torch.int64, device=graph.device)
        indptr[1:] = torch.cumsum(counts, 0)
        indices = (graph.indices[keep].long() - c0).to(torch.int32)
        self.graph = Graph(indptr, indices, n_cols=int(c1 - c0))
        self.edge_ids = torch.nonzero(keep, as_tuple=False).flatten()  # global edge id of each local edge
        self.c0, self.c1 = int(c0), int(c1)


def make_shard(graph, rank, world, cuts=None):
    cuts = column_cuts(graph, world) if cuts is None else cuts
    c0, c1 = int(cuts[rank]), int(cuts[rank + 1])
    src = graph.indices
    mask = (src >= c0) & (src < c1)
    return Shard(graph, mask, c0, c1)


def row_chunks(n_rows, n_chunks):
    step = -(-n_rows // n_chunks)
    return [(r, min(n_rows, r + step)) for r in range(0, n_rows, step)]


def sub_rows(graph, r0, r1):
    """Row-range view [r0, r1) sharing indices/edge tensors (indptr stays global)."""
    return Graph(graph.indptr[r0:r1 + 1], graph.indices, n_cols=graph.n_cols)


class ChunkedRows:
    """Destination-row chunks of a graph, each with its own (cached) aggregate plan."""

    def __init__(self, graph, n_chunks=4, chunk=512):
        self.graph = graph
        self.parts = []
        for r0, r1 in row_chunks(graph.n_rows, max(1, n_chunks)):
            g = sub_rows(graph, r0, r1) if n_chunks > 1 else graph
            plan = g.plan(chunk) if (chunk and g.device.type == "cuda") else None
            self.parts.append((r0, r1, g, plan))


def distributed_aggregate(chunked, x_local, w_local, out, group=None, aggregate_fn=None):
    """Y = sum over ranks of the shard aggregates, computed and all-reduced per row chunk.

    Each chunk's all-reduce is enqueued right after its aggregate, so RCCL moves
    chunk k while the next chunk computes.  aggregate_fn(graph, x, w, out_view,
    plan) computes one chunk (default: libgta via ops.aggregate); out holds Y."""
    import torch.distributed as dist
    if aggregate_fn is None:
        from . import ops

        def aggregate_fn(g, x, w, o, plan):
            return ops.aggregate(g, x, "src", w, out=o, plan=plan)
    multi = dist.is_initialized() and dist.get_world_size() > 1
    works = []
    for r0, r1, g, plan in chunked.parts:
        aggregate_fn(g, x_local, w_local, out[r0:r1], plan)
        if multi:
            works.append(dist.all_reduce(out[r0:r1], op=dist.ReduceOp.SUM, group=group, async_op=True))
    for wk in works:
        wk.wait()
    return out
