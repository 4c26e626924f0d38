"""Multi-GPU execution of a whole layer's instruction stream (BASELINE configs 4-5).

Partition (the reference's column axis j of its T-row x 1-column edge tiles,
code/preprocessing.py:26-38): the nodes are cut into `world` contiguous ranges
[c_p, c_{p+1}) balanced by source-column nnz (partition.column_cuts).  Rank p
  * owns the node rows of its range: every node tensor of the layer (model
    input, GEMM outputs, aggregates) is held as that [n_p, F] row block;
  * owns the edges whose SOURCE lies in its range, as a CSR over all
    destination rows with local column ids, so a scatter C / aggregate
    gathers only from its own row block.
The CSR's destination rows are laid out padded, block q at rows
[q*m, q*m + n_q) with m = max_q n_q, so a gather's partial [world*m, F]
result is exactly the input of one reduce-scatter (RCCL over xGMI under the
"nccl" backend) that hands each rank the summed rows of its own block.  This is
the one exchange step of GCN / GraphSAGE / GIN layers: half the bytes of an
all-reduce, and the next layer's scatter C reads the block the rank now owns.
A scatter R (destination side, GAT's scores) needs every row: one all-gather
of the [n_p, F] blocks.

RowShard is the other layout (the metric aggregate's default, bench.py): rank p
owns the destination rows [r_p, r_{p+1}) (nnz-balanced) with all their in-edges.
A gather lands on the rank's own rows, a destination-side scatter reads them as
they are, per-row sums (GAT's softmax) stay on one rank, so the executor keeps
its fusions; the exchange is one all-gather of each source-side table, after
the node-side GEMM that feeds it (x W, 128 columns, not x, 602).
"""
import torch
import torch.distributed as dist

from . import graph as G, ops, partition
from .graph import Graph


def row_cuts(graph, world):
    """Destination-row cut points [world+1] balancing nnz (the indptr itself is the prefix sum)."""
    ip = graph.indptr
    targets = torch.arange(1, world, device=ip.device, dtype=torch.float64) * (graph.nnz / world)
    inner = torch.searchsorted(ip[1:].to(torch.float64), targets) + 1
    return [0] + [min(int(v), graph.n_rows) for v in inner.cpu()] + [graph.n_rows]



NODE_OPS = ("scatter", "applynode")   # their external inputs are node rows
EDGE_OPS = ("applyedge", "gather")    # theirs are edge rows


def tensor_kind(key, rows, n_global, e_global, opgraph=None):
    """"w" (weights, broadcast rows: unchanged), "node" ([N, *]) or "edge" ([E, *]) for a layer
    tensor.  'ext:<op>:<slot>' inputs are classified by their op's type when the op graph is given,
    so the ambiguous N == E case (and an edge input of an applyedge op) is sliced correctly; other
    keys and calls without the op graph fall back to the row count."""
    if key.startswith("w:"):
        return "w"
    if key == "x_edge":
        return "edge"
    if opgraph is not None and key.startswith("ext:"):
        try:
            op = opgraph.ops[int(key.split(":")[1])]
        except (ValueError, IndexError):
            op = None
        if op is not None and rows not in (0, 1):
            if op.type in NODE_OPS and rows == n_global:
                return "node"
            if op.type in EDGE_OPS and rows == e_global:
                return "edge"
    if rows == e_global and rows != n_global:
        return "edge"
    if rows == n_global:
        return "node"
    return "w"

class DistShard:
    """Rank `rank`'s part of `graph` (see module docstring)."""
    local_rows = False  # gathers are partial sums over this rank's source columns

    def __init__(self, graph, rank, world, cuts=None, chunks=1):
        """chunks > 1: the padded rows are laid out chunk-major -- row j of chunk k of block q at
        k*world*mk + q*mk + j (mk = ceil(m / chunks)) -- so every chunk is a contiguous
        [world*mk, F] range holding one part per rank: one reduce-scatter per chunk, issued
        while the next chunk computes (bench.py's overlap)."""
        cuts = partition.column_cuts(graph, world) if cuts is None else torch.as_tensor(cuts)
        self.cuts = [int(c) for c in cuts]
        self.rank, self.world = rank, world
        self.c0, self.c1 = self.cuts[rank], self.cuts[rank + 1]
        self.n_local = self.c1 - self.c0
        self.m = max(self.cuts[q + 1] - self.cuts[q] for q in range(world))
        self.chunks = max(1, int(chunks))
        self.mk = -(-self.m // self.chunks)
        self.n_global, self.e_global = graph.n_rows, graph.nnz
        dev = graph.device
        src = graph.indices
        keep = (src >= self.c0) & (src < self.c1)
        rows = graph.row_of_edge().long()[keep]
        cuts_t = torch.tensor(self.cuts, device=dev, dtype=torch.int64)
        blk = torch.searchsorted(cuts_t, rows, right=True) - 1
        i = rows - cuts_t[blk]
        prow = (i // self.mk) * (world * self.mk) + blk * self.mk + i % self.mk  # monotone in rows per chunk
        n_pad = self.chunks * world * self.mk
        order = None
        if self.chunks > 1:  # rows of different chunks interleave: regroup edges by padded row (stable)
            order = torch.sort(prow, stable=True).indices
            prow = prow[order]
        counts = torch.bincount(prow, minlength=n_pad)
        indptr = torch.zeros(n_pad + 1, dtype=torch.int64, device=dev)
        indptr[1:] = torch.cumsum(counts, 0)
        local_src = (src[keep].long() - self.c0).to(torch.int32)
        self.edge_ids = torch.nonzero(keep, as_tuple=False).flatten()
        if order is not None:
            local_src, self.edge_ids = local_src[order], self.edge_ids[order]
        self.graph = Graph(indptr, local_src, n_cols=self.n_local)

    def chunk_rows(self, k):
        """Padded row range [r0, r1) of chunk k (contains one mk-row part per rank)."""
        w = self.world * self.mk
        return k * w, (k + 1) * w

    def global_rows(self, q):
        """Global row ids of rank q's reduced rows, in its [chunks*mk] output order (-1 = pad)."""
        n_q = self.cuts[q + 1] - self.cuts[q]
        j = torch.arange(self.chunks * self.mk)
        return torch.where(j < n_q, self.cuts[q] + j, torch.full_like(j, -1))

    def local_tensors(self, tensors, opgraph=None):
        """Global layer tensors -> this rank's: node tensors [N, *] -> row block, edge tensors
        [E, *] -> the shard's edges (CSR order kept), weights / broadcast rows unchanged.
        With the op graph, an 'ext:op:slot' input is classified by its op's type (tensor_kind),
        which settles N == E."""
        out = {}
        for k, t in tensors.items():
            rows = t.shape[0] if t.dim() else 0
            kind = tensor_kind(k, rows, self.n_global, self.e_global, opgraph)
            if kind == "w":
                out[k] = t
            elif kind == "edge":
                out[k] = t[self.edge_ids.to(t.device)].contiguous()
            elif kind == "node":
                out[k] = ops.pitched(t[self.c0:self.c1]) if t.dim() == 2 else t[self.c0:self.c1].contiguous()
            else:
                out[k] = t
        return out


class RowShard:
    """Rank `rank` owns destination rows [r0, r1) of `graph` (nnz-balanced cuts of the reference's
    row-tile axis, code/preprocessing.py:26-38) and all their in-edges: its CSR is the contiguous
    slice indptr[r0:r1+1], edges [e0, e1).  Node tensors are [n_p, F] row blocks, so the rank's
    gathers are complete rows and its destination-side scatters read its own block.  Source
    tables are all-gathered into the padded [world*m, F] layout (block q at rows [q*m, q*m + n_q),
    m = max n_q), so the column ids are remapped once here: column c of block q -> q*m + c - r_q.

    replicate_inputs: the layer's model inputs (node tensors handed in whole) are kept whole, in
    the padded layout, so a scatter C of one needs no exchange -- the metric's replicated X
    (bench.py); tables the layer computes are still all-gathered."""
    local_rows = True
    chunks = 1

    def __init__(self, graph, rank, world, cuts=None, replicate_inputs=True):
        self.cuts = row_cuts(graph, world) if cuts is None else [int(c) for c in cuts]
        self.rank, self.world = rank, world
        self.r0, self.r1 = self.cuts[rank], self.cuts[rank + 1]
        self.c0, self.c1 = self.r0, self.r1  # its node rows (DistShard's naming)
        self.n_local = self.r1 - self.r0
        self.m = max(1, max(self.cuts[q + 1] - self.cuts[q] for q in range(world)))
        self.n_global, self.e_global = graph.n_rows, graph.nnz
        ip = graph.indptr
        self.e0, self.e1 = int(ip[self.r0]), int(ip[self.r1])
        col = graph.indices[self.e0:self.e1].long()
        cuts_t = torch.tensor(self.cuts, device=col.device, dtype=torch.int64)
        blk = torch.searchsorted(cuts_t, col, right=True) - 1
        pcol = (blk * self.m + col - cuts_t[blk]).to(torch.int32)
        self.graph = Graph((ip[self.r0:self.r1 + 1] - ip[self.r0]).contiguous(), pcol, n_cols=world * self.m)
        self.replicate_inputs = replicate_inputs
        self.inputs_full = {}
        self._padded = {}

    def padded(self, t):
        """Global node tensor [N, *] -> the padded table layout [world*m, *] (cached per tensor)."""
        key = (id(t), t._version)  # the entry holds t, so its id stays unique (data_ptr is 0 for every empty tensor)
        hit = self._padded.get(key)
        if hit is None:
            full = (ops.node_table(self.world * self.m, t.shape[1], t.dtype, t.device) if t.dim() == 2
                    else t.new_empty(self.world * self.m, *t.shape[1:]))
            full.zero_()
            for q in range(self.world):
                a, b = self.cuts[q], self.cuts[q + 1]
                full[q * self.m: q * self.m + b - a] = t[a:b]
            hit = self._padded[key] = (t, full)
        return hit[1]

    @property
    def edge_ids(self):
        return torch.arange(self.e0, self.e1, device=self.graph.device)

    def local_tensors(self, tensors, opgraph=None):
        """Global layer tensors -> this rank's: node tensors [N, *] -> rows [r0, r1), edge tensors
        [E, *] -> edges [e0, e1), weights / broadcast rows unchanged (classified by tensor_kind)."""
        out = {}
        self.inputs_full = {}  # this layer's whole inputs only (a later layer's x is a row block)
        for k, t in tensors.items():
            rows = t.shape[0] if t.dim() else 0
            kind = tensor_kind(k, rows, self.n_global, self.e_global, opgraph)
            if kind == "w":
                out[k] = t
            elif kind == "edge":
                out[k] = t[self.e0:self.e1].contiguous()
            elif kind == "node":
                out[k] = ops.pitched(t[self.r0:self.r1]) if t.dim() == 2 else t[self.r0:self.r1].contiguous()
                self.inputs_full[k] = t
            else:
                out[k] = t
        return out


class Comm:
    """The executor's exchange hooks over torch.distributed (RCCL "nccl" or gloo).

    DistShard (source-column shards): gathers reduce-scatter (reduce_rows), dst-side scatters
    all-gather (gather_rows), source tables are local.  RowShard (destination-row shards):
    gathers and dst-side scatters are local, source tables all-gather (src_fill)."""

    def __init__(self, shard, group=None):
        self.s, self.group = shard, group
        self.on = dist.is_available() and dist.is_initialized() and shard.world > 1
        # one exchange code path for both backends: RCCL's reduce_scatter_tensor /
        # all_gather_into_tensor, which torch's gloo runs too -- so the CPU (gloo) tests execute
        # exactly the calls the 8-GPU RCCL run makes
        self.local_rows = shard.local_rows
        self.src_fill = self.src_rows if self.local_rows else None
        self.replicated_bytes = 0
        self.bytes = 0
        self._filled = {}

    @property
    def n_local(self):
        return self.s.n_local

    def reduce_rows(self, y):
        """Partial aggregate over padded rows [world*m, F] -> this rank's summed block [n_p, F]."""
        s = self.s
        if self.local_rows:  # the rank's CSR holds whole rows
            return y
        assert s.chunks == 1, "layer execution uses the one-chunk layout"
        if not self.on:
            return y[s.rank * s.m: s.rank * s.m + s.n_local]
        self.bytes += y.numel() * y.element_size()
        out = torch.empty(s.m, y.shape[1], dtype=y.dtype, device=y.device)
        dist.reduce_scatter_tensor(out, y.contiguous(), group=self.group)
        return out[:s.n_local]

    def reduce_cols(self, y):
        """A gather to the SOURCE (ISA gather DIRECTION src, ORDER C) over this rank's CSR, [n_cols, F]
        -> this rank's summed node block [n_p, F].  Column shards own their sources' every edge, so
        their sums are complete; a row shard's columns are the padded [world*m] table layout and each
        rank holds partial sums of every block: reduce-scattered like reduce_rows."""
        s = self.s
        if not self.local_rows:
            return y[:s.n_local]
        if not self.on:
            return y[s.rank * s.m: s.rank * s.m + s.n_local]
        self.bytes += y.numel() * y.element_size()
        out = torch.empty(s.m, y.shape[1], dtype=y.dtype, device=y.device)
        dist.reduce_scatter_tensor(out, y.contiguous(), group=self.group)
        return out[:s.n_local]

    def gather_rows(self, x):
        """Dst-side scatter table: column shards all-gather the blocks; row shards own the rows."""
        return x if self.local_rows else self._all_blocks(x)

    def src_rows(self, x):
        """Source-side table of a row shard: every rank's block, padded [world*m, F] (one all-gather
        per distinct tensor; the padded column ids of RowShard index it)."""
        # keyed on the tensor object: the entry holds x, so id(x) cannot be reused meanwhile.  A key on
        # data_ptr() would merge distinct zero-element tensors (data_ptr 0) on an empty shard, which
        # would then skip an all-gather its peers run (a collective mismatch)
        key = (id(x), x._version)
        hit = self._filled.get(key)
        if hit is None:
            hit = self._filled[key] = (x, self._all_blocks(x))
        return hit[1]

    def replicated(self, key):
        """A getter of the whole padded table of model input `key` when the row shard keeps inputs
        replicated (None: all-gather it like any other table)."""
        s = self.s
        if not (self.local_rows and s.replicate_inputs) or key not in s.inputs_full:
            return None
        t = s.inputs_full[key]

        def get():
            full = s.padded(t)
            self.replicated_bytes = max(self.replicated_bytes, full.numel() * full.element_size())
            return full
        return get

    def _all_blocks(self, x):
        """This rank's block [n_p, F] -> every block, padded: [world*m, F]."""
        s = self.s
        buf = torch.zeros(s.m, x.shape[1], dtype=x.dtype, device=x.device)
        buf[:s.n_local] = x
        if not self.on:
            full = torch.zeros(s.world * s.m, x.shape[1], dtype=x.dtype, device=x.device)
            full[s.rank * s.m:(s.rank + 1) * s.m] = buf
            return full
        self.bytes += buf.numel() * buf.element_size() * s.world
        full = torch.empty(s.world * s.m, x.shape[1], dtype=x.dtype, device=x.device)
        dist.all_gather_into_tensor(full, buf, group=self.group)
        return full

    def full_rows(self, x):
        """[n_p, F] blocks of every rank -> the unpadded global [N, F] (for results/tests)."""
        s = self.s
        full = self._all_blocks(x)
        return torch.cat([full[q * s.m: q * s.m + s.cuts[q + 1] - s.cuts[q]] for q in range(s.world)])


def run_stream(opgraph, stream, shard, tensors, semantics=None, group=None, plan_chunk=512):
    """Execute one layer's stream on this rank's shard; returns (ExecResult, Executor).
    `tensors` are the GLOBAL layer tensors (sliced here); outputs are this rank's row blocks."""
    import time

    from . import executor
    comm = Comm(shard, group)
    ex = executor.Executor(opgraph, stream, shard.graph, shard.local_tensors(tensors, opgraph), semantics, plan_chunk,
                           dist=comm)
    cuda = shard.graph.device.type == "cuda"
    if cuda:
        torch.cuda.synchronize(shard.graph.device)
    t0 = time.perf_counter()
    outputs = ex.run()
    if cuda:
        torch.cuda.synchronize(shard.graph.device)
    res = executor.ExecResult(ex.values, outputs, time.perf_counter() - t0, ex.alg_bytes, ex.launches)
    return res, ex


def layer_record(name, dev, rank, world, reps=3, backend=None, check=True):
    """One BASELINE config (configs.CONFIGS) forward on this rank's destination-row shard (RowShard,
    replicated model inputs), timed over `reps` forwards after one warm-up: barrier + device sync
    around each, the max over ranks.  With check, rank 0 re-assembles the output rows and compares
    them with a one-device execution of the same stream on the same inputs (max |d| / max |ref|).
    -> the record bench.py's "layers" field and scripts/dist_layers.py print (every rank gets it)."""
    import time

    from . import configs, executor
    layers, g, tensors = configs.build(name, dev)
    shard = RowShard(g, rank, world) if world > 1 else None
    times, comm_bytes = [], 0
    x = ex = None
    # two untimed forwards: on one GPU a layer's HIP graph is captured on its second call
    # and a later layer's inputs only stabilise once the layer before it replays, so by the third
    # forward every layer replays its graph; the N > 1 path runs eagerly (the exchange hooks)
    warm = 2
    for r in range(reps + warm):
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        x = None
        for lay, t in zip(layers, tensors):
            t = dict(t)
            if x is not None:
                t["x"] = x
            if world > 1:
                res, ex = run_stream(lay.opgraph, lay.stream, shard, t, lay.sem)
                if r == 0:
                    comm_bytes += ex.dist.bytes
            else:
                res, ex = executor.run_stream(lay.opgraph, lay.stream, g, t, lay.sem, sync=False)
            x = res.outputs[sorted(res.outputs)[-1]]
        torch.cuda.synchronize(dev)
        dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64,
                          device=dev if backend in (None, "nccl") else "cpu")
        if world > 1:
            dist.all_reduce(dt, op=dist.ReduceOp.MAX)
        if r >= warm:
            times.append(float(dt))
    err = None
    if world > 1 and check:
        full = ex.dist.full_rows(x)
        if rank == 0:
            y = None
            for lay, t in zip(layers, tensors):
                t = dict(t)
                if y is not None:
                    t["x"] = y
                r1, _ = executor.run_stream(lay.opgraph, lay.stream, g, t, lay.sem)
                y = r1.outputs[sorted(r1.outputs)[-1]]
            fin = torch.isfinite(y)
            err = float(((full - y).abs()[fin]).max() / (y.abs()[fin].max() + 1e-30))
    ms = 1e3 * sorted(times)[len(times) // 2]
    rec = {"config": name, "n_gpus": world, "N": g.n_rows, "E": g.nnz, "layers": [l.layer for l in layers],
           "shard_edges": shard.graph.nnz if shard is not None else g.nnz, "ms_per_forward": ms,
           "edges_per_s": g.nnz * len(layers) / (ms / 1e3), "exchanged_bytes_per_rank": comm_bytes,
           "layout": "destination-row shards, replicated model inputs, all-gathered computed tables" if world > 1
           else "one GPU", "max_norm_diff_vs_1dev": err,
           "timing": (f"median of {reps} forwards after {warm} untimed: "
                      + ("every layer a HIP-graph replay" if world == 1 and executor.AUTO_GRAPH
                         else "eager launches (exchange hooks)"))}
    del layers, g, tensors, shard, ex, x
    torch.cuda.empty_cache()
    return rec


def grid_shape(world, mode="edges"):
    """Default rank grid (row groups pr x column groups pc) of the metric aggregate.

    mode "edges" (the north-star form, bench.py's default): an edge partition of the reference's
    T-row x column tiles (code/preprocessing.py:26-38) whose partial vertex aggregates are summed
    over xGMI by RCCL -- 1x2, 2x2, 4x2, 4x4 ...: pc = 2 column groups once world >= 4 keeps the
    reduce-scatter between pairs of GPUs (15 MB per rank at 8 GPUs on Reddit), pc = world below.
    mode "rows": destination-row tiles (pc = 1), whose outputs are complete rows (the exchange
    is then the all-gather of Y for the next layer)."""
    if mode == "rows" or world == 1:
        return world, 1
    if world < 4:
        return 1, world
    pc = 2 if world <= 8 else 4
    while world % pc:
        pc //= 2
    return world // pc, pc


def row_cuts_ip(indptr, world):
    """Destination-row cut points [world+1] balancing nnz, from an indptr tensor alone."""
    ip = indptr
    n = ip.numel() - 1
    nnz = int(ip[-1])
    targets = torch.arange(1, world, device=ip.device, dtype=torch.float64) * (nnz / world)
    inner = torch.searchsorted(ip[1:].to(torch.float64), targets) + 1
    return [0] + [min(int(v), n) for v in inner.cpu()] + [n]


class GridShard:
    """Rank r = i*pc + j of a pr x pc grid owns the edges whose destination lies in row block i
    (nnz-balanced row cuts) and whose source lies in column block j (nnz-balanced column cuts),
    as a CSR over row block i's rows with local column ids.  The pc ranks of row group i sum their
    partial aggregates with one reduce-scatter: rank (i, j) ends with rows
    R_i + j*m .. R_i + (j+1)*m of the block (m = ceil(n_i / pc); the CSR is padded to pc*m rows).

    chunks = C > 1 lays the padded rows out chunk-major so the exchange can overlap the compute.
    Chunk c covers rows [off_c, off_c+1) of each rank's block (mk_c = off_c+1 - off_c): row
    R_i + j*m + off_c + v sits at padded row pc*off_c + j*mk_c + v, so chunk c is the contiguous
    [pc*mk_c] range holding one mk_c-row part per rank of the group -- one reduce-scatter per
    chunk, issued while chunk c+1 aggregates.  Rank j's output is then [off_C] rows, part c at
    off_c (owned_rows gives their global ids).  Equal chunks (fracs None): off_c = c*mk with
    mk = ceil(m / C) (the last part padded).  fracs (C weights): chunk sizes in that proportion, so
    a smaller last chunk leaves less exchange exposed after the last launch.

    Built from a whole graph (GridShard(graph, ...)) or from the rank's row group alone
    (GridShard.from_rows: the multi-GPU bench, where no rank holds the whole graph)."""

    def __init__(self, graph, rank, pr, pc, chunks=1, fracs=None):
        ip = graph.indptr
        rcuts = row_cuts_ip(ip, pr)
        ccuts = [int(c) for c in partition.column_cuts(graph, pc)]
        i = rank // pc
        r0, r1 = rcuts[i], rcuts[i + 1]
        e0, e1 = int(ip[r0]), int(ip[r1])
        self._build(rcuts, ccuts, rank, pr, pc, chunks, (ip[r0:r1 + 1] - e0).contiguous(),
                    graph.indices[e0:e1].long(), e0, fracs)

    @classmethod
    def from_rows(cls, rcuts, ccuts, rank, pr, pc, row_indptr, row_src, chunks=1, e0=0, fracs=None):
        """The shard from its row group only: row_indptr [n_i + 1] (local, from 0) and row_src (int64
        source column of each of the group's edges, columns sorted within rows); e0 = the group's
        first global edge id (edge_ids are global CSR ids, local_edge_ids index the group's edges)."""
        self = cls.__new__(cls)
        self._build(list(rcuts), list(ccuts), rank, pr, pc, chunks, row_indptr, row_src, e0, fracs)
        return self

    @staticmethod
    def chunk_offsets(m, chunks, fracs=None):
        """[off_0 = 0, ..., off_C] of a block of m rows: equal chunks of ceil(m / C) (the last
        padded past m), or sizes in proportion to fracs (sum = m, every chunk >= 1 row when m >= C)."""
        if chunks <= 1:
            return [0, m]
        if fracs is None:
            mk = -(-m // chunks)
            return [c * mk for c in range(chunks + 1)]
        if len(fracs) != chunks or min(fracs) <= 0:
            raise ValueError(f"fracs must be {chunks} positive weights")
        tot, acc, offs = float(sum(fracs)), 0.0, [0]
        for c in range(chunks - 1):
            acc += fracs[c]
            offs.append(min(max(offs[-1] + (1 if m >= chunks else 0), int(round(m * acc / tot))),
                            m - (chunks - 1 - c if m >= chunks else 0)))
        return offs + [m]

    def _build(self, rcuts, ccuts, rank, pr, pc, chunks, lip, src, e0, fracs=None):
        self.pr, self.pc, self.rank = pr, pc, rank
        self.i, self.j = divmod(rank, pc)
        self.rcuts, self.ccuts = rcuts, ccuts
        dev = lip.device
        r0, r1 = rcuts[self.i], rcuts[self.i + 1]
        c0, c1 = ccuts[self.j], ccuts[self.j + 1]
        self.r0, self.r1, self.c0, self.c1 = r0, r1, c0, c1
        self.m = max(1, -(-(r1 - r0) // pc))
        self.chunks = max(1, int(chunks))
        self.fracs = None if fracs is None or self.chunks == 1 else list(fracs)
        self.offs = self.chunk_offsets(self.m, self.chunks, self.fracs)
        self.mks = [b - a for a, b in zip(self.offs[:-1], self.offs[1:])]
        self.mk = -(-self.m // self.chunks)  # the equal-chunk size (rows mode pads every rank's chunks to it)
        keep = (src >= c0) & (src < c1)
        rows = G.expand_rows(lip, src.numel())[keep]
        local_src = (src[keep] - c0).to(torch.int32)
        self.local_edge_ids = torch.nonzero(keep, as_tuple=False).flatten()
        if self.chunks > 1:  # chunk-major padded rows; a stable sort keeps each row's edge order
            jj, u = rows // self.m, rows % self.m
            offs = torch.tensor(self.offs, device=dev)
            c = torch.searchsorted(offs, u, right=True) - 1
            rows = pc * offs[c] + jj * (offs[c + 1] - offs[c]) + (u - offs[c])
            order = torch.sort(rows, stable=True).indices
            rows, local_src, self.local_edge_ids = rows[order], local_src[order], self.local_edge_ids[order]
        self.edge_ids = self.local_edge_ids + e0
        n_pad = pc * self.offs[-1]
        counts = torch.bincount(rows, minlength=n_pad)
        indptr = torch.zeros(n_pad + 1, dtype=torch.int64, device=dev)
        indptr[1:] = torch.cumsum(counts, 0)
        self.graph = Graph(indptr, local_src, n_cols=c1 - c0)

    def chunk_rows(self, c):
        """Padded row range [a, b) of chunk c: the input of its reduce-scatter."""
        return self.pc * self.offs[c], self.pc * self.offs[c + 1]

    def part(self, c):
        """Row range [a, b) of chunk c inside this rank's reduce-scatter output."""
        return self.offs[c], self.offs[c + 1]

    def out_rows(self):
        """Rows of this rank's reduce-scatter output (off_C: = m when chunks == 1)."""
        return self.offs[-1]

    def owned_rows(self, rank):
        """Global row ids of `rank`'s reduce-scatter output ([out_rows] rows; -1 = padding)."""
        i, j = divmod(rank, self.pc)
        r0, r1 = self.rcuts[i], self.rcuts[i + 1]
        m = max(1, -(-(r1 - r0) // self.pc))
        u = torch.arange(self.chunk_offsets(m, self.chunks, self.fracs)[-1])
        t = r0 + j * m + u
        return torch.where((u < m) & (t < r1), t, torch.full_like(t, -1))


def row_groups(pr, pc):
    """torch.distributed groups of the pc ranks of each row (every rank must create all of them)."""
    return [dist.new_group(list(range(i * pc, (i + 1) * pc))) for i in range(pr)]
