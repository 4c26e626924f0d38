"""CSR graph container and deterministic synthetic graph generators.

Layout (the reference's row-tile axis, code/preprocessing.py:26-38): CSR sorted
by DESTINATION row (direction R), `indices` = SOURCE column of each edge
(direction C).  indptr int64 [N+1], indices int32 [E]; edge tensors are [E, F]
in CSR order.  The reference holds adjacency only as a dense .npy
(code/preprocessing.py:14) or a CSR .npz it never uses (code/simulator.py:63-73);
this CSR is the device-resident form of the same matrix (rows = dst, cols = src).

Synthetic shapes: Cora N=2708/E=10556, CiteSeer 3327/9228, PubMed 19717/88648, Flickr 89250/899756,
Reddit 232965/114615892, ogbn-products 2449029/123718280.  Degrees are
lognormal (sigma 1) scaled to the exact edge count; sources are uniform
(or "locality": near the destination id).
"""
import math

import torch

SHAPES = {  # node counts as the reference hard-codes them (code/compiler.py:491-498, interpreter.py:808-815)
    "cora": (2708, 10556),
    "citeseer": (3327, 9228),    # V2/GAT_Cora.yaml's dimensions (feature_number 3327, output_number 9228)
    "pubmed": (19717, 88648),
    "flickr": (89250, 899756),
    "reddit": (232965, 114615892),
    "products": (2449029, 123718280),
}


class Graph:
    """Destination-sorted CSR.  All tensors live on one device."""

    def __init__(self, indptr, indices, n_cols=None):
        if indptr.dtype != torch.int64 or indices.dtype != torch.int32:
            raise TypeError("indptr must be int64 and indices int32")
        if indptr.device != indices.device:
            raise ValueError("indptr and indices on different devices")
        self.indptr = indptr.contiguous()
        self.indices = indices.contiguous()
        self.n_rows = indptr.numel() - 1
        self.n_cols = self.n_rows if n_cols is None else int(n_cols)
        self.nnz = indices.numel()
        self._plans = {}
        self._row_of_edge = None
        self._deg = None

    @property
    def device(self):
        return self.indptr.device

    def to(self, device):
        return Graph(self.indptr.to(device), self.indices.to(device), self.n_cols)

    def degrees(self):
        if self._deg is None:
            self._deg = (self.indptr[1:] - self.indptr[:-1])
        return self._deg

    def row_of_edge(self):
        """int32 [E]: destination row of each edge (for scatter-R gathers in edge GEMMs)."""
        if self._row_of_edge is None:
            rows = torch.arange(self.n_rows, device=self.device, dtype=torch.int32)
            self._row_of_edge = torch.repeat_interleave(rows, self.degrees())
        return self._row_of_edge

    def csc(self):
        """Cached CSC view (ops.CSC: edges ordered by source column, built on the device once)."""
        if "csc" not in self._plans:
            from . import ops
            self._plans["csc"] = ops.CSC(self)
        return self._plans["csc"]

    def plan(self, chunk=512):
        """Cached device-side aggregate plan (row chunks of <= chunk edges)."""
        if chunk not in self._plans:
            from . import ops
            self._plans[chunk] = ops.AggregatePlan(self, chunk)
        return self._plans[chunk]

    def blocked_plan(self, blocks=32, item_edges=None, row_edges=None):
        """Cached column-blocked plan (segment table over `blocks` source-column blocks, work items
        of <= item_edges edges, light rows' blocks merged toward row_edges edges per item; None =
        the ops.BlockedPlan defaults)."""
        from . import ops
        key = ("blocked", blocks, int(item_edges or ops.BlockedPlan.ITEM_EDGES),
               int(ops.BlockedPlan.ROW_EDGES if row_edges is None else row_edges))
        if key not in self._plans:
            self._plans[key] = ops.BlockedPlan(self, blocks, key[2], key[3])
        return self._plans[key]

    def numpy(self):
        return self.indptr.cpu().numpy(), self.indices.cpu().numpy()

    def __repr__(self):
        return f"Graph(N={self.n_rows}, E={self.nnz}, device={self.device})"


def from_numpy(indptr, indices, device="cpu", n_cols=None):
    return Graph(torch.as_tensor(indptr, dtype=torch.int64).to(device),
                 torch.as_tensor(indices, dtype=torch.int32).to(device), n_cols)


def lognormal_degrees(n, e, seed=0, sigma=1.0, device="cpu"):
    """Per-row degrees ~ lognormal(sigma), scaled so that sum == e exactly."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    z = torch.randn(n, generator=g, device=device, dtype=torch.float64)
    raw = torch.exp(sigma * z)
    scaled = raw * (e / raw.sum())
    deg = torch.floor(scaled).to(torch.int64)
    rem = int(e - int(deg.sum().item()))
    if rem > 0:  # hand the remainder to the rows with the largest fractional parts
        frac = scaled - deg.to(torch.float64)
        top = torch.topk(frac, rem).indices
        deg[top] += 1
    return deg


def synthetic(n, e, seed=0, kind="lognormal", sigma=1.0, device="cpu", sort_cols=True, dedupe=False,
              locality_width=None):
    """Deterministic synthetic CSR of n nodes / ~e edges.

    kind: "lognormal" (degree skew, Reddit-like) or "uniform" (equal degrees).
    locality_width: None = uniform random sources; else sources within +-width of the row.
    dedupe: drop duplicate (dst, src) pairs and self loops (then nnz <= e).
    """
    device = torch.device(device)
    if kind == "uniform":
        deg = torch.full((n,), e // n, dtype=torch.int64, device=device)
        deg[: e - int(deg.sum())] += 1
    elif kind == "lognormal":
        deg = lognormal_degrees(n, e, seed=seed, sigma=sigma, device=device)
    else:
        raise ValueError(kind)
    g = torch.Generator(device=device)
    g.manual_seed(seed + 1)
    rows = torch.repeat_interleave(torch.arange(n, device=device, dtype=torch.int64), deg)
    if locality_width is None:
        cols = torch.randint(0, n, (e,), generator=g, device=device, dtype=torch.int64)
    else:
        off = torch.randint(-locality_width, locality_width + 1, (e,), generator=g, device=device,
                            dtype=torch.int64)
        cols = torch.remainder(rows + off, n)
    if dedupe:
        keep = cols != rows
        rows, cols = rows[keep], cols[keep]
    if sort_cols or dedupe:
        key = rows * n + cols
        key = torch.unique(key) if dedupe else torch.sort(key).values
        rows = torch.div(key, n, rounding_mode="floor")
        cols = key - rows * n
        del key
    counts = torch.bincount(rows, minlength=n)
    indptr = torch.zeros(n + 1, dtype=torch.int64, device=device)
    indptr[1:] = torch.cumsum(counts, 0)
    return Graph(indptr, cols.to(torch.int32))


M32 = 0xFFFFFFFF


def _mulmod32(x, c):
    """(x * c) mod 2^32 for uint32 values held in int64 tensors, without int64 overflow."""
    lo = (x * (c & 0xFFFF)) & M32
    hi = ((x * (c >> 16)) & 0xFFFF) << 16
    return (lo + hi) & M32


def mix32(x):
    """lowbias32 integer hash of uint32 values in an int64 tensor: exact (bitwise equal) on CPU and GPU."""
    x = x & M32
    x = x ^ (x >> 16)
    x = _mulmod32(x, 0x7FEB352D)
    x = x ^ (x >> 15)
    x = _mulmod32(x, 0x846CA68B)
    return x ^ (x >> 16)


def hash32(idx, seed, stream):
    """Counter-based 32-bit hash of (seed, stream, idx) for idx < 2^32 (int64 tensor)."""
    key = mix32(torch.tensor((seed * 0x9E3779B9 + stream * 0x85EBCA6B + 0x27D4EB2F) & M32, dtype=torch.int64))
    return mix32(mix32(idx ^ int(key)) + int(stream))


def hash_normal(idx, seed, stream, dtype=torch.float32):
    """N(0, 1) values keyed by idx (Box-Muller on two counter hashes): any subset of a table can be
    generated on its own, on any device, in any order."""
    u1 = (hash32(idx, seed, 2 * stream).to(torch.float64) + 0.5) * (1.0 / 4294967296.0)
    u2 = hash32(idx, seed, 2 * stream + 1).to(torch.float64) * (1.0 / 4294967296.0)
    return (torch.sqrt(-2.0 * torch.log(u1)) * torch.cos(6.283185307179586 * u2)).to(dtype)


def lognormal_degrees_host(n, e, seed=0, sigma=1.0):
    """lognormal_degrees on the host (numpy, fp64): the same int64 [n] on every rank and device."""
    import numpy as np
    z = np.random.default_rng(seed).standard_normal(n)
    raw = np.exp(sigma * z)
    scaled = raw * (e / raw.sum())
    deg = np.floor(scaled).astype(np.int64)
    rem = int(e - int(deg.sum()))
    if rem > 0:
        frac = scaled - deg
        top = np.argsort(-frac, kind="stable")[:rem]
        deg[top] += 1
    return deg


class CounterCSR:
    """A synthetic destination-sorted CSR whose every edge is a pure function of (seed, edge id).

    Same shape model as synthetic() (lognormal degrees scaled to exactly e edges, uniform random
    sources, columns sorted within each row), but the sources come from a counter
    hash instead of a sequential generator, so a rank builds only its own rows -- and, after the
    column filter, only its own (row group x column group) tile -- with no global pass
    (multi-GPU bench, distributed.GridShard.from_rows).  Edge ids are generation order: edge e of
    row r lies in [indptr[r], indptr[r+1]); per-edge data (GAT logits) are keyed by that id, so
    sorting a row's columns moves nothing it depends on."""

    def __init__(self, n, e, seed=0, sigma=1.0):
        import numpy as np
        self.n, self.e, self.seed = int(n), int(e), int(seed)
        deg = lognormal_degrees_host(self.n, self.e, seed, sigma)
        self.indptr_np = np.zeros(self.n + 1, np.int64)
        np.cumsum(deg, out=self.indptr_np[1:])

    def indptr(self, device):
        return torch.from_numpy(self.indptr_np).to(device)

    def sources(self, e0, e1, device):
        """int64 source column of edges [e0, e1) in generation order."""
        idx = torch.arange(e0, e1, device=device, dtype=torch.int64)
        return (hash32(idx, self.seed, 1) * self.n) >> 32

    def rows(self, r0, r1, device):
        """Rows [r0, r1): (local indptr int64 [r1-r0+1], sources int64 in CSR order (sorted within
        each row), gen int64 = the generation id of each CSR edge)."""
        ip = self.indptr(device)
        e0, e1 = int(self.indptr_np[r0]), int(self.indptr_np[r1])
        src = self.sources(e0, e1, device)
        lip = (ip[r0:r1 + 1] - e0).contiguous()
        row = expand_rows(lip, e1 - e0)
        order = torch.sort(row * self.n + src, stable=True).indices  # duplicates keep generation order
        del row
        return lip, src[order].contiguous(), order + e0

    def graph(self, device):
        lip, src, _ = self.rows(0, self.n, device)
        return Graph(lip, src.to(torch.int32))


def dataset_graph(name, seed=0, device="cpu", **kw):
    n, e = SHAPES[name]
    return synthetic(n, e, seed=seed, device=device, **kw)


def gcn_norm_weights(graph):
    """w_e = 1/sqrt(d_dst * d_src) (GCN edge weight); degrees = in-degree, min 1."""
    deg = graph.degrees().to(torch.float32).clamp_min(1.0)
    dst = graph.row_of_edge().long()
    src = graph.indices.long()
    return (deg[dst] * deg[src]).rsqrt()


def mean_weights(graph):
    """SAGE-mean row scale 1/deg(i) (0-degree rows scale by 1)."""
    return 1.0 / graph.degrees().to(torch.float32).clamp_min(1.0)


def expand_rows(lip, nnz):
    """int64 [nnz]: the row of each edge of a CSR row range (lip local, from 0).  On the device this
    is libgta's one-wave-per-row gta_row_ids, not torch.repeat_interleave, whose device-wide scan
    stalled the 8-process one-GPU rehearsal; on the CPU, repeat_interleave."""
    if lip.is_cuda:
        from . import ops
        return ops.row_ids(lip, nnz)
    return torch.repeat_interleave(torch.arange(lip.numel() - 1, device=lip.device, dtype=torch.int64),
                                   lip[1:] - lip[:-1])


def ceil_div(a, b):
    return -(-a // b)


def tiles(n_rows, T):
    return math.ceil(n_rows / T)
