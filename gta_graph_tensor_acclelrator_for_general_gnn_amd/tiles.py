"""Tile-nnz metadata from a CSR on the GPU (f2): the inputs compile() and simulate() read.

Reference: preprocessing.py builds, from a DENSE adjacency .npy, the nnz of every
(T-row x 1-column) block (calculate_sparsity, code/preprocessing.py:12-40), the
largest block per T (cal_min_sparsity :53-63) and the tile-size list (gen_size
:65-72); its Reddit/Flickr variant re-blocks rows by summation
("FinalVersion For Paper/preprocessing_forReditFlickr.py":6-41).  A dense
232,965^2 matrix is 217 GB, so here the counts come straight from the CSR with
one integer-atomic histogram kernel (gta_tile_nnz); equal to the dense count for
a CSR with column-sorted rows, duplicates included (tests/test_gpu_ops.py pins it
to the reference's output).
"""
import math

import numpy as np
import torch

from . import ops
from .graph import Graph


def gen_size(start, end):
    """code/preprocessing.py:65-72."""
    size = [start]
    i = 1
    while size[-1] < end:
        i += 1
        size.append(start * i)
    return size


def tile_counts(graph, T):
    """int32 [ceil(N/T), N] nnz per (T-row block, source column)."""
    return ops.tile_nnz(graph, T)


def max_tile(graph, T, dense_limit_bytes=2 << 30):
    """Largest (T-row block, column) count.  Small tile grids use the gta_tile_nnz histogram;
    grids over dense_limit_bytes (ogbn-products at T=64 would be 375 GB) use a sort of the
    (block, column) keys of the non-self-loop edges and the longest run."""
    nt = -(-graph.n_rows // T)
    if nt * graph.n_cols * 4 <= dense_limit_bytes:
        c = ops.tile_nnz(graph, T)
        m = int(c.max().item()) if c.numel() else 0
        del c
        return max(m, 0)
    rows = graph.row_of_edge().long()
    cols = graph.indices.long()
    keep = rows != cols
    keys = torch.sort((rows[keep] // T) * graph.n_cols + cols[keep]).values
    _, counts = torch.unique_consecutive(keys, return_counts=True)
    m = int(counts.max().item()) if counts.numel() else 0
    del rows, cols, keep, keys, counts
    return m


def sparse_counts(graph, T):
    """calculate_sparsity(T, 1) of the CSR as costmodel.TileCounts: the nonzero (T-row block, source
    column) counts with the same rule as gta_tile_nnz (self loops dropped, a column that repeats
    its row's previous entry counted once), from one sort of the edges' tile keys -- O(E) memory
    instead of the [ceil(N/T), n_cols] grid.  dense() falls back to gta_tile_nnz (GPU) or a scatter
    of these counts (CPU)."""
    from .costmodel import TileCounts
    nt = -(-graph.n_rows // T)
    length = nt * graph.n_cols
    if graph.nnz == 0:
        return TileCounts(length, np.zeros(0, np.int64), 0, lambda: np.zeros(length, np.int64))
    rows = graph.row_of_edge().long()
    cols = graph.indices.long()
    keep = rows != cols
    if graph.nnz > 1:  # the previous entry of the same row repeats this column: counted once
        keep[1:] &= ~((rows[1:] == rows[:-1]) & (cols[1:] == cols[:-1]))
    keys = (rows[keep] // T) * graph.n_cols + cols[keep]
    del rows, cols, keep
    uk, counts = torch.unique(keys, return_counts=True)
    del keys
    uk, counts = uk.cpu().numpy(), counts.cpu().numpy().astype(np.int64)
    first = int(counts[0]) if uk.size and uk[0] == 0 else 0

    def dense():
        if graph.device.type == "cuda":
            return ops.tile_nnz(graph, T).flatten().cpu().numpy()
        d = np.zeros(length, np.int64)
        d[uk] = counts
        return d
    return TileCounts(length, counts, first, dense)


def metadata(graph, start=64, end=None):
    """(sizelist, maxlist) as preprocessing.py writes them for compile()."""
    end = graph.n_rows if end is None else end
    sizes = gen_size(start, end)
    maxl = [max_tile(graph, T) for T in sizes]
    torch.cuda.empty_cache()
    return sizes, maxl


def nnz_in_tiles(graph):
    """Sum of all tile counts (edges minus self loops): the edge-tile total simulate() sweeps."""
    return int(ops.tile_nnz(graph, graph.n_rows).sum().item())


# ---- the Reddit/Flickr variant ("FinalVersion For Paper/preprocessing_forReditFlickr.py") ----
REDDIT_FLICKR_FRACTION = 0.25      # slice_matrix (:10-13): the first quarter of the 16x1 tile rows
REDDIT_FLICKR_BLOCKS = [64, 128, 256, 512, 1024, 1600, 2048, 2560, 3200, 3840, 4480, 5120, 5760, 6400, 7040,
                        7680, 8192]  # process_and_save's list (:40)


def reblock(counts16, block, fraction=REDDIT_FLICKR_FRACTION):
    """preprocessing_forReditFlickr.py:10-24 on a 16x1 tile-count matrix [ceil(N/16), N]: keep the
    first int(rows * fraction) tile rows, then sum every `block` consecutive rows into one
    (ceil(kept / block) rows, float64 like the reference's np.zeros accumulator; counts are
    integers, so the sum order cannot change a value)."""
    m = np.asarray(counts16)
    keep = int(m.shape[0] * fraction)
    nr = math.ceil(keep / block)
    out = np.zeros((nr, m.shape[1]), dtype=np.float64)
    if keep:
        pad = np.zeros((nr * block, m.shape[1]), dtype=np.float64)
        pad[:keep] = m[:keep]
        out[:] = pad.reshape(nr, block, m.shape[1]).sum(axis=1)
    return out


def reddit_flickr_tiles(graph, block, fraction=REDDIT_FLICKR_FRACTION):
    """The same matrix straight from the CSR on the GPU, without the [ceil(N/16), N] 16x1 matrix:
    a 16x1 tile's count is the number of distinct (dst, src) pairs in its 16 rows, so summing
    `block` tiles is the tile count at T = 16 * block over the kept rows (the first
    16 * int(ceil(N/16) * fraction) rows): one gta_tile_nnz launch on that row range.
    float64 [ceil(kept / block), N]."""
    tiles16 = -(-graph.n_rows // 16)
    keep = int(tiles16 * fraction)
    rows = min(graph.n_rows, 16 * keep)
    if rows == 0:
        return torch.zeros(0, graph.n_cols, dtype=torch.float64, device=graph.device)
    sub = Graph(graph.indptr[:rows + 1], graph.indices[:int(graph.indptr[rows])], n_cols=graph.n_cols)
    c = ops.tile_nnz(sub, 16 * block)
    return c.to(torch.float64)
