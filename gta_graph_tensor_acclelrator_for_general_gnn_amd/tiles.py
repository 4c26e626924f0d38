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
import torch

from . import ops


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
