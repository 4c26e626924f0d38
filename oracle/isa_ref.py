"""fp64 NumPy restatement of GTA ISA op semantics (TEST ORACLE ONLY, see oracle/__init__.py).

Graph convention: CSR sorted by destination row (indptr [N+1], indices [E] =
source column); edge e of row i.  Each function cites the reference construct
it restates.
"""
import numpy as np


def row_of_edge(indptr):
    return np.repeat(np.arange(len(indptr) - 1, dtype=np.int64), np.diff(indptr))


def _bcast(t, width):
    """Head broadcast of the narrower operand: column c uses t[:, c // (width // t.shape[1])]."""
    if t.shape[1] == width:
        return t
    g = width // t.shape[1]
    assert g * t.shape[1] == width, "widths must divide"
    return np.repeat(t, g, axis=1)


def edge_operand(indptr, indices, t, mode):
    """Rows of an edge operand: "edge" = t itself [E,F]; "src" = t[indices] (scatter C);
    "dst" = t[row(e)] (scatter R).  ISA scatter, template/ISA_defination.yaml:33-44."""
    if mode == "edge":
        return t
    if mode == "src":
        return t[np.asarray(indices, dtype=np.int64)]
    return t[row_of_edge(indptr)]


def scatter(indptr, indices, x, direction):
    """ISA `scatter` DIRECTION dst/src (template/ISA_defination.yaml:33-44):
    R -> edge gets its destination row's feature, C -> its source column's."""
    return edge_operand(indptr, indices, x, "dst" if direction == "R" else "src").copy()


def gather_add(indptr, xe, direction="R", indices=None, n_cols=None):
    """ISA `gather` with COMPUTE mul: add (template/ISA_defination.yaml:46-61), DIRECTION dst/src
    (:48): "R" sums each edge row into its destination row (y [N]), "C" into its source column
    (y [n_cols], "from edges to src (column-wise)"; needs indices, n_cols defaults to N)."""
    if direction == "R":
        out = np.zeros((len(indptr) - 1, xe.shape[1]), dtype=np.float64)
        np.add.at(out, row_of_edge(indptr), xe.astype(np.float64))
        return out
    if direction != "C" or indices is None:
        raise ValueError("gather_add: direction 'R', or 'C' with indices")
    n = len(indptr) - 1 if n_cols is None else n_cols
    out = np.zeros((n, xe.shape[1]), dtype=np.float64)
    np.add.at(out, np.asarray(indices, dtype=np.int64), xe.astype(np.float64))
    return out


def sf(kind, v):
    """SF special functions (the build's choices; the reference never defines them)."""
    v = np.asarray(v, dtype=np.float64)
    if kind in (None, "NONE"):
        return v
    if kind == "RELU":
        return np.maximum(v, 0.0)
    if kind == "EXP_LEAKY_RELU":
        return np.exp(np.where(v > 0, v, 0.2 * v))
    if kind == "ELU":
        return np.where(v > 0, v, np.expm1(v))
    if kind == "EXP":
        return np.exp(v)
    if kind == "LEAKY_RELU":
        return np.where(v > 0, v, 0.2 * v)
    if kind == "SIGMOID":
        return 1.0 / (1.0 + np.exp(-v))
    if kind == "TANH":
        return np.tanh(v)
    if kind == "RECIP":
        return 1.0 / v
    raise ValueError(kind)


def binop(kind, a, b):
    if kind in (None, "NONE") or b is None:
        return a
    width = max(a.shape[1], b.shape[1])
    a, b = _bcast(a, width), _bcast(b, width)
    if kind == "ADD":
        return a + b
    if kind == "MUL":
        return a * b
    if kind == "DIV":
        with np.errstate(divide="ignore", invalid="ignore"):  # 0/0 at isolated nodes (GAT-trans op 11) is expected
            return a / b
    if kind == "SUB":
        return a - b
    raise ValueError(kind)


def apply_edge(indptr, indices, bin_kind, sf_kind, a, a_mode="edge", b=None, b_mode="edge", b_broadcast_row=False):
    """applyedge element-wise (genGraphOP.py:36, 55-60) with head broadcast."""
    A = edge_operand(indptr, indices, np.asarray(a, np.float64), a_mode)
    B = None
    if b is not None:
        b = np.asarray(b, np.float64)
        B = np.broadcast_to(b[:1], (A.shape[0], b.shape[1])) if b_broadcast_row else edge_operand(indptr, indices, b, b_mode)
    return sf(sf_kind, binop(bin_kind, A, B))


def apply_node(bin_kind, sf_kind, a, b=None, b_broadcast_row=False):
    """applynode element-wise (genGraphOP.py:62, 94-95, 103-108)."""
    A = np.asarray(a, np.float64)
    B = None
    if b is not None:
        b = np.asarray(b, np.float64)
        B = np.broadcast_to(b[:1], (A.shape[0], b.shape[1])) if b_broadcast_row else b[: A.shape[0]]
    return sf(sf_kind, binop(bin_kind, A, B))


def edge_softmax(indptr, indices, a_dst, b_src, sf_kind="EXP_LEAKY_RELU", normalize=True):
    """GAT ops 6-10 composed from the ISA ops above (vTCAD/GraphOP/genGraphOP.py:51-60;
    "/" per template/GAT_op.png): v = sf(scatter_R(a) + scatter_C(b)), sums = gather_R(v),
    out = v / scatter_R(sums) (normalize) or v.  Returns (out, sums)."""
    v = apply_edge(indptr, indices, "ADD", sf_kind, a_dst, "dst", b_src, "src")
    sums = gather_add(indptr, v)
    if not normalize:
        return v, sums
    with np.errstate(divide="ignore", invalid="ignore"):
        return v / sums[row_of_edge(indptr)], sums


def gat_aggregate(indptr, indices, x, a_dst, b_src, sf_kind="EXP_LEAKY_RELU", normalize=True):
    """GAT ops 6-12 without the final SF, composed from the ISA ops (genGraphOP.py:51-64):
    original (normalize): gather_R( scatter_C(x) * alpha ), alpha = edge_softmax;
    trans: numerator gather_R( scatter_C(x) * v ) and denominator gather_R(v).  Returns (y, sums)."""
    v, sums = edge_softmax(indptr, indices, a_dst, b_src, sf_kind, normalize=False)
    w = edge_softmax(indptr, indices, a_dst, b_src, sf_kind, normalize=True)[0] if normalize else v
    return aggregate(indptr, indices, x, "src", w), sums


def aggregate(indptr, indices, x, x_mode="src", w=None, row_scale=None):
    """Fused applyedge MUL -> gather ADD with the scatter FETCH removed
    (hardware_info.yaml Inst_fused [applyedge,gather][MUL,ADD]; code/interpreter.py:575-636, 764-802):
    y[i] = row_scale[i] * sum_{e in row i} w(e) (.) x[idx(e)]."""
    X = edge_operand(indptr, indices, np.asarray(x, np.float64), x_mode)
    if w is not None:
        w = np.asarray(w, np.float64)
        if w.ndim == 1:
            w = w[:, None]
        X = X * _bcast(w, X.shape[1])
    y = gather_add(indptr, X)
    if row_scale is not None:
        y = y * np.asarray(row_scale, np.float64)[:, None]
    return y


def aggregate_abs(indptr, indices, x, x_mode="src", w=None, row_scale=None):
    """sum of |terms| per output element -- the scale of the fp32 summation error bound."""
    ax = np.abs(np.asarray(x, np.float64))
    aw = None if w is None else np.abs(np.asarray(w, np.float64))
    rs = None if row_scale is None else np.abs(np.asarray(row_scale, np.float64))
    return aggregate(indptr, indices, ax, x_mode, aw, rs)


def mm(x, w, row_idx=None, sf_kind=None):
    """applynode MM `j,ij->i` (template/ISA_defination.yaml:1-31): y = x[r] . W."""
    X = np.asarray(x, np.float64)
    if row_idx is not None:
        X = X[np.asarray(row_idx, np.int64)]
    return sf(sf_kind, X @ np.asarray(w, np.float64))


def tile_nnz(indptr, indices, n_cols, T):
    """calculate_sparsity(T, 1) restated on CSR (code/preprocessing.py:12-40):
    self loops removed (:17), rows padded to a multiple of T (:23-27), count of
    non-zeros per (T-row block, single column) block (:30-38) -> int [ceil(N/T), n_cols].
    A dense matrix counts each (dst, src) once, so duplicates are collapsed here too."""
    n = len(indptr) - 1
    rows = row_of_edge(indptr)
    cols = np.asarray(indices, np.int64)
    keep = rows != cols
    rows, cols = rows[keep], cols[keep]
    key = np.unique(rows * n_cols + cols)
    rows, cols = key // n_cols, key % n_cols
    nt = -(-n // T)
    out = np.zeros((nt, n_cols), dtype=np.int64)
    np.add.at(out, (rows // T, cols), 1)
    return out


def gen_size(start, end):
    """code/preprocessing.py:65-72: multiples of `start` until one reaches `end`."""
    size = [start]
    i = 1
    while size[-1] < end:
        i += 1
        size.append(start * i)
    return size


def max_tile(counts):
    """cal_min_sparsity (code/preprocessing.py:53-63): largest tile count (0 floor)."""
    return max(0, int(np.max(counts))) if counts.size else 0
