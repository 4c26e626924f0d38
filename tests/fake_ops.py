"""TEST-ONLY stand-in for gta...ops on CPU tensors, computed by the fp64 oracle.

Used by CPU tests to exercise the executor's block planning / fusion mapping
without a GPU (monkeypatched over executor.ops).  Never used by the product.
"""
import numpy as np
import torch

from oracle import isa_ref


def _np(t):
    return None if t is None else t.detach().cpu().double().numpy()


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.float32))


SELF_TERM_CALLS = [0]  # aggregates that formed a self term (the executor's GIN ops 3-4 fusion)
BF16_OUT_CALLS = [0]   # of those, the ones that stored y in bf16 (the handoff to the fused MLP)
# bf16 aggregate outputs -> the unrounded values: the real fused MLP rounds an fp32 x to bf16 on
# load, so MLP(bf16(y)) is bitwise MLP(y); the fp64 stand-in models it by reading y itself
_BF16_EXACT = {}


def aggregate(graph, x, x_mode="src", w=None, row_scale=None, out=None, accumulate=False, plan=None, self_term=None,
              out_dtype=torch.float32):
    ip, ix = graph.numpy()
    y = isa_ref.aggregate(ip, ix, _np(x), x_mode, _np(w), _np(row_scale))
    if self_term is not None:
        SELF_TERM_CALLS[0] += 1
        xs, sc = self_term
        y = _np(xs)[:graph.n_rows] * float(_np(sc).reshape(-1)[0]) + y
        if out_dtype == torch.bfloat16:
            BF16_OUT_CALLS[0] += 1
            yb = _t(y).to(torch.bfloat16)
            _BF16_EXACT[yb.data_ptr()] = (yb, _t(y))
            return yb
    elif out_dtype != torch.float32:
        raise ValueError("aggregate: a bfloat16 out is written by the self-term form only")
    if out is not None:
        y = y + (_np(out) if accumulate else 0)
        out.copy_(_t(y))
        return out
    return _t(y)


EXPR_CALLS = [0]  # fused expression gathers (the executor's DGN / PNA edge-expression fusion)


def aggregate_expr(graph, shape, operands, bins, sfs=None, swap=False, plan=None):
    """The oracle's apply_edge steps, then its gather (gta_aggregate_expr's definition)."""
    EXPR_CALLS[0] += 1
    ip, ix = graph.numpy()
    sfs = list(sfs or []) + [None] * 3

    def step(b, sf, x, y):
        (xa, xm), (ya, ym) = x, (y if y is not None else (None, "edge"))
        if xm == "row":
            xa, xm = np.repeat(xa[:1], graph.nnz, axis=0), "edge"
        return isa_ref.apply_edge(ip, ix, b, sf, xa, xm, ya, "edge" if ym == "row" else ym, ym == "row"), "edge"

    L = [(_np(t), m) for t, m in operands]
    u = step(bins[0], sfs[0], L[0], L[1] if len(L) > 1 else None)
    if shape == 1:
        t = u
    elif shape == 2:
        t = step(bins[1], sfs[1], L[2], u) if swap else step(bins[1], sfs[1], u, L[2])
    else:
        t = step(bins[2], sfs[2], u, step(bins[1], sfs[1], L[2], L[3]))
    return _t(isa_ref.aggregate(ip, ix, t[0], "edge", None, None))


def gather_add(graph, xe, out=None, accumulate=False, direction="R"):
    if direction == "C":
        ip, ix = graph.numpy()
        y = isa_ref.gather_add(ip, _np(xe), "C", ix, graph.n_cols)
        if out is not None:
            out.copy_(_t(y + (_np(out) if accumulate else 0)))
            return out
        return _t(y)
    return aggregate(graph, xe, "edge", None, out=out, accumulate=accumulate)


class _CSC:
    """CPU stand-in of ops.CSC: numpy's stable argsort by source column (the same permutation the
    device radix sort builds)."""

    def __init__(self, graph):
        from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G
        ip, ix = graph.numpy()
        perm = np.argsort(ix, kind="stable")
        colptr = np.zeros(graph.n_cols + 1, np.int64)
        np.cumsum(np.bincount(ix, minlength=graph.n_cols), out=colptr[1:])
        rows = isa_ref.row_of_edge(ip)[perm]
        cols = np.sort(ix, kind="stable")
        self.colptr, self.perm, self.rows = colptr, perm, rows
        self._views = {"edge": G.from_numpy(colptr, perm, n_cols=graph.nnz),
                       "dst": G.from_numpy(colptr, rows, n_cols=graph.n_rows),
                       "src": G.from_numpy(colptr, cols, n_cols=graph.n_cols)}

    def view(self, kind):
        return self._views[kind]


def csc(graph):
    c = graph._plans.get("fake_csc")
    if c is None:
        c = graph._plans["fake_csc"] = _CSC(graph)
    return c


def scatter(graph, x, direction, out=None):
    ip, ix = graph.numpy()
    return torch.from_numpy(isa_ref.scatter(ip, ix, x.detach().cpu().numpy(), direction))


def apply_edge(graph, bin, sf, a, a_mode="edge", b=None, b_mode="edge", out=None, b_broadcast_row=False):
    ip, ix = graph.numpy()
    return _t(isa_ref.apply_edge(ip, ix, bin, sf, _np(a), a_mode, _np(b), b_mode, b_broadcast_row))


def edge_softmax(graph, a_dst, b_src, sf="EXP_LEAKY_RELU", normalize=True, out=None, sums=None, want_sums=False):
    ip, ix = graph.numpy()
    o, su = isa_ref.edge_softmax(ip, ix, _np(a_dst), _np(b_src), sf, normalize)
    return _t(o), (_t(su) if (want_sums or sums is not None) else None)


def gat_aggregate_blocked(graph, x, a_dst, b_src, sf="EXP_LEAKY_RELU", normalize=True, out=None, sums=None,
                          want_sums=False, plan=None, blocks=16, sf_out=None):
    ip, ix = graph.numpy()
    y, su = isa_ref.gat_aggregate(ip, ix, _np(x), _np(a_dst), _np(b_src), sf, normalize)
    if sf_out is not None:
        y = isa_ref.sf(sf_out, y)
    return _t(y), (_t(su) if (want_sums or sums is not None) else None)


def blocked_ready(graph, blocks):
    ip, ix = graph.numpy()
    return all(np.all(np.diff(ix[ip[r]:ip[r + 1]]) >= 0) for r in range(len(ip) - 1))


class BlockedPlan:  # shape rules of the real plan (ops.BlockedPlan), no device state
    DTYPES = (torch.float32,)

    @staticmethod
    def supports(F, heads, dtype=torch.float32):
        return False

    @staticmethod
    def supports_att(F, heads):
        if F not in (64, 128, 256) or heads <= 0 or F % heads:
            return False
        fh, vq = F // heads, F // 16
        return fh % vq == 0 and 16 % (fh // vq) == 0

    @staticmethod
    def auto_blocks(graph, F, elem=4):
        return 1


def apply_node(bin, sf, a, b=None, out=None, b_broadcast_row=False):
    return _t(isa_ref.apply_node(bin, sf, _np(a), _np(b), b_broadcast_row))


def update_mm(x, w, row_idx=None, sf=None, out=None, m=None):
    xr = _np(x)
    if row_idx is None and m is not None:
        xr = xr[:m]
    return _t(isa_ref.mm(xr, _np(w), None if row_idx is None else row_idx.cpu().numpy(), sf))


MLP_CALLS = [0]  # fused MM -> SF -> MM -> SF launches (the executor's GIN MLP fusion)


def update_mlp_weights_ok(K1, w1, w2):
    return (w1.dtype == torch.bfloat16 and w2.dtype == torch.bfloat16 and K1 == w1.shape[0]
            and max(w1.shape[0], w1.shape[1], w2.shape[1]) <= 128)


def update_mlp_supported(x, w1, w2):
    return x.dtype in (torch.float32, torch.bfloat16) and update_mlp_weights_ok(x.shape[1], w1, w2)


def update_mlp(x, w1, w2, sf1=None, sf2=None, out=None):
    """The two products in fp64, as this module's update_mm computes each (the bf16 rounding of the
    real kernel is the GPU tests' business)."""
    MLP_CALLS[0] += 1
    if x.dtype == torch.bfloat16:
        x = _BF16_EXACT[x.data_ptr()][1]
    return _t(isa_ref.mm(isa_ref.mm(_np(x), _np(w1), None, sf1), _np(w2), None, sf2))


def tile_nnz(graph, T):
    ip, ix = graph.numpy()
    return torch.from_numpy(isa_ref.tile_nnz(ip, ix, graph.n_cols, T).astype(np.int32))
