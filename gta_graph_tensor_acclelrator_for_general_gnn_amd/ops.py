"""ISA ops on device tensors -> libgta (include/gta.h).  No CPU fallback.

One function per ISA op / fused pattern of the GTA stream:
  scatter      ISA `scatter`  (template/ISA_defination.yaml:33-44)        -> gta_scatter
  gather_add   ISA `gather` R/C (template/ISA_defination.yaml:46-61)      -> gta_gather_add (+ gta_csc_build for C)
  aggregate    fused applyedge MUL -> gather ADD (+ removed scatter FETCH)
               (hardware_info.yaml Inst_fused :35-38, code/interpreter.py:575-636, 764-802) -> gta_aggregate
  apply_edge   applyedge ADD/MUL/SF (genGraphOP.py:36, 55-60)              -> gta_apply_edge
  aggregate_expr  a tree of applyedge ops -> gather ADD, fused (DGN, PNA)   -> gta_aggregate_expr
  apply_node   applynode ADD/MUL/SF (genGraphOP.py:62, 94-95, 103-108)     -> gta_apply_node
  update_mm    applynode/applyedge MM, `j,ij->i` (ISA_defination.yaml:1-31) -> gta_update_mm
  tile_nnz     calculate_sparsity (code/preprocessing.py:12-40)            -> gta_tile_nnz
Shapes and strides are validated on the host before any launch.
"""
import ctypes
import math
import threading
import weakref

import torch

from . import _lib
from ._lib import check

_MODES = {"edge": _lib.IDX_EDGE, "src": _lib.IDX_SRC, "dst": _lib.IDX_DST}
_BINS = {None: _lib.BIN_NONE, "NONE": _lib.BIN_NONE, "ADD": _lib.BIN_ADD, "MUL": _lib.BIN_MUL,
         "DIV": _lib.BIN_DIV, "SUB": _lib.BIN_SUB}


def _L():
    return _lib.load()


def _stream(dev):
    return torch.cuda.current_stream(dev).cuda_stream


def _need_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise _lib.GTAError("libgta ops take device (HIP) tensors; got a CPU tensor -- there is no CPU path")


def _rows(t, name, dtype=torch.float32):
    if t.dtype != dtype:
        raise TypeError(f"{name}: expected {dtype}, got {t.dtype}")
    if t.dim() != 2:
        raise ValueError(f"{name}: need a row-major 2-D tensor with unit column stride")
    if t.shape[0] <= 1:  # a single row: its row stride is meaningless (torch may report 1)
        return max(t.shape[1], 1)
    if t.stride(1) != 1 and t.shape[1] > 1 or t.stride(0) < t.shape[1]:
        raise ValueError(f"{name}: need a row-major 2-D tensor with unit column stride")
    return t.stride(0)


LINE_BYTES = 128  # the L2 / fabric line a gathered row is fetched in (MI355X_MICROARCH.md)


def _lines_per_row(row_bytes, pitch_bytes):
    """Mean number of LINE_BYTES lines a row_bytes-long row touches when rows start every
    pitch_bytes from a line-aligned base (the start offsets cycle with period line / gcd)."""
    period = LINE_BYTES // math.gcd(pitch_bytes, LINE_BYTES)
    return sum(-(-((r * pitch_bytes) % LINE_BYTES + row_bytes) // LINE_BYTES) for r in range(period)) / period


def line_pitch(F, elem_size, max_extra=0.5):
    """Row pitch (elements) of a node table the aggregates gather whole rows from: F rounded up to
    whole 128-B lines when that lowers the mean number of lines a gathered row touches, at most
    max_extra more bytes; F otherwise.  GIN products' bf16 model input: 200-B rows touch 2.5 lines
    at a 200-B pitch and 2 at 256 B, and the layer's aggregate runs 5.38 -> 4.66 ms
    (profiles/r05/gin_ld_ab_*.log, bitwise the same sums).  fp32 rows of 128 floats are whole lines already."""
    row = int(F) * int(elem_size)
    if row == 0:
        return F
    padded = -(-row // LINE_BYTES) * LINE_BYTES
    if padded == row or padded - row > max_extra * row:
        return F
    return padded // elem_size if _lines_per_row(row, padded) < _lines_per_row(row, row) else F


def node_table(n, F, dtype, device=None):
    """A [n, F] node table on line-pitched storage (line_pitch), the padding zero."""
    P = line_pitch(F, torch.empty(0, dtype=dtype).element_size())
    if P == F:
        return torch.empty(n, F, dtype=dtype, device=device)
    buf = torch.empty(n, P, dtype=dtype, device=device)
    buf[:, F:].zero_()
    return buf[:, :F]


def pitched(t):
    """The 2-D node table t on line-pitched storage (node_table): t itself when its rows already
    sit at that pitch (a row block of a pitched table is a view, no copy), else a copy.  The
    layout a table should have before the aggregates gather it, chosen once where the table is
    made (the model input, a shard's rows, the all-gathered table), never per call."""
    if t.dim() != 2:
        return t.contiguous()
    P = line_pitch(t.shape[1], t.element_size())
    if t.shape[0] > 1 and t.stride(1) == 1 and t.stride(0) == P:
        return t
    out = node_table(t.shape[0], t.shape[1], t.dtype, t.device)
    out.copy_(t)
    return out


def _sf(sf):
    if sf is None:
        return 0
    if isinstance(sf, int):
        return sf
    return _lib.SF[sf.upper()]


def _ptr(t):
    return None if t is None else t.data_ptr()


class AggregatePlan:
    """Device plan that splits rows longer than `chunk` edges over several wavefronts."""

    def __init__(self, graph, chunk=512):
        _need_gpu(graph.indptr)
        if chunk <= 0 or chunk % 64:
            raise ValueError("chunk must be a positive multiple of 64")
        L = _L()
        self.graph, self.chunk = graph, int(chunk)
        nbytes = check(L.gta_aggregate_plan_bytes(graph.n_rows, graph.nnz, self.chunk), "plan_bytes")
        self.buf = torch.empty(int(nbytes), dtype=torch.uint8, device=graph.device)
        check(L.gta_aggregate_plan_build(_ptr(graph.indptr), graph.n_rows, graph.nnz, self.chunk,
                                         _ptr(self.buf), int(nbytes), _stream(graph.device)), "plan_build")
        self._ws = {}
        # rows split over several wavefronts (read once, at build): none -> aggregate() runs the
        # one-wave-per-row form, which needs no combine launch (small graphs: Cora)
        self.splits = self.n_split()

    def workspace(self, F):
        if F not in self._ws:
            L = _L()
            nb = check(L.gta_aggregate_workspace_bytes(self.graph.n_rows, self.graph.nnz, self.chunk, F),
                       "workspace_bytes")
            self._ws[F] = torch.empty(int(nb), dtype=torch.uint8, device=self.graph.device)
        return self._ws[F]

    def n_items(self):
        return int(self.buf[:8].view(torch.int64).item())

    def n_split(self):
        return int(self.buf[8:16].view(torch.int64).item())


def aggregate(graph, x, x_mode="src", w=None, row_scale=None, out=None, accumulate=False, plan=None, self_term=None,
              out_dtype=torch.float32):
    """y[i] (+)= row_scale[i] * sum_{e in row i} w(e) * x[idx(e)]  (K6/K7/K2).

    self_term: None, or (x_self, s): y[i] = x_self[i] * s + row_scale[i] * sum (gta_aggregate_self,
    no accumulate; x_self [>= N, F] of x's dtype, s a one-element float32 device tensor) -- without
    row_scale bitwise apply_node("MUL", x_self, s) followed by the accumulating aggregate (GIN ops
    3-4); with row_scale the scaled sum is rounded before the add.
    out_dtype: torch.bfloat16 (self_term only, ABI 10) stores y rounded to bf16 (round to nearest
    even, the rounding the fused MLP applies to an fp32 x); a fresh out is then a [N, F] view of
    [N, ceil8(F)] rows (16-B aligned, what gta_update_mlp reads).

    x_mode: "src" (x is [N_src, F], fused scatter C), "dst" (fused scatter R),
            "edge" (x is an edge tensor [E, F]).  x float32, or bfloat16 for "src" / "dst" with
            head weights or none (rows widened exactly, fp32 sums).
    w: None, or [E, H] with H | F (H == F: full-width edge weights).
    plan: None (one wavefront per row), an AggregatePlan, or an int chunk (cached plan).
    """
    _need_gpu(x, w, row_scale, out, graph.indptr)
    F = x.shape[1]
    if x.dtype == torch.bfloat16 and x_mode == "edge":
        raise TypeError("aggregate: bfloat16 rows are gathered by index (src / dst)")
    ldx = _rows(x, "x", torch.bfloat16 if x.dtype == torch.bfloat16 else torch.float32)
    x_dt = _lib.GTA_BF16 if x.dtype == torch.bfloat16 else _lib.GTA_F32
    if x_mode == "edge" and x.shape[0] < graph.nnz:
        raise ValueError("edge-mode x must have E rows")
    if x_mode == "src" and x.shape[0] < graph.n_cols:
        raise ValueError("src-mode x must have n_cols rows")
    if x_mode == "dst" and x.shape[0] < graph.n_rows:
        raise ValueError("dst-mode x must have n_rows rows")
    ldw, heads = 0, 0
    if w is not None:
        if w.dim() == 1:
            w = w.view(-1, 1)
        ldw = _rows(w, "w")
        heads = w.shape[1]
        if w.shape[0] < graph.nnz or F % heads:
            raise ValueError(f"w must be [E, H] with H | F (got {tuple(w.shape)}, F={F})")
    if row_scale is not None and (row_scale.dtype != torch.float32 or row_scale.numel() < graph.n_rows
                                  or not row_scale.is_contiguous()):
        raise ValueError("row_scale must be contiguous float32 [N]")
    if out_dtype not in (torch.float32, torch.bfloat16) or out_dtype == torch.bfloat16 and self_term is None:
        raise ValueError("aggregate: a bfloat16 out is written by the self-term form only")
    if out is None:
        if out_dtype == torch.bfloat16:
            out = torch.empty(graph.n_rows, (F + 7) // 8 * 8, dtype=out_dtype, device=x.device)[:, :F]
        else:
            out = (torch.zeros if accumulate else torch.empty)(graph.n_rows, F, dtype=torch.float32, device=x.device)
    ldy = _rows(out, "out", out_dtype)
    if out.shape[0] < graph.n_rows or out.shape[1] != F:
        raise ValueError("out must be [N, F]")
    if graph.n_rows == 0:
        return out
    if isinstance(plan, int):
        plan = graph.plan(plan)
        if plan.splits == 0:  # no row is split: the per-row form (same sums, no combine launch)
            plan = None
    pbuf = ws = None
    chunk = 0
    if plan is not None:
        if plan.graph is not graph:
            raise ValueError("plan built for another graph")
        pbuf, ws, chunk = plan.buf, plan.workspace(F), plan.chunk
    if self_term is not None:
        xs, sc = self_term
        if accumulate or xs.dtype != x.dtype or xs.shape[0] < graph.n_rows or xs.shape[1] != F:
            raise ValueError("aggregate self_term: x_self [N, F] of x's dtype, no accumulate")
        if sc.dtype != torch.float32 or sc.numel() != 1:
            raise ValueError("aggregate self_term: s must be a one-element float32 tensor")
        _need_gpu(xs, sc)
        ldxs = _rows(xs, "x_self", xs.dtype)
        check(_L().gta_aggregate_self(_ptr(graph.indptr), _ptr(graph.indices), graph.n_rows, graph.nnz, _MODES[x_mode],
                                      _ptr(x), ldx, F, x_dt, _ptr(w), ldw, heads, _ptr(row_scale), _ptr(xs), ldxs,
                                      _ptr(sc.contiguous()), _ptr(out), ldy,
                                      _lib.GTA_BF16 if out_dtype == torch.bfloat16 else _lib.GTA_F32,
                                      _ptr(pbuf), chunk, _ptr(ws),
                                      _stream(x.device)), "aggregate_self")
        return out
    check(_L().gta_aggregate(_ptr(graph.indptr), _ptr(graph.indices), graph.n_rows, graph.nnz, _MODES[x_mode],
                             _ptr(x), ldx, F, x_dt, _ptr(w), ldw, heads, _ptr(row_scale), _ptr(out), ldy,
                             int(bool(accumulate)), _ptr(pbuf), chunk, _ptr(ws), _stream(x.device)), "aggregate")
    return out


EXPR_SHAPES = {1: 2, 2: 3, 3: 4}  # gta_aggregate_expr shape -> operand count


def aggregate_expr(graph, shape, operands, bins, sfs=None, swap=False, plan=None):
    """y[i] = sum_{e in row i} t(e) with t an apply_edge expression (gta_aggregate_expr, ABI 14):
      shape 1: t = sf0(L0 bin0 L1)   (bins[0] None: sf0(L0))
      shape 2: u = sf0(L0 bin0 L1); t = sf1(L2 bin1 u if swap else u bin1 L2)
      shape 3: u = sf0(L0 bin0 L1); v = sf1(L2 bin1 L3); t = sf2(u bin2 v)
    operands: [(tensor, mode)] with mode "edge" / "src" / "dst", or "row" (a [1, F] row broadcast to
    every edge); fp32, F columns each.  Bitwise equal to the apply_edge ops followed by
    aggregate(..., "edge", plan=plan) of their output.  Returns None when an operand's alignment
    does not admit that aggregate's vector width (GTA_ERR_UNSUPPORTED: run the ops unfused)."""
    if shape not in EXPR_SHAPES:
        raise ValueError(f"aggregate_expr: shape must be 1, 2 or 3 (got {shape})")
    n_ops = shape
    bins = list(bins) + [None] * (3 - len(bins))
    sfs = list(sfs or []) + [None] * (3 - len(sfs or []))
    n_l = 1 if (shape == 1 and bins[0] is None) else EXPR_SHAPES[shape]
    if len(operands) != n_l:
        raise ValueError(f"aggregate_expr: shape {shape} takes {n_l} operands (got {len(operands)})")
    ts = [t for t, _ in operands]
    _need_gpu(graph.indptr, *ts)
    F = ts[0].shape[1]
    ptrs, modes, lds = (ctypes.c_void_p * 4)(), (ctypes.c_int * 4)(), (ctypes.c_int64 * 4)()
    for l, (t, m) in enumerate(operands):
        if t.shape[1] != F:
            raise ValueError("aggregate_expr: every operand has the same width")
        ld = _rows(t, f"operand {l}")
        if m == "row":
            m, ld = "edge", 0
            if t.shape[0] < 1:
                raise ValueError("aggregate_expr: a broadcast row needs one row")
        else:
            need = {"edge": graph.nnz, "src": graph.n_cols, "dst": graph.n_rows}[m]
            if t.shape[0] < need:
                raise ValueError(f"aggregate_expr operand {l}: {m}-mode operand needs {need} rows")
        ptrs[l], modes[l], lds[l] = t.data_ptr(), _MODES[m], ld
    cb = (ctypes.c_int * 3)(*[_BINS[b] for b in bins])
    cs = (ctypes.c_int * 3)(*[_sf(s) for s in sfs])
    out = torch.empty(graph.n_rows, F, dtype=torch.float32, device=ts[0].device)
    if graph.n_rows == 0:
        return out
    if isinstance(plan, int):
        plan = graph.plan(plan)
        if plan.splits == 0:  # as aggregate: no split row, the per-row form
            plan = None
    pbuf = ws = None
    chunk = 0
    if plan is not None:
        if plan.graph is not graph:
            raise ValueError("plan built for another graph")
        pbuf, ws, chunk = plan.buf, plan.workspace(F), plan.chunk
    rc = _L().gta_aggregate_expr(_ptr(graph.indptr), _ptr(graph.indices), graph.n_rows, graph.nnz, n_ops,
                                 ptrs, modes, lds, cb, cs, int(bool(swap)), F, _ptr(out), F, _ptr(pbuf), chunk,
                                 _ptr(ws), _stream(ts[0].device))
    if rc == _lib.ERR_UNSUPPORTED:
        return None
    check(rc, "aggregate_expr")
    return out


class BlockedPlan:
    """Column-blocked aggregate plan (gta_aggregate_blocked_plan_build): per-row segment table over
    B source-column blocks, heaviest-first row order, and the work items -- every (block, row)
    segment cut into parts of <= item_edges edges -- with each row's item list for the ordered
    reduce."""

    ITEM_EDGES = 256  # default part length (profiles/r01_item_sweep.json)
    ROW_EDGES = 0     # default merge target for light rows (0 = off)

    def __init__(self, graph, blocks=32, item_edges=None, row_edges=None):
        _need_gpu(graph.indptr)
        L = _L()
        self.graph, self.blocks = graph, int(blocks)
        self.item_edges = int(item_edges or BlockedPlan.ITEM_EDGES)
        self.row_edges = int(BlockedPlan.ROW_EDGES if row_edges is None else row_edges)
        nb = check(L.gta_aggregate_blocked_plan_bytes(graph.n_rows, graph.nnz, self.blocks, self.item_edges),
                   "blocked_plan_bytes")
        self.buf = torch.empty(int(nb), dtype=torch.uint8, device=graph.device)
        check(L.gta_aggregate_blocked_plan_build(_ptr(graph.indptr), _ptr(graph.indices), graph.n_rows, graph.n_cols,
                                                 graph.nnz, self.blocks, self.item_edges, self.row_edges,
                                                 _ptr(self.buf), int(nb),
                                                 _stream(graph.device)),
              "blocked_plan_build")
        hdr = self.buf[:64].view(torch.int64).cpu()
        self.sorted = int(hdr[3]) == 0
        self.n_items = int(hdr[4])
        self._ws = {}

    def workspace(self, F):
        """Per-item partial rows for the single-launch form ([items, F] fp32)."""
        if F not in self._ws:
            nb = check(_L().gta_aggregate_blocked_workspace_bytes(self.graph.n_rows, self.graph.nnz, self.blocks, F,
                                                                  self.item_edges),
                       "blocked_workspace_bytes")
            self._ws[F] = torch.empty(int(nb), dtype=torch.uint8, device=self.graph.device)
        return self._ws[F]

    def workspace_att(self, F, heads):
        """Partial rows of the fused attention aggregate ([items, F + heads padded to 4])."""
        key = ("att", F, heads)
        if key not in self._ws:
            nb = check(_L().gta_gat_aggregate_blocked_workspace_bytes(self.graph.n_rows, self.graph.nnz, self.blocks,
                                                                      F, heads, self.item_edges),
                       "gat_workspace_bytes")
            self._ws[key] = torch.empty(int(nb), dtype=torch.uint8, device=self.graph.device)
        return self._ws[key]

    @staticmethod
    def supports_att(F, heads):
        """Shapes of gta_gat_aggregate_blocked: F in {64, 128, 256}, (F/heads) a multiple of F/16
        with lanes per head dividing 16."""
        if F not in (64, 128, 256) or heads <= 0 or F % heads:
            return False
        fh, vq = F // heads, F // 16
        return fh % vq == 0 and 16 % (fh // vq) == 0

    DTYPES = (torch.float32,)  # gathered-table dtypes of the blocked kernels

    @staticmethod
    def auto_blocks(graph, F, elem=4):
        """Column blocks for a gathered table of graph.n_cols x F elements of `elem` bytes: slices
        of ~6 MB (measured optima with the lean half-wave kernel: B = 20 for the 119 MB Reddit
        table, B = 10 for the 60 MB column half of a 2-D grid tile; profiles/r01_blocks_rowmerge_sweep.json,
        r01_shard_b_sweep.json), capped so a row keeps >= 24 edges per block on average (each
        (block, row) item pays a start-up and a partial row written and re-read).
        Below 4 the single-pass row-chunk kernel is the better choice."""
        table_mb = graph.n_cols * F * elem / 1e6
        avg_deg = graph.nnz / max(1, graph.n_rows)
        return int(max(1, min(24, round(table_mb / 6.0), avg_deg // 24)))

    @staticmethod
    def supports(F, heads, dtype=torch.float32):
        """Shapes libgta's blocked kernels take: an fp32 table, F in {64, 128, 256} and, with head
        weights, the quarter-wave form's lanes per head (F/heads)/(F/16) in {1, 2, 4, 8, 16} or the
        one-item-per-wave form's (F/heads)/(F/64) in {4, 8, 16}."""
        if dtype not in BlockedPlan.DTYPES or F not in (64, 128, 256):
            return False
        if not heads:
            return True
        if F % heads:
            return False
        fh, vq, vw = F // heads, F // 16, F // 64
        quarter = fh % vq == 0 and (fh // vq) in (1, 2, 4, 8, 16)
        single = fh % vw == 0 and (fh // vw) in (4, 8, 16)
        return quarter or single


def aggregate_blocked(graph, x, w=None, row_scale=None, out=None, accumulate=False, plan=None, blocks=32,
                      single_launch=True):
    """Same result as aggregate(graph, x, "src", w, ...) computed column block by column block so the
    gathered X slice stays L2-resident.  single_launch: one launch over (block, row) items into per-block
    slabs + an ordered reduce; otherwise B dependent launches accumulating into out."""
    _need_gpu(x, w, row_scale, out, graph.indptr)
    F = x.shape[1]
    ldx = _rows(x, "x")
    if x.shape[0] < graph.n_cols:
        raise ValueError("x must have n_cols rows")
    ldw, heads = 0, 0
    if w is not None:
        if w.dim() == 1:
            w = w.view(-1, 1)
        ldw = _rows(w, "w")
        heads = w.shape[1]
    if not BlockedPlan.supports(F, heads, x.dtype):
        raise ValueError(f"aggregate_blocked: unsupported F={F}, heads={heads}, dtype={x.dtype}")
    if plan is None:
        plan = graph.blocked_plan(blocks)
    if not plan.sorted:
        raise ValueError("aggregate_blocked needs every CSR row's columns sorted")
    if out is None:
        out = (torch.zeros if accumulate else torch.empty)(graph.n_rows, F, dtype=torch.float32, device=x.device)
    ldy = _rows(out, "out")
    ws = plan.workspace(F) if single_launch else None
    check(_L().gta_aggregate_blocked(_ptr(graph.indptr), _ptr(graph.indices), graph.n_rows, graph.n_cols, graph.nnz,
                                     _ptr(x), ldx, F, _ptr(w), ldw, heads, _ptr(row_scale), _ptr(out), ldy,
                                     int(bool(accumulate)), _ptr(plan.buf), plan.blocks, plan.item_edges, _ptr(ws),
                                     _stream(x.device)), "aggregate_blocked")
    return out


def blocked_ready(graph, blocks):
    """True when the column-blocked kernels can run on this graph (rows' columns sorted)."""
    return graph.blocked_plan(blocks).sorted


def gat_aggregate_blocked(graph, x, a_dst, b_src, sf="EXP_LEAKY_RELU", normalize=True, out=None, sums=None,
                          want_sums=False, plan=None, blocks=16, sf_out=None):
    """Fused GAT attention aggregate (gta_gat_aggregate_blocked): with v = sf(a_dst[dst] + b_src[src]),
    normalize: out[i] = sum_e v x[src] / sum_e v per head (GAT ops 6-12); else the numerator alone.
    sf_out: an SF applied to out as it is written (GAT op 13; None = none), bitwise equal to
    apply_node(None, sf_out, out).  sums[i, h] = sum_e v (want_sums / sums given).  Returns (out, sums)."""
    _need_gpu(x, a_dst, b_src, out, sums, graph.indptr)
    F, H = x.shape[1], a_dst.shape[1]
    if b_src.shape[1] != H:
        raise ValueError("gat_aggregate_blocked: a_dst and b_src need the same head count")
    if not BlockedPlan.supports_att(F, H):
        raise ValueError(f"gat_aggregate_blocked: unsupported F={F}, heads={H}")
    if x.shape[0] < graph.n_cols or b_src.shape[0] < graph.n_cols or a_dst.shape[0] < graph.n_rows:
        raise ValueError("gat_aggregate_blocked: x / b_src need n_cols rows, a_dst n_rows")
    if plan is None:
        plan = graph.blocked_plan(blocks)
    if not plan.sorted:
        raise ValueError("gat_aggregate_blocked needs every CSR row's columns sorted")
    if out is None:
        out = torch.empty(graph.n_rows, F, dtype=torch.float32, device=x.device)
    if sums is None and want_sums:
        sums = torch.empty(graph.n_rows, H, dtype=torch.float32, device=x.device)
    if sums is not None and (not sums.is_contiguous() or tuple(sums.shape) != (graph.n_rows, H)):
        raise ValueError("gat_aggregate_blocked: sums must be a contiguous [N, heads] tensor")
    ws = plan.workspace_att(F, H)
    check(_L().gta_gat_aggregate_blocked(_ptr(graph.indptr), _ptr(graph.indices), graph.n_rows, graph.n_cols,
                                         graph.nnz, _ptr(x), _rows(x, "x"), F, _ptr(a_dst), _rows(a_dst, "a_dst"), _ptr(b_src),
                                         _rows(b_src, "b_src"), H, _sf(sf), 1 if normalize else 0, _sf(sf_out), _ptr(out),
                                         _rows(out, "out"), _ptr(sums), _ptr(plan.buf), plan.blocks, plan.item_edges,
                                         _ptr(ws),
                                         _stream(x.device)), "gat_aggregate_blocked")
    return out, sums


class CSC:
    """The CSR's edges ordered by SOURCE column (gta_csc_build, ABI 11): colptr int64 [n_cols + 1],
    perm int32 [E] (CSR edge id at each position), rows int32 [E] (that edge's destination row).
    Stable: a column's edges keep CSR order, so every sum over them has a fixed order.  Built once
    per graph on the device (Graph.csc()).  The ISA's DIRECTION src (ORDER C) for gather
    (template/ISA_defination.yaml:46-48) runs the ordered row kernels over these transposed views."""

    def __init__(self, graph):
        _need_gpu(graph.indptr)
        L = _L()
        dev = graph.device
        self.graph = graph
        self.colptr = torch.empty(graph.n_cols + 1, dtype=torch.int64, device=dev)
        self.perm = torch.empty(graph.nnz, dtype=torch.int32, device=dev)
        self.rows = torch.empty(graph.nnz, dtype=torch.int32, device=dev)
        nb = check(L.gta_csc_workspace_bytes(graph.n_cols, graph.nnz), "csc_workspace_bytes")
        ws = torch.empty(int(nb), dtype=torch.uint8, device=dev)
        check(L.gta_csc_build(_ptr(graph.indptr), _ptr(graph.indices), graph.n_rows, graph.n_cols, graph.nnz,
                              _ptr(self.colptr), _ptr(self.perm), _ptr(self.rows), _ptr(ws), int(nb),
                              _stream(dev)), "csc_build")
        self._views = {}

    def view(self, kind):
        """A Graph over the n_cols source nodes whose row j lists column j's edges in CSC order, with
        "indices" = what an operand of those edges is read by: "edge" -> the CSR edge id (an edge
        tensor read as a table of E rows), "dst" -> the destination row (a scatter R operand),
        "src" -> j itself (a scatter C operand)."""
        if kind not in self._views:
            from . import graph as G
            g = self.graph
            if kind == "edge":
                v = G.Graph(self.colptr, self.perm, n_cols=g.nnz)
            elif kind == "dst":
                v = G.Graph(self.colptr, self.rows, n_cols=g.n_rows)
            elif kind == "src":
                cols = torch.arange(g.n_cols, device=g.device, dtype=torch.int32)
                v = G.Graph(self.colptr, torch.repeat_interleave(cols, self.colptr[1:] - self.colptr[:-1]),
                            n_cols=g.n_cols)
            else:
                raise ValueError(kind)
            self._views[kind] = v
        return self._views[kind]


def csc(graph):
    """graph's cached CSC view (Graph.csc())."""
    return graph.csc()


def gather_add(graph, xe, out=None, accumulate=False, direction="R"):
    """ISA gather ADD of an edge tensor xe [E, F] (CSR order), both DIRECTIONs (ABI 11):
    "R": y[i] (+)= sum_{e in row i} xe[e]            (to the destination; y [n_rows, F])
    "C": y[j] (+)= sum_{e : src(e) = j} xe[e]         (to the source; y [n_cols, F]), summed in the
         stable CSC order of graph.csc() -- deterministic, no atomics."""
    _need_gpu(xe, out, graph.indptr)
    if direction not in ("R", "C"):
        raise ValueError("gather_add: direction must be 'R' or 'C'")
    ldx = _rows(xe, "xe")
    F = xe.shape[1]
    if xe.shape[0] < graph.nnz:
        raise ValueError("xe must be [E, F]")
    n_out = graph.n_rows if direction == "R" else graph.n_cols
    if out is None:
        out = (torch.zeros if accumulate else torch.empty)(n_out, F, dtype=torch.float32, device=xe.device)
    ldy = _rows(out, "out")
    if out.shape[0] < n_out or out.shape[1] != F:
        raise ValueError(f"out must be [{n_out}, {F}]")
    colptr = perm = None
    if direction == "C":
        c = graph.csc()
        colptr, perm = c.colptr, c.perm
    check(_L().gta_gather_add(_lib.DIR_R if direction == "R" else _lib.DIR_C, _ptr(graph.indptr), graph.n_rows,
                              graph.nnz, _ptr(colptr), _ptr(perm), graph.n_cols, _ptr(xe), ldx, F, _ptr(out), ldy,
                              int(bool(accumulate)), _stream(xe.device)), "gather_add")
    return out


def scatter(graph, x, direction, out=None):
    """out[e] = x[dst(e)] (direction "R") or x[src(e)] (direction "C"); bit-exact copy."""
    _need_gpu(x, out, graph.indptr)
    if x.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError("scatter supports float32 / bfloat16")
    ldx = _rows(x, "x", x.dtype)
    F = x.shape[1]
    d = {"R": _lib.DIR_R, "C": _lib.DIR_C}[direction]
    need = graph.n_rows if d == _lib.DIR_R else graph.n_cols
    if x.shape[0] < need:
        raise ValueError(f"scatter {direction}: x has {x.shape[0]} rows < {need}")
    if out is None:
        out = torch.empty(graph.nnz, F, dtype=x.dtype, device=x.device)
    ldo = _rows(out, "out", x.dtype)
    dt = _lib.GTA_F32 if x.dtype == torch.float32 else _lib.GTA_BF16
    check(_L().gta_scatter(d, _ptr(graph.indptr), _ptr(graph.indices), graph.n_rows, graph.nnz, _ptr(x), ldx, F, dt,
                           _ptr(out), ldo, _stream(x.device)), "scatter")
    return out


def _out_width(Fa, Fb):
    if Fb is None:
        return Fa
    Fo = max(Fa, Fb)
    if Fo % Fa or Fo % Fb:
        raise ValueError(f"operand widths {Fa} and {Fb} do not broadcast")
    return Fo


def apply_edge(graph, bin, sf, a, a_mode="edge", b=None, b_mode="edge", out=None, b_broadcast_row=False):
    """out[e] = sf(a[ia(e)] bin b[ib(e)]) with head broadcast of the narrower operand."""
    _need_gpu(a, b, out, graph.indptr)
    lda = _rows(a, "a")
    ldb = _rows(b, "b") if b is not None else 0
    if b_broadcast_row:
        ldb = 0
    Fo = _out_width(a.shape[1], None if b is None else b.shape[1])
    if out is None:
        out = torch.empty(graph.nnz, Fo, dtype=torch.float32, device=a.device)
    ldo = _rows(out, "out")
    if out.shape[1] != Fo:
        raise ValueError("out width mismatch")
    for t, m, name in ((a, a_mode, "a"), (b, b_mode, "b")):
        if t is None or (name == "b" and b_broadcast_row):
            continue
        need = {"edge": graph.nnz, "src": graph.n_cols, "dst": graph.n_rows}[m]
        if t.shape[0] < need:
            raise ValueError(f"apply_edge {name}: {m}-mode operand needs {need} rows")
    if APPLY_EDGE_FLAT and Fo in (64, 128, 256) and graph.nnz > 0 and _flat_aligned(Fo, a, lda, b, ldb, out, ldo):
        # edge-parallel form (ABI 13): 32 edges per wave whatever the row lengths
        dst = "dst" in (a_mode, None if (b is None or b_broadcast_row) else b_mode)
        check(_L().gta_apply_edge_flat(_BINS[bin], _sf(sf), _ptr(graph.row_of_edge()) if dst else None,
                                       _ptr(graph.indices), graph.nnz, _ptr(a), _MODES[a_mode], lda, a.shape[1],
                                       _ptr(b), _MODES[b_mode], ldb, 0 if b is None else b.shape[1], _ptr(out), ldo,
                                       _stream(a.device)), "apply_edge_flat")
        return out
    check(_L().gta_apply_edge(_BINS[bin], _sf(sf), _ptr(graph.indptr), _ptr(graph.indices), graph.n_rows, graph.nnz,
                              _ptr(a), _MODES[a_mode], lda, a.shape[1], _ptr(b), _MODES[b_mode], ldb,
                              0 if b is None else b.shape[1], _ptr(out), ldo, _stream(a.device)), "apply_edge")
    return out


APPLY_EDGE_FLAT = True  # gta_apply_edge_flat where it applies (round 6); False: the row-sweep forms (A/B)


def _flat_aligned(Fo, a, lda, b, ldb, out, ldo):
    """The vector width of gta_apply_edge_flat (Fo / 64) divides every row start it reads or writes."""
    vw = Fo // 64

    def ok(t, ld, width):
        if t is None:
            return True
        g = Fo // width
        return (ld % vw == 0 and t.data_ptr() % (4 * vw) == 0) if g == 1 else g % vw == 0
    return ok(a, lda, a.shape[1]) and ok(b, ldb, None if b is None else b.shape[1]) and ok(out, ldo, Fo)


def edge_softmax(graph, a_dst, b_src, sf="EXP_LEAKY_RELU", normalize=True, out=None, sums=None,
                 want_sums=False):
    """Fused GAT edge-softmax (GAT ops 6-10, vTCAD/GraphOP/genGraphOP.py:51-60):
    v[e] = sf(a_dst[dst(e)] + b_src[src(e)]); sums[i] = sum_{e in row i} v[e];
    out[e] = v[e] / sums[dst(e)] (normalize) or v[e].  Returns (out [E, H], sums [N, H] or None)."""
    _need_gpu(a_dst, b_src, out, sums, graph.indptr)
    H = a_dst.shape[1]
    if b_src.shape[1] != H:
        raise ValueError("edge_softmax: a_dst and b_src need the same head count")
    if a_dst.shape[0] < graph.n_rows or b_src.shape[0] < graph.n_cols:
        raise ValueError("edge_softmax: score tensors have too few rows")
    if out is None:
        out = torch.empty(graph.nnz, H, dtype=torch.float32, device=a_dst.device)
    if not out.is_contiguous() or tuple(out.shape) != (graph.nnz, H):
        raise ValueError("edge_softmax: out must be a contiguous [E, H] tensor")
    if sums is None and want_sums:
        sums = torch.empty(graph.n_rows, H, dtype=torch.float32, device=a_dst.device)
    if sums is not None and (not sums.is_contiguous() or tuple(sums.shape) != (graph.n_rows, H)):
        raise ValueError("edge_softmax: sums must be a contiguous [N, H] tensor")
    check(_L().gta_edge_softmax(_ptr(graph.indptr), _ptr(graph.indices), graph.n_rows, graph.nnz, _ptr(a_dst),
                                _rows(a_dst, "a_dst"), _ptr(b_src), _rows(b_src, "b_src"), H, _sf(sf),
                                1 if normalize else 0, _ptr(out), _ptr(sums), _stream(a_dst.device)),
          "edge_softmax")
    return out, sums


def apply_node(bin, sf, a, b=None, out=None, b_broadcast_row=False):
    """out[i] = sf(a[i] bin b[i]); b_broadcast_row: b is a single row for all i (e.g. (1+eps)).
    a float32 or bfloat16 (widened exactly); b and out float32."""
    _need_gpu(a, b, out)
    lda = _rows(a, "a", torch.bfloat16 if a.dtype == torch.bfloat16 else torch.float32)
    ldb = _rows(b, "b") if b is not None else 0
    if b is not None and not b_broadcast_row and b.shape[0] < a.shape[0]:
        raise ValueError("apply_node: b has fewer rows than a")
    if b_broadcast_row:
        ldb = 0
    n = a.shape[0]
    Fo = _out_width(a.shape[1], None if b is None else b.shape[1])
    if out is None:
        out = torch.empty(n, Fo, dtype=torch.float32, device=a.device)
    ldo = _rows(out, "out")
    a_dt = _lib.GTA_BF16 if a.dtype == torch.bfloat16 else _lib.GTA_F32
    check(_L().gta_apply_node(_BINS[bin], _sf(sf), n, _ptr(a), lda, a.shape[1], a_dt, _ptr(b), ldb,
                              0 if b is None else b.shape[1], _ptr(out), ldo, _stream(a.device)), "apply_node")
    return out


def update_mm(x, w, row_idx=None, sf=None, out=None, m=None):
    """out[m] = sf(x[r(m)] . w); x/w float32, bfloat16, or float32 x with bfloat16 w (x rounded
    to bf16 on its way into LDS); out float32.

    row_idx: None (r(m) = m, M = x.shape[0]) or int32 [M] of x rows (gather-GEMM)."""
    _need_gpu(x, w, row_idx, out)
    mixed = x.dtype == torch.float32 and w.dtype == torch.bfloat16
    if not mixed and (x.dtype != w.dtype or x.dtype not in (torch.float32, torch.bfloat16)):
        raise TypeError("update_mm: x/w must be f32/f32, bf16/bf16, or f32 x with bf16 w")
    ldx = _rows(x, "x", x.dtype)
    ldw = _rows(w, "w", w.dtype)
    K, N = w.shape
    if x.shape[1] != K:
        raise ValueError(f"update_mm: x width {x.shape[1]} != W rows {K}")
    if row_idx is not None:
        if row_idx.dtype != torch.int32 or not row_idx.is_contiguous():
            raise TypeError("row_idx must be contiguous int32")
        M = row_idx.numel() if m is None else m
    else:
        M = x.shape[0] if m is None else m
    if out is None:
        out = torch.empty(M, N, dtype=torch.float32, device=x.device)
    ldo = _rows(out, "out")
    dt = _lib.GTA_F32_BF16 if mixed else (_lib.GTA_F32 if x.dtype == torch.float32 else _lib.GTA_BF16)
    splits = _mm_splits(M, K, N, dt, x.device) if MM_FORM == "rows" else 1
    if splits > 1:  # few rows: split K over blocks, slices summed in order (deterministic)
        wt = _transposed(w)
        nb = check(_L().gta_update_mm_t_split_workspace_bytes(M, K, N, splits), "update_mm_t_split_workspace_bytes")
        ws = torch.empty(max(1, nb // 4), dtype=torch.float32, device=x.device)
        check(_L().gta_update_mm_t_split(_ptr(x), ldx, _ptr(row_idx), M, K, _ptr(wt), _rows(wt, "w^T", wt.dtype), N,
                                         dt, _sf(sf), _ptr(out), ldo, splits, _ptr(ws), nb, _stream(x.device)),
              "update_mm_t_split")
    elif MM_FORM == "rows" and M >= MM_ROWS_MIN_M:  # row-streaming kernel on W^T (cached per weight version)
        wt = _transposed(w)
        check(_L().gta_update_mm_t(_ptr(x), ldx, _ptr(row_idx), M, K, _ptr(wt), _rows(wt, "w^T", wt.dtype), N, dt, _sf(sf),
                                   _ptr(out), ldo, _stream(x.device)), "update_mm_t")
    else:
        check(_L().gta_update_mm(_ptr(x), ldx, _ptr(row_idx), M, K, _ptr(w), ldw, N, dt, _sf(sf), _ptr(out), ldo,
                                 _stream(x.device)), "update_mm")
    return out


def update_mlp_weights_ok(K1, w1, w2):
    """The weight half of update_mlp_supported: bf16 W1 [K1, N1] and W2 [N1, N2], K1 % 4 == 0,
    K1, N1, N2 <= 128."""
    return (w1.dtype == torch.bfloat16 and w2.dtype == torch.bfloat16 and w1.dim() == 2 and w2.dim() == 2
            and K1 == w1.shape[0] and w1.shape[1] == w2.shape[0] and K1 % 4 == 0
            and max(K1, w1.shape[1], w2.shape[1]) <= 128)


def update_mlp_supported(x, w1, w2):
    """Shapes gta_update_mlp takes: fp32 or bf16 x [M, K1] with unit column stride and 16-B aligned
    rows, K1 % 4 == 0, bf16 W1 [K1, N1] and W2 [N1, N2], K1, N1, N2 <= 128."""
    row_elems = 8 if x.dtype == torch.bfloat16 else 4
    return (x.dtype in (torch.float32, torch.bfloat16) and x.dim() == 2 and update_mlp_weights_ok(x.shape[1], w1, w2)
            and (x.shape[0] <= 1 or x.stride(1) == 1) and (x.shape[0] <= 1 or x.stride(0) % row_elems == 0)
            and x.data_ptr() % 16 == 0)


def update_mlp(x, w1, w2, sf1=None, sf2=None, out=None):
    """out = sf2(bf16(sf1(x W1)) W2) in one launch (gta_update_mlp: GIN's MM -> SF -> MM -> SF,
    genGraphOP.py:103-108), bitwise equal to update_mm(update_mm(x, w1, sf=sf1), w2, sf=sf2) with
    fp32 x and bf16 weights, without the [M, N1] intermediate in HBM.  A bf16 x (ABI 10) gives the
    same bits as the fp32 x it was rounded from: the kernel rounds an fp32 x to bf16 on load."""
    _need_gpu(x, w1, w2, out)
    if not update_mlp_supported(x, w1, w2):
        raise ValueError("update_mlp: fp32 / bf16 x [M, K1], bf16 W1 [K1, N1], bf16 W2 [N1, N2], K1, N1, N2 <= 128")
    M, K1 = x.shape
    N1, N2 = w1.shape[1], w2.shape[1]
    w1t, w2t = _transposed(w1), _transposed(w2)
    if out is None:
        out = torch.empty(M, N2, dtype=torch.float32, device=x.device)
    if out.shape[0] < M or out.shape[1] != N2:
        raise ValueError("update_mlp: out must be [M, N2]")
    xb = x.dtype == torch.bfloat16
    ldx = _rows(x, "x", x.dtype)
    if M <= 1:  # one row: its stride is never used; give the kernel the 16-B multiple it checks
        step = 8 if xb else 4
        ldx = -(-ldx // step) * step
    check(_L().gta_update_mlp(_ptr(x), ldx, M, K1, _ptr(w1t), _rows(w1t, "w1^T", torch.bfloat16), N1, _sf(sf1),
                              _ptr(w2t), _rows(w2t, "w2^T", torch.bfloat16), N2, _sf(sf2), _lib.GTA_BF16 if xb else _lib.GTA_F32_BF16,
                              _ptr(out), _rows(out, "out"), _stream(x.device)), "update_mlp")
    return out


MM_FORM = "rows"  # "rows": gta_update_mm_t (x read once per output); "tile": gta_update_mm 64x64 tiles
MM_ROWS_MIN_M = 0  # smallest M for the row-streaming entry (k_mm_ring / k_mm_rows); below, the
                   # 64x64-tile kernel. With the ring the row form wins at every M measured: GCN Cora's
                   # [2708 x 128].[128 x 64] took the forward 0.093 -> 0.081 ms (profiles/r02_layer_bench_mmrows.log)
_WT_CACHE = {}
# (w, W^T) pairs handed out while a HIP graph is being captured (executor.GraphedRun takes them: the
# graph keeps those W^T tensors alive and refreshes them when a weight changes in place)
_CAPTURED_WT = []


def _mm_splits(M, K, N, dtype=_lib.GTA_F32, dev=None):
    """K slices for gta_update_mm_t_split, as libgta picks them (gta_update_mm_t_splits: about one
    (row group, slice) block per CU for fp32, slices of >= 64 k, only for K >= 256 on few row
    groups; knob mm_split overrides: the knob set attached to dev's current stream, else the calling
    thread's); 1 = no split."""
    st = _stream(dev) if dev is not None and dev.type == "cuda" else None
    return int(check(_L().gta_update_mm_t_splits(M, K, N, dtype, st), "update_mm_t_splits"))


def _transposed(w):
    """W^T [N, K] contiguous, cached per weight tensor object and version (weights are reused on
    every layer call).  The entry holds a weak reference: a freed weight's address can be reused
    by another tensor, so the address alone is never the key."""
    ent = _WT_CACHE.get(id(w))
    if ent is not None and ent[0]() is w and ent[1] == w._version:
        if torch.cuda.is_current_stream_capturing():
            _CAPTURED_WT.append((w, ent[2]))
        return ent[2]
    if len(_WT_CACHE) >= 64:
        _WT_CACHE.clear()
    K, N = w.shape
    per16 = 16 // w.element_size()
    ld = -(-K // per16) * per16  # rows padded to 16 B: the ring GEMM DMAs W^T in 16-B pieces
    wt = w.new_zeros(N, ld)[:, :K]
    wt.copy_(w.t())
    _WT_CACHE[id(w)] = (weakref.ref(w), w._version, wt)
    if torch.cuda.is_current_stream_capturing():
        _CAPTURED_WT.append((w, wt))
    return wt


def tile_nnz(graph, T):
    """int32 [ceil(N/T), n_cols]: edges per (T-row tile, source column), self loops excluded."""
    _need_gpu(graph.indptr)
    nt = -(-graph.n_rows // T)
    counts = torch.zeros(nt, graph.n_cols, dtype=torch.int32, device=graph.device)
    check(_L().gta_tile_nnz(_ptr(graph.indptr), _ptr(graph.indices), graph.n_rows, graph.n_cols, T, _ptr(counts),
                            _stream(graph.device)), "tile_nnz")
    return counts


def synth_alpha(indptr, gen, heads, seed, logit_stream):
    """GAT alpha [nnz, heads] fp32 of a CSR row range (indptr local, from 0) from counter-hashed
    logits keyed by gen[e] * heads + h: per-row softmax with an fp64 edge-order row sum
    (gta_synth_alpha; metric.alpha_rows).  One wave per row, no device-wide scan."""
    _need_gpu(indptr, gen)
    indptr = indptr.to(torch.int64).contiguous()
    gen = gen.to(torch.int64).contiguous()
    n_rows, nnz = indptr.numel() - 1, gen.numel()
    out = torch.empty(nnz, heads, dtype=torch.float32, device=gen.device)
    check(_L().gta_synth_alpha(_ptr(indptr), _ptr(gen), n_rows, nnz, int(heads), int(seed), int(logit_stream), _ptr(out),
                               _stream(gen.device)), "synth_alpha")
    return out


def row_ids(indptr, nnz):
    """int64 [nnz]: the row of every CSR edge (torch.repeat_interleave(arange, degrees) without a
    device-wide scan; gta_row_ids)."""
    _need_gpu(indptr)
    indptr = indptr.to(torch.int64).contiguous()
    out = torch.empty(int(nnz), dtype=torch.int64, device=indptr.device)
    check(_L().gta_row_ids(_ptr(indptr), indptr.numel() - 1, int(nnz), _ptr(out), _stream(indptr.device)), "row_ids")
    return out


_ATTACHED = {}  # raw stream handle -> id of the Tuning whose values it carries (the executor stays eager on them)
_TLS = threading.local()  # per thread: {key: (value before the first set, current value)} of knobs set here


def knob_state():
    """The calling thread's libgta knobs that differ from the values they had before this thread
    first set them, as a sorted tuple of (key, value): part of the executor's HIP-graph cache key.
    Knobs are per thread in libgta, so is this; a knob set back to its old value drops out, so a
    set-then-restore (bench's PMC child, tests) keys the same graphs again instead of recapturing."""
    return getattr(_TLS, "state", ())


def set_debug(key, value):
    """Set a tuning knob of libgta for the CALLING thread (include/gta.h: gta_debug_set)."""
    d = getattr(_TLS, "knobs", None)
    if d is None:
        d = _TLS.knobs = {}
    before = d[key][0] if key in d else get_debug(key)
    check(_L().gta_debug_set(key.encode(), int(value)), "debug_set")
    if int(value) == before:
        d.pop(key, None)
    else:
        d[key] = (before, int(value))
    _TLS.state = tuple(sorted((k, v) for k, (_, v) in d.items()))


def get_debug(key):
    """The calling thread's value of a libgta tuning knob."""
    import ctypes
    v = ctypes.c_int64(0)
    check(_L().gta_debug_get(key.encode(), ctypes.byref(v)), "debug_get")
    return int(v.value)


class Tuning:
    """A libgta knob set scoped to a STREAM (include/gta.h gta_tuning_*): attach(stream) copies
    these values onto the stream, and every call made on it -- from any thread -- then reads them
    instead of the calling thread's knobs (set_debug).  Change a value, attach again to apply it;
    detach(stream) drops the stream's set.  Unknown keys raise GTAError.
    The set is keyed by the raw stream handle: detach before the stream is destroyed (a new stream
    may reuse the handle), and attaching to the null stream (0) governs every default-stream call.
    A Tuning that is garbage-collected detaches the streams still carrying its values (not those
    another Tuning attached to since).
    The executor's automatic HIP-graph replay stays eager on a stream with an attached set."""

    def __init__(self, **knobs):
        self._lib = _L()
        self._h = self._lib.gta_tuning_create()
        if not self._h:
            raise _lib.GTAError("gta_tuning_create failed")
        for k, v in knobs.items():
            self.set(k, v)

    def set(self, key, value):
        check(self._lib.gta_tuning_set(self._h, key.encode(), int(value)), "tuning_set")
        return self

    def get(self, key):
        import ctypes
        v = ctypes.c_int64(0)
        check(self._lib.gta_tuning_get(self._h, key.encode(), ctypes.byref(v)), "tuning_get")
        return int(v.value)

    @staticmethod
    def _ptr(stream):
        """A torch.cuda.Stream, or a raw hipStream_t value (int; 0 = the null stream)."""
        return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)

    def attach(self, stream):
        check(self._lib.gta_tuning_attach(self._ptr(stream), self._h), "tuning_attach")
        _ATTACHED[self._ptr(stream)] = id(self)

    @classmethod
    def detach(cls, stream):
        check(_L().gta_tuning_attach(cls._ptr(stream), None), "tuning_attach")
        _ATTACHED.pop(cls._ptr(stream), None)

    @staticmethod
    def attached(stream):
        """True if a knob set is attached to this stream (torch.cuda.Stream or raw handle)."""
        return Tuning._ptr(stream) in _ATTACHED

    def __del__(self):
        h, self._h = getattr(self, "_h", None), None
        for sp in [sp for sp, owner in list(_ATTACHED.items()) if owner == id(self)]:
            self._lib.gta_tuning_attach(sp, None)  # the stream no longer carries a dead set's values
            _ATTACHED.pop(sp, None)
        if h:
            self._lib.gta_tuning_destroy(h)
