"""Op-local fp64 checks of an executed layer on sampled rows (TEST ORACLE ONLY).

For graphs too large for the whole-graph oracle (Reddit, ogbn-products), every
materialised op output is re-derived in fp64 at a random sample of rows from
the executor's own values of that op's inputs -- recursively through virtual
scatters and fused (never materialised) intermediates -- with the ISA
semantics of isa_ref.  Together the per-op checks cover every kernel launch of
the layer at full size.  On small graphs (every golden stream on Cora) the same
check runs at every row.

Tolerance, per element: |got - exp| <= 1e-5 * sum|terms| + 1e-6, with sum|terms|
the fp64 magnitude sum of the terms the op adds or multiplies, taken op-locally from the same
executor inputs: a gather's sum of |edge values|, |a| + |b| for ADD / SUB, |a * b| and |a / b| for
MUL / DIV, |f(x)| for an SF, sum_k |x_ik| |w_kj| for an MM (bf16 W: x rounded to bf16 as the kernel
rounds it), |x| for a copy.  A value the executor stores in bf16 (GIN's sum handed to the fused MLP,
ABI 10) adds its one RNE rounding, 2^-8 |exp|.
"""
import numpy as np
import torch

from . import isa_ref


class SampledChecker:
    def __init__(self, executor, indptr, indices):
        self.ex = executor
        self.g = executor.g
        self.sem = executor.sem
        self.ip = np.asarray(indptr, np.int64)
        self.ix = np.asarray(indices, np.int64)
        self.tensors = executor.tensors

    def _rows(self, t, idx):
        t2 = t.view(-1, 1) if t.dim() == 1 else t
        return t2[torch.as_tensor(idx, device=t2.device, dtype=torch.long)].double().cpu().numpy()

    def dst_of(self, e):
        return np.searchsorted(self.ip, e, side="right") - 1

    def value_at(self, v, kind, idx):
        """Rows idx (node or edge ids) of an executor value object."""
        from gta_graph_tensor_acclelrator_for_general_gnn_amd import executor as X
        if isinstance(v, X.Lazy):
            v = v.force()
        if isinstance(v, X.NodeT):
            if kind != "node":
                raise TypeError("node value read per edge")
            return self._rows(v.t, idx)
        if isinstance(v, X.EdgeT):
            return self._rows(v.t, idx)
        if isinstance(v, X.Scat):
            rows = self.ix[idx] if v.mode == "src" else self.dst_of(idx)
            return self._rows(v.t, rows)
        if isinstance(v, X.Deferred):
            return self.expected(self.g.ops[v.op], "edge", idx)
        if isinstance(v, tuple) and v[0] == "row":
            r = self._rows(v[1], [0])
            return np.repeat(r, len(idx), axis=0)
        raise TypeError(type(v).__name__)

    def input_at(self, op, slot, kind, idx):
        src = self.g.inputs[op.idx][slot]
        if src.kind == "op":
            return self.value_at(self.ex.values[src.op], kind, idx)
        return self.value_at(self.ex._source(op, slot), kind, idx)

    def expected(self, op, kind, idx):
        """fp64 value of op at rows idx, from its inputs' executor values."""
        return self.expected2(op, kind, idx)[0]

    def _col_edges(self, j):
        """Edges whose source is column j, in CSR order (gather with DIRECTION src, ORDER C)."""
        if getattr(self, "_csc", None) is None:
            perm = np.argsort(self.ix, kind="stable")
            cnt = np.bincount(self.ix, minlength=int(getattr(self.ex.graph, "n_cols", 0) or 0))
            self._csc = (np.concatenate([[0], np.cumsum(cnt)]).astype(np.int64), perm)
        ptr, perm = self._csc
        return perm[ptr[j]:ptr[j + 1]] if j + 1 < len(ptr) else perm[:0]

    def expected2(self, op, kind, idx):
        """(fp64 value, fp64 sum|terms|) of op at rows idx, from its inputs' executor values."""
        idx = np.asarray(idx, np.int64)
        nin = len(self.g.inputs[op.idx])
        if op.type == "scatter":
            rows = self.ix[idx] if op.order == "C" else self.dst_of(idx)
            v = self.input_at(op, 0, "node", rows)
            return v, np.abs(v)
        if op.type == "gather":
            lists = [self._col_edges(r) if op.order == "C" else np.arange(self.ip[r], self.ip[r + 1]) for r in idx]
            edges = np.concatenate(lists) if lists else np.zeros(0, np.int64)
            if edges.size == 0:
                z = np.zeros((len(idx), self.g.ops[op.idx].out_width))
                return z, z.copy()
            vals = self.input_at(op, 0, "edge", edges)  # every sampled row's edges in one read
            seg = np.repeat(np.arange(len(idx)), [len(x) for x in lists])
            out = np.zeros((len(idx), vals.shape[1]))
            mag = np.zeros_like(out)
            np.add.at(out, seg, vals)
            np.add.at(mag, seg, np.abs(vals))
            return out, mag
        k = "edge" if op.type == "applyedge" else "node"
        if op.comp == "MM":
            W = self.tensors[f"w:{op.idx}"].double().cpu().numpy()
            x = self.input_at(op, 0, k, idx)
            if self.tensors[f"w:{op.idx}"].dtype == torch.bfloat16:
                x = torch.from_numpy(x).to(torch.bfloat16).double().numpy()
            return x @ W, np.abs(x) @ np.abs(W)
        if op.comp == "SF":
            v = isa_ref.sf(self.sem.sf_of(op), self.input_at(op, 0, k, idx))
            return v, np.abs(v)
        b = self.sem.bin_of(op)
        ins = [self.input_at(op, s, k, idx) for s in range(nin)]
        extra = self.tensors.get(f"ext:{op.idx}:1")
        if nin == 1 and extra is not None:
            ins.append(self.value_at(self.ex._wrap_ext(extra), k, idx))
        if len(ins) == 1:
            return ins[0], np.abs(ins[0])
        A, B = ins[0], ins[1]
        if b == "RDIV":
            A, B, b = B, A, "DIV"
        v = isa_ref.binop(b, A, B)
        mag = isa_ref.binop("ADD" if b in ("ADD", "SUB") else b, np.abs(A), np.abs(B))
        return v, np.abs(mag)

    def special_rows(self, per_class=2):
        """{class: node ids} checked in every op on top of the random sample: the first
        and last row, the heaviest rows, the lightest non-empty and the empty rows, rows cut into
        several work items (> 256 edges: blocked-plan items; > 512: row-chunk plan slices; > 1024:
        three or more slices), and rows holding edges on both sides of a source-column block
        boundary of every blocked plan the executor's graph built (B blocks of ceil(n_cols / B)
        columns, gta_aggregate_blocked_plan_build)."""
        deg = np.diff(self.ip)
        N = len(deg)
        if N == 0:
            return {}
        out = {"first": np.array([0]), "last": np.array([N - 1])}
        order = np.argsort(deg, kind="stable")
        out["heaviest"] = order[-2 * per_class:][::-1]
        nz = np.flatnonzero(deg > 0)
        out["lightest"] = nz[np.argsort(deg[nz], kind="stable")[:per_class]]
        out["empty"] = np.flatnonzero(deg == 0)[:per_class]
        for name, lo, hi in (("items_256", 256, 512), ("plan_512", 512, 1024), ("plan_1024", 1024, None)):
            m = deg > lo if hi is None else (deg > lo) & (deg <= hi)
            out[name] = np.flatnonzero(m)[:per_class]
        graph = getattr(self.ex, "graph", None)
        n_cols = getattr(graph, "n_cols", N)
        blocks = sorted({k[1] for k in getattr(graph, "_plans", {})
                         if isinstance(k, tuple) and k[0] == "blocked" and k[1] > 1})
        for B in blocks:
            bsize = -(-n_cols // B)
            rows = []
            for b in sorted({bsize, (B // 2) * bsize, (B - 1) * bsize}):
                if not 0 < b < n_cols:
                    continue
                lo_rows = self.dst_of(np.flatnonzero(self.ix == b - 1))
                hi_rows = self.dst_of(np.flatnonzero(self.ix == b))
                both = np.intersect1d(lo_rows, hi_rows)
                rows.extend((both if both.size else hi_rows)[:1])
            out[f"block_edge_B{B}"] = np.asarray(rows, np.int64)
        return {k: np.asarray(v, np.int64) for k, v in out.items() if len(v)}

    def check(self, n_samples=48, seed=0, rtol=None, skip_ops=(), n_gather=128):
        """Returns {op: max err / bound}; raises AssertionError when any element of any checked op
        exceeds the per-element bound of the module docstring (rtol: None = that bound; a number =
        the old normalised max|d| / max|ref| criterion instead).  Node values are checked at
        n_samples random rows (n_gather for gathers, the aggregates) plus every row of
        special_rows(); edge values at n_samples random edges plus the first and last edge of each
        special row (n_samples >= the row count: every row).  The special rows are named in the
        assertion message and kept in self.special; self.detail[op] = (max err, its bound, max
        err / bound, elements checked)."""
        from gta_graph_tensor_acclelrator_for_general_gnn_amd import executor as X
        rng = np.random.default_rng(seed)
        N, E = len(self.ip) - 1, len(self.ix)
        self.special = self.special_rows()
        sp_rows = np.unique(np.concatenate(list(self.special.values()))) if self.special else np.zeros(0, np.int64)
        nz = sp_rows[self.ip[sp_rows + 1] > self.ip[sp_rows]]
        sp_edges = np.unique(np.concatenate([self.ip[nz], self.ip[nz + 1] - 1])) if nz.size else np.zeros(0, np.int64)
        listing = ", ".join(f"{k}={v.tolist()}" for k, v in self.special.items())
        report, self.detail = {}, {}
        for op in self.g.ops:
            if op.idx in skip_ops:
                continue
            v = self.ex.values.get(op.idx)
            if isinstance(v, X.Lazy):  # fused-away intermediate: materialise it to check it too
                v = v.force()
            if not isinstance(v, (X.NodeT, X.EdgeT)):
                continue
            kind = "node" if isinstance(v, X.NodeT) else "edge"
            total = N if kind == "node" else E
            if op.type == "gather" and op.order == "C":
                total = v.t.shape[0]  # one row per source column
            k = n_gather if op.type == "gather" else n_samples
            idx = rng.choice(total, size=min(k, total), replace=False)
            idx = np.unique(np.concatenate([idx, (sp_rows[sp_rows < total] if kind == "node" else sp_edges)]))
            got = self.value_at(v, kind, idx)
            exp, mag = self.expected2(op, kind, idx)
            fin = np.isfinite(exp)
            assert np.array_equal(np.isfinite(got), fin), f"op {op.idx}: non-finite pattern differs ({listing})"
            if not fin.any():
                report[op.idx] = 0.0
                continue
            d = np.abs(got[fin] - exp[fin])
            if rtol is not None:
                scale = np.abs(exp[fin]).max()
                err = float(d.max() / (scale + 1e-30))
                report[op.idx] = err
                assert err <= rtol, (f"op {op.idx} ({op.type}/{op.comp}): normalised max err {err:.2e} over "
                                     f"{idx.size} {kind}s incl. special rows {listing}")
                continue
            bound = 1e-5 * mag[fin] + 1e-6
            if v.t.dtype == torch.bfloat16:  # stored rounded: one RNE rounding to bf16
                bound = bound + 2.0 ** -8 * np.abs(exp[fin])
            ratio = d / bound
            j = int(np.argmax(ratio))
            self.detail[op.idx] = (float(d[j]), float(bound[j]), float(ratio[j]), int(d.size))
            report[op.idx] = float(ratio[j])
            assert ratio[j] <= 1.0, (f"op {op.idx} ({op.type}/{op.comp}): |d| {d[j]:.3e} > bound {bound[j]:.3e} "
                                     f"(1e-5 sum|terms| + 1e-6) over {idx.size} {kind}s incl. special rows {listing}")
        return report


def gin_unrounded_errors(checker, t32, rows):
    """The bf16 GIN layer (configs 'gin-products': x, W5, W7 stored in bf16, every sum in fp32)
    against fp64 evaluated from the UNROUNDED fp32 inputs t32 (workloads.make_tensors with fp32
    dtypes and the same seed: the values the bf16 configuration rounds), at node rows `rows`.
    GIN op graph (vTCAD/GraphOP/genGraphOP.py:97-108; SFs of semantics.py):
        op 2 = sum_{e -> i} x[src(e)] * w_e (w_e = 1, op 1's -1 input)   op 3 = x * (1 + eps)
        op 4 = op 2 + op 3      op 5 = op 4 . W5     op 6 = relu     op 7 = op 6 . W7     op 8 = relu
    Returns {op: (max |d| / max |ref|, max |d| / sum|terms|, elements)} for every op the executor
    holds a value of: the error the bf16 storage choice adds end to end, which the op-local checks
    (inputs rounded as the kernel rounds them) do not see.  SURVEY.md §8c's bound is rtol 2e-2."""
    rows = np.asarray(rows, np.int64)
    ip, ix = checker.ip, checker.ix

    def host(t, idx=None):
        t2 = t.view(-1, 1) if t.dim() == 1 else t
        if idx is not None:
            t2 = t2[torch.as_tensor(idx, device=t2.device, dtype=torch.long)]
        return t2.double().cpu().numpy()

    x_rows = host(t32["x"], rows)
    agg = np.zeros_like(x_rows)
    agg_abs = np.zeros_like(x_rows)
    w_e = t32["ext:1:1"]
    for k, r in enumerate(rows):
        e = np.arange(ip[r], ip[r + 1])
        if e.size:
            xs = host(t32["x"], ix[e]) * host(w_e, e)
            agg[k] = xs.sum(axis=0)
            agg_abs[k] = np.abs(xs).sum(axis=0)
    eps1 = float(host(t32["ext:3:1"]).ravel()[0])
    m3 = x_rows * eps1
    a4 = agg + m3
    w5, w7 = host(t32["w:5"]), host(t32["w:7"])
    z5 = a4 @ w5
    s6 = np.maximum(z5, 0.0)
    z7 = s6 @ w7
    # an SF's error is its input's (relu passes it or drops it): its terms are the GEMM's before it
    m5, m7 = (agg_abs + np.abs(m3)) @ np.abs(w5), np.abs(s6) @ np.abs(w7)
    ref = {2: (agg, agg_abs), 3: (m3, np.abs(m3)), 4: (a4, agg_abs + np.abs(m3)),
           5: (z5, m5), 6: (s6, m5), 7: (z7, m7), 8: (np.maximum(z7, 0.0), m7)}
    out = {}
    for op, (exp, mag) in ref.items():
        v = checker.ex.values.get(op)
        if v is None:
            continue
        got = checker.value_at(v, "node", rows)
        d = np.abs(got - exp)
        out[op] = (float(d.max() / (np.abs(exp).max() + 1e-30)), float((d / (mag + 1e-30)).max()), int(d.size))
    return out
