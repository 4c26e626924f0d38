"""Op-local fp64 checks of an executed layer on sampled rows (TEST ORACLE ONLY).

For graphs too large for the whole-graph oracle (Reddit, ogbn-products), every
materialised op output is re-derived in fp64 at a random sample of rows from
the executor's own values of that op's inputs -- recursively through virtual
scatters and fused (never materialised) intermediates -- with the ISA
semantics of isa_ref.  Together the per-op checks cover every kernel launch of
the layer at full size.
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
        idx = np.asarray(idx, np.int64)
        nin = len(self.g.inputs[op.idx])
        if op.type == "scatter":
            rows = self.ix[idx] if op.order == "C" else self.dst_of(idx)
            return self.input_at(op, 0, "node", rows)
        if op.type == "gather":
            out = []
            for r in idx:
                e = np.arange(self.ip[r], self.ip[r + 1])
                vals = self.input_at(op, 0, "edge", e) if len(e) else None
                out.append(vals.sum(0) if vals is not None else None)
            width = next((o.shape[0] for o in out if o is not None), None)
            if width is None:
                width = self.g.ops[op.idx].out_width
            return np.stack([o if o is not None else np.zeros(width) for o in out])
        k = "edge" if op.type == "applyedge" else "node"
        if op.comp == "MM":
            W = self.tensors[f"w:{op.idx}"].double().cpu().numpy()
            x = self.input_at(op, 0, k, idx)
            if self.tensors[f"w:{op.idx}"].dtype == torch.bfloat16:
                x = torch.from_numpy(x).to(torch.bfloat16).double().numpy()
            return x @ W
        if op.comp == "SF":
            return isa_ref.sf(self.sem.sf_of(op), self.input_at(op, 0, k, idx))
        b = self.sem.bin_of(op)
        ins = [self.input_at(op, s, k, idx) for s in range(nin)]
        extra = self.tensors.get(f"ext:{op.idx}:1")
        if nin == 1 and extra is not None:
            ins.append(self.value_at(self.ex._wrap_ext(extra), k, idx))
        if len(ins) == 1:
            return ins[0]
        A, B = ins[0], ins[1]
        if b == "RDIV":
            A, B, b = B, A, "DIV"
        return isa_ref.binop(b, A, B)

    def check(self, n_samples=48, seed=0, rtol=2e-4, skip_ops=()):
        """Returns {op: normalised max error}; raises AssertionError beyond rtol."""
        from gta_graph_tensor_acclelrator_for_general_gnn_amd import executor as X
        rng = np.random.default_rng(seed)
        N, E = len(self.ip) - 1, len(self.ix)
        report = {}
        for op in self.g.ops:
            if op.idx in skip_ops:
                continue
            v = self.ex.values.get(op.idx)
            if isinstance(v, X.Lazy):  # fused-away intermediate: materialise it to check it too
                v = v.force()
            if not isinstance(v, (X.NodeT, X.EdgeT)):
                continue
            kind = "node" if isinstance(v, X.NodeT) else "edge"
            idx = rng.choice(N if kind == "node" else E, size=min(n_samples, N if kind == "node" else E),
                             replace=False)
            got = self.value_at(v, kind, idx)
            exp = self.expected(op, kind, idx)
            fin = np.isfinite(exp)
            assert np.array_equal(np.isfinite(got), fin), f"op {op.idx}: non-finite pattern differs"
            scale = np.abs(exp[fin]).max() if fin.any() else 0.0
            err = float(np.abs(got[fin] - exp[fin]).max() / (scale + 1e-30)) if fin.any() else 0.0
            report[op.idx] = err
            assert err <= rtol, f"op {op.idx} ({op.type}/{op.comp}): normalised max err {err:.2e}"
        return report
