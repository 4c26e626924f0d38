"""fp64 op-by-op evaluation of a GTA op graph (TEST ORACLE ONLY, see oracle/__init__.py).

Ignores blocks and fusion entirely: every op is evaluated unfused, in the op
graph's data-flow order, with the ISA semantics of oracle/isa_ref.py.  The
data flow (which op feeds which slot) is resolved here from the raw YAML records
(opgraph.records) by oracle/opgraph_ref.py, not taken from the product's
ir.OpGraph resolution; the per-network choices the YAML leaves open (which SF,
GAT op 9's "/", GAT op 10's input patch) come from semantics.Semantics, the
written spec.  All arithmetic here is independent of the product code.
"""
import numpy as np

from . import isa_ref, opgraph_ref


class _OpView:  # what Semantics.sf_of / bin_of read: position and COMP_TYPE
    __slots__ = ("idx", "comp")

    def __init__(self, idx, comp):
        self.idx, self.comp = idx, comp


def _as_operand(t, n, e):
    t = np.asarray(t, np.float64)
    if t.ndim == 1:
        t = t[:, None]
    if t.shape[0] == 1:
        return ("row", t)
    if t.shape[0] == e and t.shape[0] != n:
        return ("edge", t)
    if t.shape[0] == n and t.shape[0] != e:
        return ("node", t)
    return ("edge", t)


def execute_ref(opgraph, sem, indptr, indices, tensors):
    """Returns {op index: ("node"|"edge", float64 array)} for every op."""
    n = len(indptr) - 1
    e = len(indices)
    ip, ix = np.asarray(indptr, np.int64), np.asarray(indices, np.int64)
    vals = {}

    recs = opgraph.records
    patches = getattr(opgraph, "patches", None) or {}
    flow = opgraph_ref.dataflow(recs, patches)

    def src(op, slot):
        kind, ref = flow[op.idx][slot]
        if kind == "op":
            return vals[ref]
        key = f"ext:{op.idx}:{slot}"
        if key in tensors:
            return _as_operand(tensors[key], n, e)
        if kind == "ext":
            raise KeyError(key)
        if op.type == "applyedge":
            return ("edge", np.asarray(tensors["x_edge"], np.float64))
        return ("node", np.asarray(tensors["x"], np.float64))

    def edge_rows(v):
        kind, t = v
        if kind == "edge":
            return t
        if kind == "row":
            return np.broadcast_to(t, (e, t.shape[1]))
        raise TypeError("node value used as an edge operand")

    def node_rows(v):
        kind, t = v
        if kind == "node":
            return t
        if kind == "row":
            return np.broadcast_to(t, (n, t.shape[1]))
        raise TypeError("edge value used as a node operand")

    class _Rec:
        __slots__ = ("idx", "type", "comp", "order")

    for i in opgraph_ref.topo(recs, patches):
        r = recs[i]
        op = _Rec()
        op.idx, op.type, op.comp, op.order = i, r["TYPE"], r.get("COMP_TYPE", "NONE"), r.get("ORDER", "R")
        nin = len(flow[i])
        if op.type == "scatter":
            vals[i] = ("edge", isa_ref.scatter(ip, ix, node_rows(src(op, 0)), "R" if op.order == "R" else "C"))
        elif op.type == "gather":
            vals[i] = ("node", isa_ref.gather_add(ip, edge_rows(src(op, 0)), "C" if op.order == "C" else "R", ix))
        else:
            edge = op.type == "applyedge"
            rows = edge_rows if edge else node_rows
            kind = "edge" if edge else "node"
            if op.comp == "MM":
                W = np.asarray(tensors[f"w:{i}"], np.float64)
                X = rows(src(op, 0))
                if W.dtype != np.float64:
                    W = W.astype(np.float64)
                vals[i] = (kind, X @ W)
            elif op.comp == "SF":
                vals[i] = (kind, isa_ref.sf(sem.sf_of(_OpView(i, op.comp)), rows(src(op, 0))))
            else:
                b = sem.bin_of(_OpView(i, op.comp))
                ins = [src(op, s) for s in range(nin)]
                if len(ins) == 1 and f"ext:{i}:1" in tensors:
                    ins.append(_as_operand(tensors[f"ext:{i}:1"], n, e))
                if len(ins) == 1:
                    vals[i] = (kind, rows(ins[0]).copy())
                    continue
                A, B = rows(ins[0]), rows(ins[1])
                if b == "RDIV":
                    A, B, b = B, A, "DIV"
                vals[i] = (kind, isa_ref.binop(b, A, B))
    return vals
