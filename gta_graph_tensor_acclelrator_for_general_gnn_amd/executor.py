"""HIP executor for GTA instruction streams -- the drop-in for the reference's simulate().

Reference boundary: `interpret()` writes Results/Insts/<net>-<ds>-<layer>-<map>.yaml
(code/interpreter.py:805-849) and `simulate(tile_size_list, dataset, network,
layer, isReorder, isSinput) -> (cycles, rw)` replays it as a cycle model
(code/simulator.py:370-502).  `execute()` takes the same leading arguments,
reads the same two YAML files, and runs the stream on real device tensors:

  * blocks run in dependency order (the stream's block order is the
    compiler's component sort, code/compiler.py:60, not a schedule);
  * inside a block, ops run in data-flow order and are mapped onto libgta
    kernels following the stream's own fusion decisions:
      - a scatter whose FETCH was removed (fuse_fetch, code/interpreter.py:764-802)
        is never materialised: its consumer gathers rows by index
        (GTA_IDX_SRC for ORDER C, GTA_IDX_DST for ORDER R);
      - a COMP_MUL_COMP_ADD / COMP_MM_COMP_ADD pair (inst_fusion_x2, :575-636;
        hardware_info.yaml Inst_fused) becomes one aggregate kernel (MUL) or
        an edge GEMM + gather (MM);
      - scatters with a STORE_E are materialised with gta_scatter;
  * numerics the YAML leaves open come from semantics.py.
Returns ExecResult(values per op, outputs of sink ops, elapsed_s, alg_bytes).
"""
import os
import time
import weakref

import numpy as np
import torch

from . import ir, ops
from .semantics import Semantics


# [W | W_s1 | ...] column concatenations of sibling weights, cached per source-weight objects and
# versions (weak references: an address alone is never the key), so a forward reuses one tensor --
# and ops._transposed its W^T -- instead of a cat + W^T per call.  Entries are only made outside a
# HIP graph capture; a capture that reads one records (sources, concatenation) in _CAPTURED_WCAT,
# and GraphedRun re-concatenates it when a source weight changes in place.
_WCAT = {}
_CAPTURED_WCAT = []


def _sibling_cat(srcs):
    key = tuple(id(w) for w in srcs)
    vers = tuple(w._version for w in srcs)
    capturing = srcs[0].is_cuda and torch.cuda.is_current_stream_capturing()
    ent = _WCAT.get(key)
    if ent is not None and ent[1] == vers and all(r() is w for r, w in zip(ent[0], srcs)):
        if capturing:
            _CAPTURED_WCAT.append((list(srcs), ent[2]))
        return ent[2]
    Wc = torch.cat(srcs, dim=1).contiguous()
    if not capturing:  # a tensor from the capture's private pool is never handed to eager runs
        if len(_WCAT) >= 64:
            _WCAT.clear()
        _WCAT[key] = (tuple(weakref.ref(w) for w in srcs), vers, Wc)
    return Wc


class NodeT:
    __slots__ = ("t",)

    def __init__(self, t):
        self.t = t


class EdgeT:
    __slots__ = ("t",)

    def __init__(self, t):
        self.t = t


class Scat:
    """A scatter kept virtual: edge e reads row idx(e) of node tensor t (mode 'src' or 'dst').

    On a destination-row shard (distributed.RowShard) a source-side table is first this rank's
    row block `local`; `fill` exchanges it into the full table (one all-gather) the first time a
    kernel indexes it through `t`.  Node-side GEMMs of the scatter run on `local` and keep `fill`,
    so the exchange carries the GEMM's output, not its input.  `own` (a replicated model input)
    returns this scatter's whole table without an exchange; derived scatters do not inherit it."""
    __slots__ = ("local", "mode", "fill", "own", "_full")

    def __init__(self, t, mode, fill=None, own=None):
        self.local, self.mode, self.fill, self.own, self._full = t, mode, fill, own, None

    @property
    def t(self):
        if self.fill is None and self.own is None:
            return self.local
        if self._full is None:
            self._full = self.own() if self.own is not None else self.fill(self.local)
        return self._full


class Deferred:
    """An applyedge MUL/MM fused into its gather consumer (evaluated by the gather)."""
    __slots__ = ("op",)

    def __init__(self, op):
        self.op = op


class Lazy:
    """An intermediate whose only consumer was fused with it (e.g. an SF post-op);
    computed on demand if anything else ever asks for it."""
    __slots__ = ("fn", "v")

    def __init__(self, fn):
        self.fn, self.v = fn, None

    def force(self):
        if self.v is None:
            self.v = self.fn()
        return self.v


class ExecResult:
    """Real outputs + measured time, and the reference's modelled (cycles, rw) for the same stream."""

    def __init__(self, values, outputs, elapsed_s, alg_bytes, launches):
        self.values, self.outputs = values, outputs
        self.elapsed_s, self.alg_bytes, self.launches = elapsed_s, alg_bytes, launches
        self.model_cycles = None  # simulate()'s first result (code/simulator.py:502), if requested
        self.model_rw = None      # simulate()'s second result: modelled DRAM bytes
        self.trace = None         # Chrome trace events when execute(..., trace=...) asked for them
        self.model_insts = None   # per-instruction model (costmodel.per_instruction), when a model was asked for
        self.model_spans = None   # model="full": (block, index) -> [first start, first cost, last end] cycles
        self.model_arch = None    # (architecture_name, flexible) of a vTCAD-style call

    def simulate_tuple(self):
        """(cycles, rw) in the shape the reference's simulate() returns."""
        return self.model_cycles, self.model_rw

    def __repr__(self):
        return (f"ExecResult(outputs={sorted(self.outputs)}, elapsed_s={self.elapsed_s:.6f}, "
                f"alg_bytes={self.alg_bytes}, launches={self.launches}, model=({self.model_cycles}, "
                f"{self.model_rw}))")


def _forced(v):
    return v.force() if isinstance(v, Lazy) else v


EDGE_EXPR = True  # Executor.edge_expr's default (gta_aggregate_expr for applyedge trees); False: unfused (A/B)

MAX_MATERIALIZE_BYTES = 96 << 30  # refuse to materialise a single edge tensor larger than this


class Executor:
    def __init__(self, opgraph, stream, graph, tensors, semantics=None, plan_chunk=512, dist=None):
        self.g = opgraph
        # dist (distributed.Comm): node tensors are this rank's row block; gathers are
        # reduce-scattered to it and dst-side scatters all-gather it (distributed.py)
        self.dist = dist
        self.n_nodes = dist.n_local if dist is not None else (graph.n_rows if graph is not None else 0)
        self.stream = stream
        self.graph = graph
        self.tensors = dict(tensors)
        self.sem = semantics or Semantics()
        self.plan_chunk = plan_chunk
        self.values = {}
        self._nmm = {}  # node GEMMs of _node_mm in this run: (op, x) -> x W
        self.alg_bytes = 0
        self.launches = 0
        # trace: per evaluated op, device time (HIP events), algorithmic bytes and launches, as
        # Chrome trace events in the reference's schema (vTCAD/code/simulator.py:360-382)
        self.trace = False
        self.trace_events = None
        # execution-level fusion beyond the stream's (results bitwise unchanged):
        #   elide_scatter_stores: a STORE_E'd scatter read back by a later block is read by index
        #   fuse_sf: an SF whose producer feeds only it runs as the producer's post-op
        self.elide_scatter_stores = True
        self.fuse_sf = True
        #   fuse_mlp: MM -> SF -> MM -> SF chains of node GEMMs (GIN's MLP) as one gta_update_mlp launch
        self.fuse_mlp = FUSE_MLP
        self.mlp_bf16_sum = MLP_BF16_SUM
        # weighted/unweighted SpMM aggregates whose gathered table exceeds the chip's L2
        # run column-blocked (L2-resident slices) when the shape allows it
        self.blocked_min_table_bytes = 32 << 20
        self.blocked_blocks = "auto"  # ops.BlockedPlan.auto_blocks, or a fixed count (0 = never)
        self.consumers = {i: [] for i in range(len(opgraph))}
        for i in range(len(opgraph)):
            for src in opgraph.inputs[i]:
                if src.kind == "op":
                    self.consumers[src.op].append(i)
        #   fuse_softmax: GAT's score -> SF -> per-row sum (-> divide) chain runs as one
        #   gta_edge_softmax launch (results equal to fp32 rounding, not bitwise)
        # column shards: per-row sums span ranks (unfused ops + exchanges); row shards own whole rows
        self.fuse_softmax = dist is None or dist.local_rows or dist.s.world == 1
        self.softmax = self._match_softmax()
        #   fuse_attention: the softmax chain's alpha (or v) * scatter_C(x) -> gather runs as one
        #   column-blocked gta_gat_aggregate_blocked (no [E, heads] tensor); attention_blocks
        #   None = ops.BlockedPlan.auto_blocks (used when >= 4), or a fixed block count
        self.fuse_attention = True
        self.attention_blocks = None
        self.attn = self._match_attention()
        self._att_state = {}
        #   mm_first: a gather whose only consumer is a narrowing applynode MM is executed as
        #   MM-then-aggregate (sum_e w_e x_src) W == sum_e w_e (x W)_src -- the layer's output
        #   to fp32 rounding, the gather's own value computed only if something asks for it
        self.mm_first = True
        self.reorder = self._match_mm_first()
        #   and through two hops (SGC: gather -> scatter C -> MUL -> gather -> MM): A (A x) W == A (A (x W)),
        #   both aggregates at the narrow width; the first gather's value computed only if asked for
        self.two_hop = self._match_two_hop() if dist is None else {}
        #   node_mm: an applyedge MM of a scatter runs on the node tensor, (x W)[r(e)] == x[r(e)] W
        #   (bitwise: the same dot product per row), and stays a virtual scatter of x W
        #   mm_pushdown: MM(scatter a (+) scatter b) == (a W)[r(e)] (+) (b W)[r'(e)] (DGN op 2 -> 3),
        #   to fp32 rounding; the [E, F_in] sum is never built
        self.node_mm = True
        self.mm_pushdown = True
        #   sibling_mm: applynode MMs that multiply the same node tensor run as ONE GEMM over the
        #   concatenated weights (x read once; e.g. GraphSAGE's x W3 and x W4, GAT's scores W1, W2)
        self.sibling_mm = True
        self.pushdown = self._match_pushdown()
        #   gather_acc: applynode ADD(gather G, node op T), each the other's only reader (GIN op 4:
        #   agg + (1+eps) x), runs as the aggregate accumulating into T's fresh output buffer:
        #   T + sum == sum + T bitwise, and the ADD pass over [N, F] disappears.  G and T stay
        #   available (recomputed on demand).
        self.gather_acc = dist is None or dist.local_rows or dist.s.world == 1
        self.gacc = self._match_gather_acc()
        self.gacc_t = {T: A for A, (_, _, T) in self.gacc.items()}  # node op T -> its ADD consumer
        #   edge_expr: a gather R whose edge value is a tree of applyedge ops (ADD / SUB / MUL / DIV,
        #   SF post-ops, a pushed-down MM), each read only by the next, runs as one
        #   gta_aggregate_expr: no [E, F] tensor for any op of the tree, bitwise the unfused ops and
        #   gather (DGN ops 2-8, PNA ops 5-8).  The tree's ops stay available, computed unfused if read.
        self.edge_expr = EDGE_EXPR
        self.expr = self._match_edge_expr()
        self.expr_nodes = {i for e in self.expr.values() for i in e["nodes"]}

    # ---------------------------------------------------------------- inputs
    def _ext(self, op, slot):
        return self.tensors.get(f"ext:{op.idx}:{slot}")

    def _source(self, op, slot):
        src = self.g.inputs[op.idx][slot]
        if src.kind == "op":
            if src.op not in self.values:
                raise RuntimeError(f"op {op.idx} reads op {src.op} before it was produced")
            v = self.values[src.op]
            return v.force() if isinstance(v, Lazy) else v
        t = self._ext(op, slot)
        if src.kind == "ext":
            if t is None:
                raise KeyError(f"op {op.idx} slot {slot}: external input 'ext:{op.idx}:{slot}' not given")
            return self._wrap_ext(t, op)
        if t is not None:  # explicit override of the model input for this slot
            return self._wrap_ext(t, op)
        if op.type == "applyedge":
            t = self.tensors.get("x_edge")
            if t is None:
                raise KeyError(f"edge op {op.idx} reads the model input: give 'x_edge' or 'ext:{op.idx}:{slot}'")
            return EdgeT(t)
        return NodeT(self.tensors["x"])

    def _wrap_ext(self, t, op=None):
        if t.dim() == 1:
            t = t.view(-1, 1)
        if op is not None and op.type in ("scatter", "applynode") and t.shape[0] == self.n_nodes \
                and t.shape[0] != 1:  # N == E (e.g. an empty row shard): these ops read node rows
            return NodeT(t)
        if t.shape[0] == self.graph.nnz and t.shape[0] != self.n_nodes:
            return EdgeT(t)
        if t.shape[0] == 1:
            return ("row", t)
        if t.shape[0] == self.n_nodes and t.shape[0] != self.graph.nnz:
            return NodeT(t)
        return EdgeT(t)  # ambiguous N == E: edge tensor

    def _inputs(self, op):
        return [self._source(op, s) for s in range(len(self.g.inputs[op.idx]))]

    # ---------------------------------------------------------- materialise
    def _edge_operand(self, v):
        """-> (tensor, mode, broadcast_row) usable by apply_edge / aggregate."""
        if isinstance(v, Deferred):
            v = self._materialize_deferred(v)
        if isinstance(v, EdgeT):
            return v.t, "edge", False
        if isinstance(v, Scat):  # (a bf16 node table is widened: the element-wise kernels are fp32)
            return (v.t if v.t.dtype == torch.float32 else v.t.float()), v.mode, False
        if isinstance(v, tuple) and v[0] == "row":
            return v[1], "edge", True
        raise TypeError(f"not an edge operand: {type(v).__name__}")

    def _to_edge_tensor(self, v):
        if isinstance(v, EdgeT):
            return v.t
        if isinstance(v, Scat):
            nbytes = self.graph.nnz * v.t.shape[1] * v.t.element_size()
            if nbytes > MAX_MATERIALIZE_BYTES:
                raise MemoryError(f"stream materialises a {nbytes / 2**30:.0f} GiB edge tensor (scatter not fused "
                                  "with its consumer); choose a fusion partition that keeps it virtual")
            self._count(self.graph.nnz * v.t.shape[1] * 4 * 2 + self.graph.nnz * 4)
            t = v.t if v.t.dtype == torch.float32 else v.t.float()  # edge tensors are fp32 (exact widening)
            return ops.scatter(self.graph, t, "C" if v.mode == "src" else "R")
        if isinstance(v, Deferred):
            return self._materialize_deferred(v).t
        raise TypeError(type(v).__name__)

    def _materialize_deferred(self, d):
        op = self.g.ops[d.op]
        v = self._eval_applyedge(op)
        self.values[d.op] = v
        return v

    def _count(self, nbytes):
        self.alg_bytes += int(nbytes)
        self.launches += 1

    # ------------------------------------------------------- edge softmax
    def _match_softmax(self):
        """GAT edge-softmax chains keyed by their score op A (vTCAD/GraphOP/genGraphOP.py:51-60):
            A = applyedge ADD(scatter R(a), scatter C(b));  V = applyedge SF(A);  G = gather R(V)
          original (ops 6,7,8,10,9): D = applyedge V / scatter R(G)  -> alpha, one launch
          trans    (ops 6,8,9):      V and G from one launch (V's other consumer aggregates it)"""
        ops_, ins, cons = self.g.ops, self.g.inputs, self.consumers

        def only(i):  # the single consumer of op i, or None
            return cons[i][0] if len(cons[i]) == 1 else None

        found = {}
        for A in ops_:
            if A.type != "applyedge" or A.comp != "ADD" or len(ins[A.idx]) != 2:
                continue
            srcs = [x.op for x in ins[A.idx] if x.kind == "op"]
            if len(srcs) != 2:
                continue
            orders = sorted(ops_[i].order for i in srcs if ops_[i].type == "scatter")
            if orders != ["C", "R"] or self.sem.bin_of(A) != "ADD":
                continue
            v = only(A.idx)
            if v is None or ops_[v].type != "applyedge" or ops_[v].comp != "SF":
                continue
            gs = [c for c in cons[v] if ops_[c].type == "gather" and ops_[c].order == "R"]
            if len(gs) != 1:
                continue
            G = gs[0]
            pat = {"A": A.idx, "V": v, "G": G, "D": None}
            S = only(G)
            if S is not None and ops_[S].type == "scatter" and ops_[S].order == "R":
                D = only(S)
                if D is not None and set(cons[v]) == {G, D} and ops_[D].type == "applyedge":
                    dins = [x.op if x.kind == "op" else None for x in ins[D]]
                    b = self.sem.bin_of(ops_[D])
                    if (b == "DIV" and dins == [v, S]) or (b == "RDIV" and dins == [S, v]):
                        pat["D"], pat["S"] = D, S
            found[A.idx] = pat
        return found

    def _match_mm_first(self):
        """{gather G: MM op M} for G -> M with M the only consumer, narrowing the width, and G
        reading a scatter C directly or through a (weight) MUL (GraphSAGE / GCN layer 1)."""
        found = {}
        for G in self.g.ops:
            if G.type != "gather" or G.order != "R" or len(self.consumers[G.idx]) != 1:
                continue
            M = self.g.ops[self.consumers[G.idx][0]]
            if M.type != "applynode" or M.comp != "MM" or len(self.g.inputs[M.idx]) != 1:
                continue
            if not (M.out_width and G.out_width and M.out_width < G.out_width):
                continue
            src = self.g.inputs[G.idx][0]
            if src.kind != "op":
                continue
            P = self.g.ops[src.op]
            if P.type == "applyedge" and P.comp == "MUL":
                scat = [x.op for x in self.g.inputs[P.idx] if x.kind == "op" and self.g.ops[x.op].type == "scatter"]
                if len(scat) != 1 or self.g.ops[scat[0]].order != "C":
                    continue
            elif not (P.type == "scatter" and P.order == "C"):
                continue
            found[G.idx] = M.idx
        return found

    def _match_two_hop(self):
        """{first gather G1: second gather G2} for G1 -> scatter C -> [MUL by an edge weight] -> G2 with
        G2 in reorder (its narrowing MM), each intermediate read only by the next op, and G1 of the
        form mm_first takes (a scatter C of a node tensor, directly or through a weight MUL)."""
        ops_, ins, cons = self.g.ops, self.g.inputs, self.consumers
        found = {}
        for G2 in self.reorder:
            P = ops_[ins[G2][0].op]
            if P.type == "scatter":
                S = P
            else:
                sc = [x.op for x in ins[P.idx] if x.kind == "op" and ops_[x.op].type == "scatter"]
                if len(sc) != 1 or cons[sc[0]] != [P.idx]:
                    continue
                S = ops_[sc[0]]
            if S.order != "C" or not ins[S.idx] or ins[S.idx][0].kind != "op":
                continue
            G1 = ops_[ins[S.idx][0].op]
            if G1.type != "gather" or G1.order != "R" or G1.comp != "ADD" or cons[G1.idx] != [S.idx]:
                continue
            src = ins[G1.idx][0]
            if src.kind != "op":
                continue
            P1 = ops_[src.op]
            if P1.type == "applyedge" and P1.comp == "MUL":
                sc1 = [x.op for x in ins[P1.idx] if x.kind == "op" and ops_[x.op].type == "scatter"]
                if len(sc1) != 1 or ops_[sc1[0]].order != "C":
                    continue
            elif not (P1.type == "scatter" and P1.order == "C"):
                continue
            found[G1.idx] = G2
        return found

    def _match_pushdown(self):
        """{applyedge ADD of two scatters: its only consumer, a single-input applyedge MM}."""
        found = {}
        for op in self.g.ops:
            if op.type != "applyedge" or op.comp != "ADD" or len(self.g.inputs[op.idx]) != 2:
                continue
            srcs = [x.op for x in self.g.inputs[op.idx] if x.kind == "op"]
            if len(srcs) != 2 or any(self.g.ops[i].type != "scatter" for i in srcs):
                continue
            cons = self.consumers[op.idx]
            if len(cons) != 1:
                continue
            m = self.g.ops[cons[0]]
            if m.type == "applyedge" and m.comp == "MM" and len(self.g.inputs[m.idx]) == 1 \
                    and self.sem.bin_of(op) == "ADD":
                found[op.idx] = m.idx
        return found

    def _match_edge_expr(self):
        """{gather G: plan} for a gather R (ADD) of an applyedge tree that gta_aggregate_expr's shapes
        cover.  plan: shape, swap, bins, sfs, leaves ((op, slot) of a computed operand, or ("pmm", MM
        op, k): the k-th scatter of a pushed-down MM's sum, multiplied on its node rows) and nodes (the
        tree's ops, deferred until G runs).  Trees the existing fusions take are left to them: a lone
        MUL / MM (the weighted aggregate), the attention chains, the GIN self-term gathers."""
        ops_, ins, cons = self.g.ops, self.g.inputs, self.consumers
        att = set(self.attn)
        for pat in self.softmax.values():
            att.update(i for i in (pat["A"], pat["V"], pat["D"]) if i is not None)
        acc_g = {g for g, _, _ in self.gacc.values()}

        def node(i):  # -> ("bin", bin, sf, left, right, ops) | ("leaf", ref) | None (not coverable)
            o = ops_[i]
            if o.type != "applyedge" or i in att:
                return None
            if o.comp == "SF":
                if len(ins[i]) != 1 or ins[i][0].kind != "op" or cons[ins[i][0].op] != [i]:
                    return None
                c = node(ins[i][0].op)
                if c is None or c[0] != "bin" or c[2] is not None or c[1] == "PMM":
                    return None  # an SF on a pushed-down MM acts on the sum: not this tree
                return ("bin", c[1], self.sem.sf_of(o), c[3], c[4], c[5] + [i])
            if o.comp == "MM":
                src = ins[i][0] if len(ins[i]) == 1 else None
                if src is None or src.kind != "op" or self.pushdown.get(src.op) != i:
                    return None
                return ("bin", "PMM", None, ("leaf", ("pmm", i, 0)), ("leaf", ("pmm", i, 1)), [i])
            if o.comp not in ("ADD", "SUB", "MUL", "DIV") or len(ins[i]) != 2:
                return None
            b = self.sem.bin_of(o)
            kids = []
            for slot, x in enumerate(ins[i]):
                sub = None
                if x.kind == "op" and cons[x.op] == [i] and ops_[x.op].type == "applyedge":
                    sub = node(x.op)
                kids.append(sub if sub is not None else ("leaf", (i, slot)))
            if b == "RDIV":
                b, kids = "DIV", kids[::-1]
            if b not in ("ADD", "SUB", "MUL", "DIV"):
                return None
            return ("bin", b, None, kids[0], kids[1], [i])

        def leafy(t):
            return t[0] == "bin" and t[3][0] == "leaf" and t[4][0] == "leaf"

        def b_of(t):
            return "ADD" if t[1] == "PMM" else t[1]

        found = {}
        for G in ops_:
            if G.type != "gather" or G.order != "R" or G.comp != "ADD" or G.idx in acc_g:
                continue
            src = ins[G.idx][0] if len(ins[G.idx]) == 1 else None
            if src is None or src.kind != "op" or cons[src.op] != [G.idx]:
                continue
            t = node(src.op)
            if t is None:
                continue
            L, R = t[3], t[4]
            if leafy(t):
                if t[1] in ("MUL", "PMM") and t[2] is None:
                    continue  # the weighted aggregate / the pushed-down MM's own path
                e = dict(shape=1, swap=False, bins=[b_of(t)], sfs=[t[2]], leaves=[L[1], R[1]], nodes=t[5])
            elif leafy(L) and R[0] == "leaf":
                e = dict(shape=2, swap=False, bins=[b_of(L), t[1]], sfs=[L[2], t[2]], leaves=[L[3][1], L[4][1], R[1]],
                         nodes=L[5] + t[5])
            elif L[0] == "leaf" and leafy(R):
                e = dict(shape=2, swap=True, bins=[b_of(R), t[1]], sfs=[R[2], t[2]], leaves=[R[3][1], R[4][1], L[1]],
                         nodes=R[5] + t[5])
            elif leafy(L) and leafy(R):
                e = dict(shape=3, swap=False, bins=[b_of(L), b_of(R), t[1]], sfs=[L[2], R[2], t[2]],
                         leaves=[L[3][1], L[4][1], R[3][1], R[4][1]], nodes=L[5] + R[5] + t[5])
            else:
                continue
            found[G.idx] = e
        return found

    def _eval_edge_expr(self, G):
        """G's value from one gta_aggregate_expr launch, or None (then the tree runs unfused)."""
        e = self.expr[G.idx]
        for i in e["nodes"]:
            raw = self.values.get(i)
            if not (isinstance(raw, Lazy) and raw.v is None):
                return None
        operands, gathered = [], 0
        for ref in e["leaves"]:
            if ref[0] == "pmm":
                mm = self.g.ops[ref[1]]
                v = self._source(self.g.ops[self.g.inputs[mm.idx][0].op], ref[2])
                if not isinstance(v, Scat):
                    return None
                v = self._node_mm(mm, v)
            else:
                v = self._source(self.g.ops[ref[0]], ref[1])
            if isinstance(v, Scat):
                operands.append((v.t if v.t.dtype == torch.float32 else v.t.float(), v.mode))
                gathered += v.mode == "src"
            elif isinstance(v, EdgeT):
                operands.append((v.t, "edge"))
                gathered += 1
            elif isinstance(v, tuple) and v[0] == "row":
                operands.append((v[1], "row"))
            else:
                return None
        F = operands[0][0].shape[1]
        if any(t.shape[1] != F or t.dtype != torch.float32 for t, _ in operands):
            return None
        y = ops.aggregate_expr(self.graph, e["shape"], operands, e["bins"], e["sfs"], e["swap"], plan=self._plan())
        if y is None:
            return None
        for mm in {ref[1] for ref in e["leaves"] if ref[0] == "pmm"}:
            # a pushed-down MM read later is the pushed-down product, as the unfused run forms it,
            # whether or not its sum's value has been asked for in between
            mop, add = self.g.ops[mm], self.g.inputs[mm][0].op
            self.values[mm] = Lazy(lambda mop=mop, add=add: self._pushdown_mm(mop, add))
        n, E = self.graph.n_rows, self.graph.nnz
        self._count(E * (4 + 4 * F * gathered) + n * (8 + 4 * F))
        return NodeT(self.dist.reduce_rows(y) if self.dist is not None else y)

    def _match_gather_acc(self):
        """{applynode ADD A: (gather G, slot of T, node op T)} for A = ADD(G, T) where A is G's and T's
        only consumer, T a two-operand applynode ADD/MUL/DIV/SUB (so its output is a tensor it
        allocated itself) and A carries no SF post-op."""
        found = {}
        for A in self.g.ops:
            ins = self.g.inputs[A.idx]
            if A.type != "applynode" or A.comp != "ADD" or len(ins) != 2 or any(x.kind != "op" for x in ins):
                continue
            if self.sem.bin_of(A) != "ADD":
                continue
            kinds = [self.g.ops[x.op].type for x in ins]
            if sorted(kinds) != ["applynode", "gather"] or ins[0].op == ins[1].op:
                continue
            gs = 0 if kinds[0] == "gather" else 1
            G, T = self.g.ops[ins[gs].op], self.g.ops[ins[1 - gs].op]
            if G.order != "R" or self.consumers[G.idx] != [A.idx] or self.consumers[T.idx] != [A.idx]:
                continue
            if T.comp not in ("ADD", "MUL") or len(self.g.inputs[T.idx]) != 2:
                continue
            cons = self.consumers[A.idx]
            if len(cons) == 1 and self.g.ops[cons[0]].comp == "SF" and self.g.ops[cons[0]].type == "applynode":
                continue  # keep A's SF post-op fusion
            found[A.idx] = (G.idx, 1 - gs, T.idx)
        return found

    def _self_term(self, top):
        """(x, s) when node op T = applynode MUL(x, s) of a node tensor x by a one-element scalar s
        (GIN op 3: (1 + eps) x): the aggregate can form T itself (gta_aggregate_self).  Else None."""
        if top.type != "applynode" or top.comp != "MUL" or self._binary(top) != "MUL":
            return None
        ins = self._inputs(top)
        if len(ins) == 1:
            extra = self._ext(top, 1)
            ins = ins + ([self._wrap_ext(extra)] if extra is not None else [])
        if len(ins) != 2:
            return None
        xs = [z for z in ins if isinstance(z, NodeT)]
        rows = [z for z in ins if isinstance(z, tuple) and z[0] == "row"]
        if len(xs) != 1 or len(rows) != 1 or rows[0][1].numel() != 1 or rows[0][1].dtype != torch.float32:
            return None
        return xs[0].t, rows[0][1]

    def _eval_gather_acc(self, A, out_dtype=torch.float32):
        """A = ADD(G, T) as G's aggregate accumulated into T's buffer; None if G's form cannot
        accumulate (then A runs unfused).  When T = x * s (a scalar) and T was left unformed, the
        aggregate forms it in its epilogue instead (no [N, F] T written and read back); only that
        form takes out_dtype bf16 (A stored rounded, for the fused MLP that reads it)."""
        G, slot_t, T = self.gacc[A.idx]
        raw = self.values.get(G)
        if not (isinstance(raw, Lazy) and raw.v is None):
            return None
        tv = self.values.get(T)
        if isinstance(tv, Lazy) and tv.v is None:
            st = self._self_term(self.g.ops[T])
            y = self._eval_gather(self.g.ops[G], self_term=st, out_dtype=out_dtype) if st is not None else None
            if y is not None:
                return y  # T stays unformed: recomputed by its own kernel if something reads it
        if out_dtype != torch.float32:
            return None
        t = self._source(A, slot_t)
        if not isinstance(t, NodeT) or t.t.dtype != torch.float32 or not t.t.is_contiguous():
            return None
        y = self._eval_gather(self.g.ops[G], acc=t.t)
        if y.t.data_ptr() != t.t.data_ptr():  # G's form computed a fresh tensor: add it as the ADD would
            raw.v = y
            return None
        top = self.g.ops[T]
        self.values[T] = Lazy(lambda: self._eval_applynode(top))  # T's buffer now holds A
        return y

    def _node_mm(self, op, v, post_sf=None):
        """applyedge MM of a virtual scatter: the GEMM runs over the node rows, the result stays virtual.
        The two scatters of one node table under one MM (DGN op 3's x[src] + x[dst]) share a GEMM."""
        W = self.tensors[f"w:{op.idx}"]
        x, W = self._mm_dtypes(v.local, W)
        if W.shape[0] != x.shape[1]:
            raise ValueError(f"op {op.idx}: weight rows {W.shape[0]} != feature width {x.shape[1]}")
        key = (op.idx, post_sf, x.data_ptr(), tuple(x.shape), tuple(x.stride()), x.dtype)
        xw = self._nmm.get(key)
        if xw is None:
            xw = ops.update_mm(x, W, sf=post_sf)
            self._count(x.shape[0] * (x.shape[1] * x.element_size() + W.shape[1] * 4) + W.numel() * W.element_size())
            self._nmm[key] = xw
        return Scat(xw, v.mode, v.fill)

    def _pushdown_mm(self, op, add_idx, post_sf=None):
        """MM(scatter a + scatter b) as (a W)[r_a(e)] + (b W)[r_b(e)]."""
        if post_sf is not None:
            return None  # the SF acts on the sum: keep the literal order
        a, b = [self._source(self.g.ops[add_idx], k) for k in range(2)]
        if not (isinstance(a, Scat) and isinstance(b, Scat)):
            return None
        sa, sb = self._node_mm(op, a), self._node_mm(op, b)
        out = ops.apply_edge(self.graph, "ADD", None, sa.t, sa.mode, sb.t, sb.mode)
        self._count(self.graph.nnz * out.shape[1] * 4 * 3)
        return EdgeT(out)

    def _pending_siblings(self, x, main_idx, W):
        """Unevaluated applynode MM ops whose input is the node tensor x itself, with weights of
        W's dtype and K and no SF epilogue of their own."""
        if not self.sibling_mm:
            return []
        sib = []
        for op in self.g.ops:
            if op.idx == main_idx or op.idx in self.values or op.type != "applynode" or op.comp != "MM":
                continue
            ins = self.g.inputs[op.idx]
            if len(ins) != 1:
                continue
            src = ins[0]
            if src.kind == "op":
                v = self.values.get(src.op)
                if not (isinstance(v, NodeT) and v.t is x):
                    continue
            elif src.kind == "x":
                if self._ext(op, 0) is not None or self.tensors.get("x") is not x:
                    continue
            else:
                continue
            Ws = self.tensors.get(f"w:{op.idx}")
            if Ws is None or Ws.dtype != W.dtype or Ws.shape[0] != W.shape[0] or self._sf_child_any(op):
                continue
            sib.append(op)
        return sib

    def _sf_child_any(self, op):
        cons = self.consumers[op.idx]
        return self.fuse_sf and len(cons) == 1 and self.g.ops[cons[0]].comp == "SF" \
            and self.g.ops[cons[0]].type == op.type

    def _node_gemm(self, x, main_idx, W, post_sf=None):
        """x W for op main_idx; sibling MMs of the same x ride along in the same GEMM (their
        values are column views of the output).  Returns the main op's [rows, N] result."""
        sibs = [] if post_sf is not None else self._pending_siblings(x, main_idx, W)
        x2, W2 = self._mm_dtypes(x, W)
        if not sibs:
            out = ops.update_mm(x2, W2, sf=post_sf)
            self._count(x.shape[0] * (x.shape[1] * x.element_size() + W.shape[1] * 4) + W.numel() * W.element_size())
            return out
        Wc = _sibling_cat([W] + [self.tensors[f"w:{o.idx}"] for o in sibs])
        x2, Wc2 = self._mm_dtypes(x, Wc)
        out = ops.update_mm(x2, Wc2)
        self._count(x.shape[0] * (x.shape[1] * x.element_size() + Wc.shape[1] * 4) + Wc.numel() * Wc.element_size())
        off = W.shape[1]
        for o in sibs:
            n_o = self.tensors[f"w:{o.idx}"].shape[1]
            self.values[o.idx] = NodeT(out[:, off:off + n_o])
            off += n_o
        return out[:, :W.shape[1]]

    def _gather_value(self, op):
        v = self._eval_gather(op)
        if self.dist is None:
            return v
        return NodeT(self.dist.reduce_cols(v.t) if op.order == "C" else self.dist.reduce_rows(v.t))

    def _mm_first_operands(self, G):
        """(x, w, fill) of a gather G = sum_e w_e x[src(e)] (w None: unweighted), or None."""
        v = self._source(G, 0)
        if isinstance(v, Deferred):
            p = self.g.ops[v.op]
            if p.comp != "MUL" or self.sem.bin_of(p) != "MUL":
                return None
            pins = self._inputs(p)
            if len(pins) == 1:
                extra = self._ext(p, 1)
                pins = pins + ([self._wrap_ext(extra)] if extra is not None else [])
            xs = [z for z in pins if isinstance(z, Scat) and z.mode == "src"]
            ws = [z for z in pins if not (isinstance(z, Scat) and z.mode == "src")]
            if len(xs) != 1 or len(ws) > 1:
                return None
            x, w, fill = xs[0].local, None, xs[0].fill
            if ws:
                if isinstance(ws[0], tuple) or ws[0] is None:
                    return None
                w = self._to_edge_tensor(ws[0])
                if w.shape[1] != 1:
                    return None
        elif isinstance(v, Scat) and v.mode == "src":
            x, w, fill = v.local, None, v.fill
        else:
            return None
        return x, w, fill

    def _eval_two_hop(self, G2, M):
        """M = A (A x) W as A (A (x W)): the first hop G1's value and its scatter stay unformed."""
        G1 = next((g1 for g1, g2 in self.two_hop.items() if g2 == G2.idx), None)
        raw = self.values.get(G1) if G1 is not None else None
        if not (self.mm_first and isinstance(raw, Lazy) and raw.v is None):
            return None
        src = self.g.inputs[G2.idx][0]
        P = self.g.ops[src.op]
        w2 = None
        if P.type != "scatter":  # the second hop's weight MUL: its operand that is not the scatter
            pv = self.values.get(P.idx)
            if not isinstance(pv, Deferred) or P.comp != "MUL" or self.sem.bin_of(P) != "MUL":
                return None
            slots = [k for k, x in enumerate(self.g.inputs[P.idx])
                     if not (x.kind == "op" and self.g.ops[x.op].type == "scatter")]
            others = [self._source(P, k) for k in slots]
            if len(self.g.inputs[P.idx]) == 1:
                extra = self._ext(P, 1)
                others = [self._wrap_ext(extra)] if extra is not None else []
            if len(others) > 1 or (others and isinstance(others[0], (tuple, Scat))):
                return None
            if others:
                w2 = self._to_edge_tensor(others[0])
                if w2.shape[1] != 1:
                    return None
        opnd = self._mm_first_operands(self.g.ops[G1])
        if opnd is None:
            return None
        x, w1, fill = opnd
        W = self.tensors[f"w:{M.idx}"]
        if fill is not None or W.shape[0] != x.shape[1]:
            return None
        xw = self._node_gemm(x, M.idx, W).contiguous()
        z = self._spmm(xw, "src", w1)
        y = self._spmm(z, "src", w2)
        n, E, F = self.graph.n_rows, self.graph.nnz, xw.shape[1]
        for w in (w1, w2):
            self._count(E * (4 + (4 if w is not None else 0) + 4 * F) + n * (8 + 4 * F))
        self.values[M.idx] = NodeT(y)
        return Lazy(lambda: self._gather_value(G2))

    def _eval_mm_first(self, G, M):
        """Sets M's value to aggregate(x W) and returns G's value lazily; None if the operands
        do not allow it (head-wise weights, edge-tensor features)."""
        if G.idx in self.two_hop.values():
            v = self._eval_two_hop(G, M)
            if v is not None:
                return v
        opnd = self._mm_first_operands(G)
        if opnd is None:
            return None
        x, w, fill = opnd
        W = self.tensors[f"w:{M.idx}"]
        if W.shape[0] != x.shape[1]:
            return None
        xw = self._node_gemm(x, M.idx, W).contiguous()
        if fill is not None:  # row shards: exchange x W (narrower than x)
            xw = fill(xw)
        n, E, F = self.graph.n_rows, self.graph.nnz, xw.shape[1]
        y = self._spmm(xw, "src", w)
        self._count(E * (4 + (4 if w is not None else 0) + 4 * F) + n * (8 + 4 * F))
        self.values[M.idx] = NodeT(self.dist.reduce_rows(y) if self.dist is not None else y)
        return Lazy(lambda: self._gather_value(G))

    def _match_attention(self):
        """{MUL op M: (softmax pattern, gather G2, x scatter S)} for M = scatter_C(x) * alpha (original,
        alpha = the pattern's D) or * v (trans, v = V), whose only consumer is a gather R."""
        found = {}
        ops_, ins, cons = self.g.ops, self.g.inputs, self.consumers
        for A, pat in self.softmax.items():
            w_op = pat["D"] if pat["D"] is not None else pat["V"]
            cands = [c for c in cons[w_op] if c != pat["G"]]
            if len(cands) != 1:
                continue
            M = cands[0]
            m = ops_[M]
            if m.type != "applyedge" or m.comp != "MUL" or self.sem.bin_of(m) != "MUL" or len(ins[M]) != 2:
                continue
            srcs = [x.op if x.kind == "op" else None for x in ins[M]]
            other = [o for o in srcs if o != w_op]
            if len(other) != 1 or other[0] is None:
                continue
            S = other[0]
            if ops_[S].type != "scatter" or ops_[S].order != "C":
                continue
            if len(cons[M]) != 1 or ops_[cons[M][0]].type != "gather" or ops_[cons[M][0]].order != "R":
                continue
            found[M] = (pat, cons[M][0], S)
        return found

    def _eval_attention(self, G2, M, sf_out=None):
        """G2 = gather(scatter_C(x) * alpha|v) as one fused launch; None if the shapes do not allow it.
        sf_out: the SF of G2's only consumer, applied as y is written (the caller owns that op's value)."""
        pat, _, S = self.attn[M]
        st = self._att_state.get(pat["A"])
        sv = self.values.get(S)
        if st is None or not isinstance(sv, Scat) or sv.mode != "src":
            return None
        a, b, sf = st
        x = sv.t
        F, H = x.shape[1], a.shape[1]
        if x.dtype != torch.float32 or not ops.BlockedPlan.supports_att(F, H):
            return None
        B = self.attention_blocks or ops.BlockedPlan.auto_blocks(self.graph, F)
        # the lean fused kernel (F = 128, 8 heads) beats softmax + aggregate even unblocked (B = 1:
        # Flickr 102 vs 168 us; the round-4 probe, profiles/r04/layer_bench_*.log); other shapes need a blocked table
        lean = F == 128 and H == 8
        if B < (1 if (self.attention_blocks or lean) else 4) or not ops.blocked_ready(self.graph, B):
            return None
        norm = pat["D"] is not None
        G = pat["G"]
        gv = self.values.get(G)
        want = not norm and isinstance(gv, Lazy) and gv.v is None
        y, sums = ops.gat_aggregate_blocked(self.graph, x, a, b, sf, normalize=norm, want_sums=want, blocks=B,
                                            sf_out=sf_out)
        E, n = self.graph.nnz, self.graph.n_rows
        self._count(E * (4 + 4 * F + 4 * H) + n * (8 + 4 * F + 4 * H))
        if want:
            self.values[G] = NodeT(sums)
        return NodeT(y)

    def _eval_softmax(self, A, pat):
        """Registers V, G (and D) as views of one gta_edge_softmax launch; returns A's own value."""
        ins = self._inputs(A)
        if not all(isinstance(x, Scat) for x in ins) or {x.mode for x in ins} != {"dst", "src"}:
            return None
        a = next(x.t for x in ins if x.mode == "dst")
        b = next(x.t for x in ins if x.mode == "src")
        H = a.shape[1]
        if b.shape[1] != H or H > 64 or H & (H - 1):
            return None
        V, sf, norm = self.g.ops[pat["V"]], self.sem.sf_of(self.g.ops[pat["V"]]), pat["D"] is not None
        E, n = self.graph.nnz, self.graph.n_rows
        self._att_state[A.idx] = (a, b, sf)

        def launch():
            out, sums = ops.edge_softmax(self.graph, a, b, sf, normalize=norm, want_sums=True)
            self._count(E * (4 + 8 * H) + n * (8 + 8 * H))
            return out, sums
        shared = Lazy(launch)
        self.values[pat["G"]] = Lazy(lambda: NodeT(shared.force()[1]))
        if norm:
            self.values[pat["D"]] = Lazy(lambda: EdgeT(shared.force()[0]))
            self.values[V.idx] = Lazy(lambda: self._eval_applyedge(A, post_sf=sf))
        else:
            self.values[V.idx] = Lazy(lambda: EdgeT(shared.force()[0]))
        return Lazy(lambda: self._eval_applyedge(A))

    # ---------------------------------------------------------------- eval
    def _binary(self, op):
        return self.sem.bin_of(op)

    def _eval_applyedge(self, op, post_sf=None):
        E = self.graph.nnz
        pushed = (op.comp == "MM" and self.mm_pushdown and self.g.inputs[op.idx]
                  and self.g.inputs[op.idx][0].kind == "op"
                  and self.pushdown.get(self.g.inputs[op.idx][0].op) == op.idx)
        ins = [None] if pushed else self._inputs(op)
        if pushed:
            raw = self.values.get(self.g.inputs[op.idx][0].op)
            if not (isinstance(raw, Lazy) and raw.v is None):
                ins = self._inputs(op)
        if op.comp == "MM":
            src = self.g.inputs[op.idx][0]
            raw = self.values.get(src.op) if src.kind == "op" else None
            if self.mm_pushdown and src.kind == "op" and self.pushdown.get(src.op) == op.idx \
                    and isinstance(raw, Lazy) and raw.v is None:
                v = self._pushdown_mm(op, src.op, post_sf)
                if v is not None:
                    return v
            if ins[0] is None:
                ins = self._inputs(op)
            if self.node_mm and isinstance(ins[0], Scat):
                return self._node_mm(op, ins[0], post_sf)
            return EdgeT(self._edge_mm(op, ins[0], post_sf))
        if op.comp == "SF":
            a, am, _ = self._edge_operand(ins[0])
            out = ops.apply_edge(self.graph, None, self.sem.sf_of(op), a, am)
            self._count(E * (a.shape[1] * 8))
            return EdgeT(out)
        bin_ = self._binary(op)
        if len(ins) == 1:  # unary ADD/MUL: identity unless an extra operand is supplied
            extra = self._ext(op, 1)
            ins = ins + ([self._wrap_ext(extra)] if extra is not None else [])
            if len(ins) == 1:
                return EdgeT(self._to_edge_tensor(ins[0]))
        x, y = ins[0], ins[1]
        if bin_ == "RDIV":
            x, y, bin_ = y, x, "DIV"
        a, am, arow = self._edge_operand(x)
        b, bm, brow = self._edge_operand(y)
        if arow and not brow:  # keep the broadcast row in the b slot (ADD/MUL commute)
            if bin_ in ("ADD", "MUL"):
                a, am, b, bm, arow, brow = b, bm, a, am, False, True
            else:
                a = a.expand(E, a.shape[1]).contiguous()  # a broadcast row on the left of DIV/SUB
                am, arow = "edge", False
        out = ops.apply_edge(self.graph, bin_, post_sf, a, am, b, bm, b_broadcast_row=brow)
        self._count(E * out.shape[1] * 4 * 3)
        return EdgeT(out)

    def _edge_mm(self, op, v, post_sf=None):
        W = self.tensors[f"w:{op.idx}"]
        if isinstance(v, Scat):
            idx = self.graph.indices if v.mode == "src" else self.graph.row_of_edge()
            x, row_idx = v.t, idx
        else:
            x, row_idx = self._to_edge_tensor(v), None
        x, W = self._mm_dtypes(x, W)
        out = ops.update_mm(x, W, row_idx, sf=post_sf, m=self.graph.nnz if row_idx is None else None)
        self._count(self.graph.nnz * (x.shape[1] * x.element_size() + W.shape[1] * 4))
        return out

    @staticmethod
    def _mm_dtypes(x, W):
        # fp32 activations with bf16 weights go straight in: the GEMM rounds x to bf16
        # while staging it into LDS (GTA_F32_BF16); only bf16 x with fp32 W is widened
        if W.dtype == torch.float32 and x.dtype != torch.float32:
            x = x.float()
        return x, W

    def _eval_gather(self, op, acc=None, self_term=None, out_dtype=torch.float32):
        """self_term (x, s): y = x * s + the aggregate, or None if this gather's form cannot take it;
        out_dtype (self_term only): y's storage dtype."""
        if op.order == "C":
            if acc is not None or self_term is not None:
                return None
            return self._eval_gather_c(op)
        src = self.g.inputs[op.idx][0]
        if self_term is not None:
            v = self._source(op, 0) if not (self.fuse_attention and src.kind == "op" and src.op in self.attn) else None
            if isinstance(v, Deferred):
                p = self.g.ops[v.op]
                pins = self._inputs(p)
                if p.comp == "MM" or self._binary(p) != "MUL":
                    return None
                if len(pins) == 1:
                    extra = self._ext(p, 1)
                    pins = pins + ([self._wrap_ext(extra)] if extra is not None else [])
                if len(pins) != 2:
                    return None
                y = self._weighted_aggregate(pins[0], pins[1], self_term=self_term, out_dtype=out_dtype)
                return None if y is None else NodeT(y)
            if isinstance(v, Scat):
                y = self._spmm(v.t, v.mode, None, self_term=self_term, out_dtype=out_dtype)
                if y is not None:
                    n, E = self.graph.n_rows, self.graph.nnz
                    self._count(E * (4 + v.t.shape[1] * v.t.element_size()) + n * (8 + v.t.shape[1] * y.element_size()))
                    return NodeT(y)
            return None
        if self.fuse_attention and src.kind == "op" and src.op in self.attn:
            raw = self.values.get(src.op)
            if isinstance(raw, (Deferred, Lazy)):
                y = self._eval_attention(op, src.op)
                if y is not None:
                    return y
        v = self._source(op, 0)
        n, E = self.graph.n_rows, self.graph.nnz
        if isinstance(v, Deferred):
            p = self.g.ops[v.op]
            pins = self._inputs(p)
            if p.comp == "MM":
                if self.node_mm and isinstance(pins[0], Scat):  # gather(x[r(e)] W) = SpMM of x W
                    sw = self._node_mm(p, pins[0])
                    y = self._spmm(sw.t, sw.mode, None)
                    self._count(E * (4 + sw.t.shape[1] * 4) + n * (8 + sw.t.shape[1] * 4))
                    return NodeT(y)
                xe = self._edge_mm(p, pins[0])
                y = ops.gather_add(self.graph, xe)
                self._count(E * xe.shape[1] * 4 + n * xe.shape[1] * 4)
                return NodeT(y)
            bin_ = self._binary(p)
            if len(pins) == 1:
                extra = self._ext(p, 1)
                pins = pins + ([self._wrap_ext(extra)] if extra is not None else [])
            if len(pins) == 1:
                v = pins[0]
            elif bin_ == "MUL":
                return NodeT(self._weighted_aggregate(pins[0], pins[1], acc))
            else:  # a non-MUL fused pair: evaluate the producer, then gather
                v = self._materialize_deferred(v)
        if isinstance(v, Scat):
            y = self._spmm(v.t, v.mode, None, acc)
            self._count(E * (4 + v.t.shape[1] * 4) + n * (8 + v.t.shape[1] * 4))
            return NodeT(y)
        xe = self._to_edge_tensor(v)
        y = ops.aggregate(self.graph, xe, "edge", None, out=acc, accumulate=acc is not None, plan=self._plan())
        self._count(E * xe.shape[1] * 4 + n * (8 + xe.shape[1] * 4))
        return NodeT(y)

    def _plan(self):
        return self.plan_chunk if self.plan_chunk else None

    def _eval_gather_c(self, op):
        """ISA gather with DIRECTION src (ORDER C, template/ISA_defination.yaml:46-48): y[j] = sum of
        the edge value over the edges whose SOURCE is j, y [n_cols, F].  Runs the ordered row kernels
        over the graph's stable CSC view (ops.CSC, gta_csc_build): a column's edges are summed in CSR
        order, deterministic, no atomics.  A fused producer stays virtual as in direction R: a scatter
        operand is gathered by index (its CSC view: "dst" rows for scatter R, the column itself for
        scatter C), a MUL by an edge weight runs as one weighted aggregate (the weight read in CSC
        order through one permuting copy); anything else is materialised as an edge tensor and summed
        by CSC position (gta_gather_add's direction C)."""
        c = ops.csc(self.graph)
        E, nc = self.graph.nnz, self.graph.n_cols
        v = self._source(op, 0)
        if isinstance(v, Deferred):
            p = self.g.ops[v.op]
            if p.comp != "MM" and self._binary(p) == "MUL":
                pins = self._inputs(p)
                if len(pins) == 1:
                    extra = self._ext(p, 1)
                    pins = pins + ([self._wrap_ext(extra)] if extra is not None else [])
                if len(pins) == 2:
                    y = self._weighted_c(c, pins[0], pins[1])
                    if y is not None:
                        return NodeT(y)
            v = self._materialize_deferred(v)
        if isinstance(v, Scat):
            if v.mode == "dst":  # the transposed aggregate: column-blocked like direction R when the table is large
                y = self._spmm(v.t, "src", None, graph=c.view("dst"))
            else:
                y = ops.aggregate(c.view("src"), v.t, "src", None, plan=self._plan())
            self._count(E * (4 + v.t.shape[1] * v.t.element_size()) + nc * (8 + v.t.shape[1] * 4))
            return NodeT(y)
        xe = self._to_edge_tensor(v)
        y = ops.aggregate(c.view("edge"), xe, "src", None, plan=self._plan())
        self._count(E * (4 + xe.shape[1] * 4) + nc * (8 + xe.shape[1] * 4))
        return NodeT(y)

    def _weighted_c(self, c, u, v):
        """sum over a source column's edges of u(e) (.) v(e) (direction C form of _weighted_aggregate):
        the narrower operand is the (head) weight, permuted once into CSC order; None when neither
        operand is an edge/scatter tensor of a width the aggregate takes."""
        def width(z):
            if isinstance(z, tuple):
                return z[1].shape[1]
            return z.t.shape[1] if not isinstance(z, Deferred) else 0

        x, w = (u, v) if width(u) >= width(v) else (v, u)
        if isinstance(x, tuple) or isinstance(x, Deferred) or isinstance(w, Deferred):
            return None
        E, nc = self.graph.nnz, self.graph.n_cols
        if isinstance(w, tuple) and w[0] == "row":  # a constant row weight: aggregate then scale (linear)
            if isinstance(x, Scat):
                y = ops.aggregate(c.view("dst" if x.mode == "dst" else "src"), x.t, "src", None, plan=self._plan())
            else:
                y = ops.aggregate(c.view("edge"), self._to_edge_tensor(x), "src", None, plan=self._plan())
            self._count(E * (4 + 4 * y.shape[1]) + nc * (8 + 4 * y.shape[1]))
            return ops.apply_node("MUL", None, y, w[1], b_broadcast_row=True)
        wt = self._to_edge_tensor(w)
        if wt.dtype != torch.float32 or width(x) % wt.shape[1]:
            return None
        wc = ops.apply_edge(c.view("edge"), None, None, wt, "src")  # wc[k] = wt[perm[k]]: CSC order
        if isinstance(x, Scat):
            view, table = c.view("dst" if x.mode == "dst" else "src"), x.t
        else:
            view, table = c.view("edge"), self._to_edge_tensor(x)
        if isinstance(x, Scat) and x.mode == "dst":  # column-blocked like direction R when the table is large
            y = self._spmm(table, "src", wc, graph=view)
        else:
            y = ops.aggregate(view, table, "src", wc, plan=self._plan())
        F, H = table.shape[1], wc.shape[1]
        self._count(E * 8 * H + E * (4 + 4 * H + table.element_size() * F) + nc * (8 + 4 * F))
        return y

    def _weighted_aggregate(self, u, v, acc=None, self_term=None, out_dtype=torch.float32):
        """sum_e u(e) (.) v(e): the wider operand is the feature row, the narrower the (head) weight.
        self_term: see _eval_gather (None back if this form cannot take it)."""
        n, E = self.graph.n_rows, self.graph.nnz

        def width(z):
            if isinstance(z, tuple):
                return z[1].shape[1]
            return z.t.shape[1] if not isinstance(z, Deferred) else 0

        x, w = (u, v) if width(u) >= width(v) else (v, u)
        if isinstance(w, tuple) and w[0] == "row":  # constant row weight: aggregate then scale (linear)
            if self_term is not None:
                return None
            y = self._unweighted(x)
            return ops.apply_node("MUL", None, y, w[1], b_broadcast_row=True)
        wt = self._to_edge_tensor(w)
        if isinstance(x, Scat):
            xt, mode = x.t, x.mode
        else:
            xt, mode = self._to_edge_tensor(x), "edge"
        if xt.shape[1] % wt.shape[1]:
            raise ValueError(f"weighted aggregate: weight width {wt.shape[1]} does not divide {xt.shape[1]}")
        y = self._spmm(xt, mode, wt, acc, self_term, out_dtype)
        if y is None:
            return None
        self._count(E * (4 + 4 * wt.shape[1] + xt.element_size() * xt.shape[1]) + n * (8 + y.element_size() * xt.shape[1]))
        return y

    def _spmm(self, xt, mode, wt, acc=None, self_term=None, out_dtype=torch.float32, graph=None):
        """SpMM-form aggregate: column-blocked when the gathered table outgrows L2, else row-chunked.
        self_term (x, s): y = x * s + the aggregate in one launch (row-chunked form; None back when
        x's dtype is not the gathered table's, or when the column-blocked form is the better one:
        the caller then accumulates into the formed x * s instead).  graph: the graph the rows
        and indices come from (default the layer's CSR; a CSC view for the ORDER-C gathers)."""
        g = self.graph if graph is None else graph
        B = self._blocked_blocks(xt, mode, 0 if wt is None else wt.shape[1], g)
        if self_term is not None:
            xs, sc = self_term
            if B or xs.dtype != xt.dtype or xs.shape[1] != xt.shape[1] or xs.shape[0] < g.n_rows:
                return None
            return ops.aggregate(g, xt, mode, wt, plan=self._plan(), self_term=(xs, sc), out_dtype=out_dtype)
        if B:
            return ops.aggregate_blocked(g, xt, wt, out=acc, accumulate=acc is not None, blocks=B)
        return ops.aggregate(g, xt, mode, wt, out=acc, accumulate=acc is not None, plan=self._plan())

    def _blocked_blocks(self, xt, mode, heads, graph=None):
        """Column blocks of the blocked aggregate for this gathered table, or 0 for the row-chunked
        form: a source table of at least blocked_min_table_bytes (its own element size) of a dtype
        and width the blocked kernels take."""
        g = self.graph if graph is None else graph
        if not (mode == "src" and self.blocked_blocks and xt.dtype in ops.BlockedPlan.DTYPES
                and xt.shape[0] * xt.shape[1] * xt.element_size() >= self.blocked_min_table_bytes
                and ops.BlockedPlan.supports(xt.shape[1], heads, xt.dtype)):
            return 0
        B = self.blocked_blocks
        if B == "auto":
            B = ops.BlockedPlan.auto_blocks(g, xt.shape[1], xt.element_size())
            B = B if B >= 4 else 0
        return B if B and g.blocked_plan(B).sorted else 0

    def _unweighted(self, x):
        if isinstance(x, Scat):
            return ops.aggregate(self.graph, x.t, x.mode, None, plan=self._plan())
        return ops.aggregate(self.graph, self._to_edge_tensor(x), "edge", None, plan=self._plan())

    def _eval_applynode(self, op, post_sf=None):
        if self.gather_acc and post_sf is None and op.idx in self.gacc:
            y = self._eval_gather_acc(op)
            if y is not None:
                self._count(self.n_nodes * y.t.shape[1] * 4)  # the aggregate's extra read of T
                return y
        ins = self._inputs(op)
        n = self.n_nodes
        if op.comp == "MM":
            W = self.tensors[f"w:{op.idx}"]
            x = self._node(ins[0])
            return NodeT(self._node_gemm(x, op.idx, W, post_sf))
        if op.comp == "SF":
            a = self._node(ins[0])
            y = ops.apply_node(None, self.sem.sf_of(op), a)
            self._count(n * a.shape[1] * 8)
            return NodeT(y)
        bin_ = self._binary(op)
        if len(ins) == 1:
            extra = self._ext(op, 1)
            if extra is None:
                return NodeT(self._node(ins[0]))
            ins = ins + [self._wrap_ext(extra)]
        x, y = ins[0], ins[1]
        if bin_ == "RDIV":
            x, y, bin_ = y, x, "DIV"
        if isinstance(x, tuple) and bin_ in ("ADD", "MUL"):
            x, y = y, x
        a = self._node(x)
        brow = isinstance(y, tuple)
        b = y[1] if brow else self._node(y)
        out = ops.apply_node(bin_, post_sf, a, b, b_broadcast_row=brow)
        self._count(n * out.shape[1] * 4 * 3)
        return NodeT(out)

    def _node(self, v):
        if isinstance(v, NodeT):
            return v.t
        if isinstance(v, tuple) and v[0] == "row":
            return v[1].expand(self.n_nodes, v[1].shape[1]).contiguous()
        raise TypeError(f"applynode operand is not a node tensor ({type(v).__name__})")

    def _eval(self, op, block, expr=True):
        if expr and self.edge_expr and op.idx in self.expr_nodes:
            # a node of a fused expression tree: its gather runs it; computed unfused only if read
            return Lazy(lambda: _forced(self._eval(op, block, expr=False)))
        fused_into = {p: c for p, c, _ in block.fused}
        if op.type == "scatter":
            src = self.g.inputs[op.idx][0]
            raw = self.values.get(src.op) if src.kind == "op" else None
            if isinstance(raw, Lazy) and raw.v is None:  # keep a fused-away producer unforced
                return Lazy(lambda: (raw.force(), self._eval(op, block))[1])
            v = self._source(op, 0)
            if isinstance(v, tuple):
                v = NodeT(self._node(v))
            if not isinstance(v, NodeT):
                raise TypeError(f"scatter op {op.idx} needs a node tensor")
            t, fill, own = v.t, None, None
            if self.dist is not None:  # row shards fill source tables lazily; column shards gather dst rows
                if op.order == "C":
                    fill = self.dist.src_fill
                    if src.kind != "op":  # a model input the rank may hold whole
                        key = f"ext:{op.idx}:0"
                        own = self.dist.replicated(key if key in self.tensors else "x")
                else:
                    t = self.dist.gather_rows(t)
            s = Scat(t, "src" if op.order == "C" else "dst", fill, own)
            # a STORE_E'd scatter is only materialised when nothing reads it back (a sink):
            # every consumer kernel gathers by index, which is the same bytes
            if op.idx in block.stored and not (self.elide_scatter_stores and self.consumers[op.idx]):
                return EdgeT(self._to_edge_tensor(s))
            return s
        if self.fuse_softmax and op.idx in self.softmax:
            v = self._eval_softmax(op, self.softmax[op.idx])
            if v is not None:
                return v
        if self.mm_pushdown and op.idx in self.pushdown:
            return Lazy(lambda: self._eval_applyedge(op))  # its MM consumer computes through the sum
        if self.fuse_attention and op.idx in self.attn and fused_into.get(op.idx) is None:
            return Lazy(lambda: self._eval_applyedge(op))  # its gather consumer runs the fused kernel
        if op.type == "applyedge":
            c = fused_into.get(op.idx)
            if c is not None and self.g.ops[c].type == "gather" and op.comp in ("MUL", "MM"):
                return Deferred(op.idx)
        if op.type == "applynode" and op.comp == "MM":
            v = self._eval_mlp(op)
            if v is not None:
                return v
        sf_child = self._sf_child(op, block)
        if sf_child is not None:
            ev = self._eval_applyedge if op.type == "applyedge" else self._eval_applynode
            self.values[sf_child.idx] = ev(op, post_sf=self.sem.sf_of(sf_child))
            return Lazy(lambda: ev(op))
        if op.type == "applyedge":
            return self._eval_applyedge(op)
        if op.type == "gather":
            if self.edge_expr and op.idx in self.expr:
                v = self._eval_edge_expr(op)
                if v is not None:
                    return v
            if self.gather_acc and any(g == op.idx for g, _, _ in self.gacc.values()):
                return Lazy(lambda: self._gather_value(op))  # its ADD consumer accumulates it
            if self.mm_first and op.idx in self.two_hop:
                return Lazy(lambda: self._gather_value(op))  # the second hop's MM-first form runs it
            if self.mm_first and op.idx in self.reorder:
                v = self._eval_mm_first(op, self.g.ops[self.reorder[op.idx]])
                if v is not None:
                    return v
            v = self._attention_with_sf(op, block)
            if v is not None:
                return v
            return self._gather_value(op)
        if op.type == "applynode":
            if self.mlp_bf16_sum and self.gather_acc and op.idx in self.gacc and self._mlp_input(op) is not None:
                return Lazy(lambda: self._eval_applynode(op))  # the MLP it feeds may take it in bf16
            if self.gather_acc and op.idx in self.gacc_t and self._self_term(op) is not None:
                return Lazy(lambda: self._eval_applynode(op))  # its ADD consumer's aggregate may form it
            return self._eval_applynode(op)
        raise ValueError(op.type)

    def _attention_with_sf(self, op, block):
        """An attention gather whose only consumer is an applynode SF (GAT op 12 -> op 13): one fused
        launch writes the SF's value (the reduce applies it as y is stored, bitwise what apply_node
        computes); the gather's own value stays available, recomputed unfused if read.  The SF may sit
        in a later block (GAT Reddit's stream puts op 13 in a block of its own): its block then finds
        the value present, as for any fused post-op."""
        if not (self.fuse_sf and self.fuse_attention) or self.dist is not None or op.order != "R":
            return None
        src = self.g.inputs[op.idx][0]
        if src.kind != "op" or src.op not in self.attn or not isinstance(self.values.get(src.op), (Deferred, Lazy)):
            return None
        cons = self.consumers[op.idx]
        if len(cons) != 1:
            return None
        c = self.g.ops[cons[0]]
        if c.comp != "SF" or c.type != "applynode" or len(self.g.inputs[c.idx]) != 1:
            return None
        y = self._eval_attention(op, src.op, sf_out=self.sem.sf_of(c))
        if y is None:
            return None
        self.values[c.idx] = y
        return Lazy(lambda: self._gather_value(op))

    def _only_consumer(self, op, comp):
        """op's single consumer when it is an applynode of kind comp reading only op, else None."""
        cons = self.consumers[op.idx]
        if len(cons) != 1:
            return None
        c = self.g.ops[cons[0]]
        if c.type != "applynode" or c.comp != comp or len(self.g.inputs[c.idx]) != 1 or self._ext(c, 1) is not None:
            return None
        return c

    def _mlp_chain(self, a):
        """(b, c, d) of a chain a -> [SF b] -> MM c -> [SF d] of node GEMMs, each intermediate read
        only by the next op, with weights gta_update_mlp takes; else None."""
        if not (self.fuse_mlp and a.type == "applynode" and a.comp == "MM" and len(self.g.inputs[a.idx]) == 1):
            return None
        b = self._only_consumer(a, "SF") if self.fuse_sf else None
        c = self._only_consumer(b if b is not None else a, "MM")
        if c is None:
            return None
        d = self._only_consumer(c, "SF") if self.fuse_sf else None
        w1, w2 = self.tensors[f"w:{a.idx}"], self.tensors[f"w:{c.idx}"]
        return (b, c, d) if ops.update_mlp_weights_ok(w1.shape[0], w1, w2) else None

    def _mlp_input(self, A):
        """The MLP head a when node op A's only consumer heads a fusable MLP chain, else None."""
        a = self._only_consumer(A, "MM")
        return a if a is not None and self._mlp_chain(a) is not None else None

    def _eval_mlp(self, a):
        """Two chained node GEMMs a -> [SF b] -> MM c -> [SF d] (GIN's MLP, genGraphOP.py:103-108)
        as one gta_update_mlp launch when the shapes allow it (fp32 or bf16 x, bf16 weights, widths
        <= 128).  When a's input is the still-unformed GIN sum A = (1 + eps) x + aggregate, the
        aggregate stores A in bf16 (ABI 10): the MLP rounds an fp32 x to bf16 anyway, so the bits
        are unchanged and A's [N, F] write and read halve.  The chain's last value is set; A, a, b
        and c stay available, recomputed unfused (fp32) if something reads them (the tests read
        them all).  None when the chain or its operands do not fit."""
        chain = self._mlp_chain(a)
        if chain is None:
            return None
        b, c, d = chain
        w1, w2 = self.tensors[f"w:{a.idx}"], self.tensors[f"w:{c.idx}"]
        x = None
        src = self.g.inputs[a.idx][0]
        if self.mlp_bf16_sum and self.gather_acc and src.kind == "op" and src.op in self.gacc:
            raw = self.values.get(src.op)
            if isinstance(raw, Lazy) and raw.v is None:
                y = self._eval_gather_acc(self.g.ops[src.op], out_dtype=torch.bfloat16)
                if y is not None and ops.update_mlp_supported(y.t, w1, w2):
                    x = y.t
        if x is None:
            x = self._node(self._inputs(a)[0])
            if not ops.update_mlp_supported(x, w1, w2):
                return None
        sf1 = self.sem.sf_of(b) if b is not None else None
        sf2 = self.sem.sf_of(d) if d is not None else None
        out = ops.update_mlp(x, w1, w2, sf1=sf1, sf2=sf2)
        self._count(x.shape[0] * (x.shape[1] * x.element_size() + w2.shape[1] * 4) + w1.numel() * 2 + w2.numel() * 2)
        self.values[(d if d is not None else c).idx] = NodeT(out)
        if d is not None:
            self.values[c.idx] = Lazy(lambda: self._eval_applynode(c))
        if b is not None:
            self.values[b.idx] = Lazy(lambda: self._eval_applynode(a, post_sf=sf1))
        return Lazy(lambda: self._eval_applynode(a))

    def _sf_child(self, op, block):
        """The SF op this op's output feeds exclusively (same kind, same block), if fusable."""
        if not self.fuse_sf or op.type not in ("applyedge", "applynode") or op.comp == "SF" or not op.out_list:
            return None
        cons = self.consumers[op.idx]
        if len(cons) != 1:
            return None
        c = self.g.ops[cons[0]]
        if c.comp != "SF" or c.type != op.type or c.idx not in block.ops:
            return None
        if op.comp in ("ADD", "MUL") and len(self.g.inputs[op.idx]) < 2 and self._ext(op, 1) is None:
            return None  # identity pass-through: no kernel to carry the post-op
        return c

    # ---------------------------------------------------------------- run
    def block_order(self):
        owner = {}
        for b in self.stream.blocks:
            for o in b.ops:
                owner.setdefault(o, b.index)
        deps = {b.index: set() for b in self.stream.blocks}
        for b in self.stream.blocks:
            for o in b.ops:
                for p in self.g.producers(o):
                    if p in owner and owner[p] != b.index:
                        deps[b.index].add(owner[p])
        order, done = [], set()
        pending = [b.index for b in self.stream.blocks]
        while pending:
            for i in pending:
                if deps[i] <= done:
                    order.append(i)
                    done.add(i)
                    pending.remove(i)
                    break
            else:
                raise ValueError(f"stream blocks have a cyclic dependency: {pending}")
        return order

    def run(self):
        covered = set()
        for b in self.stream.blocks:
            covered.update(b.ops)
        missing = set(range(len(self.g))) - covered
        if missing:
            raise ValueError(f"stream does not cover ops {sorted(missing)}")
        tracer = _Tracer(self) if self.trace else None
        for bi in self.block_order():
            block = self.stream.blocks[bi]
            for i in self.g.topo(block.ops):
                if i in self.values:  # produced early as a fused post-op
                    continue
                if tracer:
                    tracer.begin()
                self.values[i] = self._eval(self.g.ops[i], block)
                if tracer:
                    tracer.end(i, block)
        if tracer:
            self.trace_events = tracer.events()
        outputs = {}
        for op in self.g.ops:
            if not op.out_list:
                v = self.values[op.idx]
                outputs[op.idx] = self._final(v)
        return outputs

    def _final(self, v):
        if isinstance(v, Lazy):
            v = v.force()
        if isinstance(v, (NodeT, EdgeT)):
            return v.t
        if isinstance(v, Scat):
            return self._to_edge_tensor(v)
        if isinstance(v, Deferred):
            return self._materialize_deferred(v).t
        return v

    def tensor_of(self, op_idx):
        return self._final(self.values[op_idx])


class _Tracer:
    """Brackets each op evaluation with HIP events on the current stream (host clock on CPU)."""

    def __init__(self, ex):
        self.ex = ex
        dev = ex.graph.device if ex.graph is not None else torch.device("cpu")
        self.cuda = dev.type == "cuda"
        self.dev = dev
        self.recs = []
        self.t0 = self._mark()

    def _mark(self):
        if self.cuda:
            e = torch.cuda.Event(enable_timing=True)
            e.record(torch.cuda.current_stream(self.dev))
            return e
        return time.perf_counter()

    def _us(self, a, b):
        if self.cuda:
            return a.elapsed_time(b) * 1e3
        return (b - a) * 1e6

    def begin(self):
        self.cur = (self._mark(), self.ex.alg_bytes, self.ex.launches)

    def end(self, i, block):
        m0, b0, l0 = self.cur
        self.recs.append((i, block, m0, self._mark(), self.ex.alg_bytes - b0, self.ex.launches - l0))

    def events(self):
        if self.cuda:
            torch.cuda.synchronize(self.dev)
        out = []
        for i, block, m0, m1, nbytes, nl in self.recs:
            op = self.ex.g.ops[i]
            insts = [ins for ins in getattr(block, "insts", []) if ins.kind == "comp" and
                     any(p[0] == i for p in ins.parts)]
            name = insts[0].type if insts else f"{op.type.upper()}_{op.comp}"
            cat = insts[0].id if insts else f"{i}_{op.type}_0"
            out.append({"name": name, "cat": cat, "ph": "X", "ts": self._us(self.t0, m0),
                        "dur": self._us(m0, m1), "pid": "MI355X", "tid": f"block {block.index}",
                        "args": {"op": i, "alg_bytes": nbytes, "launches": nl}})
        return out


def save_chrome_trace(events, path):
    """Chrome trace JSON (chrome://tracing, Perfetto), as the reference's save_timeline_to_json."""
    import json
    import os
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        json.dump(events, f, indent=1)


def aggregate_trace(events):
    """{name: (count, total µs, total algorithmic bytes)} -- the reference's aggregate_timeline /
    aggregate_rw_record (code/simulator.py:107-146) over measured events."""
    agg = {}
    for e in events:
        c, t, b = agg.get(e["name"], (0, 0.0, 0))
        agg[e["name"]] = (c + 1, t + e["dur"], b + e["args"]["alg_bytes"])
    return agg


# Repeated calls replay a HIP graph (execute() / run_stream / pipeline.Layer.run): the second call
# with the same op graph, stream, CSR and input tensors (same objects; their CONTENTS may change in
# place) captures the whole stream execution once (GraphedRun) and every later call replays it --
# one graph launch instead of one Python-driven launch per op, which is what small layers (Cora,
# Flickr) are bound by, and no host gaps between the kernels of large ones (round 4, every size:
# GAT Reddit 5.61 -> 5.30 ms, GraphSAGE Reddit 4.84 -> 4.73, GIN products 6.54 -> 6.47,
# profiles/r04/layer_bench_graph_all.log).  The outputs of a replayed call are the graph's own
# tensors: the next call with the same inputs overwrites them (clone what must survive it).  A
# captured graph keeps its intermediates in a private memory pool (a few GB for the Reddit-scale
# layers, against 288 GB of HBM); AUTO_GRAPH_MAX_EDGES bounds the graphs it applies to,
# AUTO_GRAPH = False turns it off (set_auto_graph(False) also drops every captured graph).  A replay is keyed by the objects AND their storage (data_ptr,
# shape, stride), the calling thread's libgta knob state (ops.knob_state) and stays eager on a stream with an attached
# knob set; weights changed in place are re-transposed into the graph's W^T before the replay.
FUSE_MLP = True  # default of Executor.fuse_mlp (layer benches A/B it)
MLP_BF16_SUM = True  # default of Executor.mlp_bf16_sum: GIN's sum stored in bf16 for the fused MLP (ABI 10)
AUTO_GRAPH = True
AUTO_GRAPH_MAX_EDGES = 1 << 40  # every graph (round 3: 1 << 23, launch-bound layers only)
AUTO_GRAPH_MAX_ENTRIES = 32
AUTO_GRAPH_MAX_POOL_BYTES = 64 << 30  # private pools of all captured graphs together: the
                                      # largest other entries are dropped beyond it
_AUTO = {}


class _AutoEntry:
    def __init__(self, refs, tensors):
        self.refs, self.tensors = refs, tensors  # strong references: ids and addresses stay unique
        self.ptrs = {k: t.data_ptr() for k, t in tensors.items()}
        self.src = None                          # the caller's dict last seen with these tensors
        self.calls, self.run, self.failed = 0, None, False
        self.pool_bytes = 0                      # device memory the capture reserved (its private pool)
        self.last_use = 0                        # _AUTO_CLOCK value of the latest call (LRU eviction)
        self.evicted = False                     # its graph was dropped for room: it stays eager from then on


_AUTO_CLOCK = [0]
_AUTO_FAST = {}  # (ids of the call's objects, id of its tensors dict, knob state) -> entry: the per-call lookup


def clear_auto_graphs():
    """Drop every captured graph (and the inputs, CSRs and memory pools they hold)."""
    _AUTO.clear()
    _AUTO_FAST.clear()


def set_auto_graph(flag):
    global AUTO_GRAPH
    AUTO_GRAPH = bool(flag)
    if not AUTO_GRAPH:
        clear_auto_graphs()


def _auto_graph(opgraph, stream, graph, tensors, semantics, plan_chunk):
    """-> a GraphedRun to replay for this call, or None (run eagerly)."""
    if ops.Tuning.attached(torch.cuda.current_stream(graph.device)):
        return None  # a knob set on this stream: every call reads it (gta.h), so no cached graph
    refs = (opgraph, stream, graph, semantics)
    fkey = (id(opgraph), id(stream), id(graph), id(semantics), plan_chunk, id(tensors), ops.knob_state())
    ent = _AUTO_FAST.get(fkey)
    if ent is not None and not (ent.src is tensors and all(a is b for a, b in zip(ent.refs, refs)) and
                                len(tensors) == len(ent.tensors) and
                                all(tensors.get(k) is t and t.data_ptr() == ent.ptrs[k]
                                    for k, t in ent.tensors.items())):
        ent = None
    if ent is None:
        if not all(torch.is_tensor(t) and t.is_cuda for t in tensors.values()):
            return None
        key = fkey[:5] + (fkey[6],
                          tuple(sorted((k, id(t), t.data_ptr(), tuple(t.shape), tuple(t.stride()), t.dtype)
                                       for k, t in tensors.items())))
        ent = _AUTO.get(key)
        if ent is not None and not all(a is b for a, b in zip(ent.refs, refs)):
            ent = None
        if ent is None:
            if len(_AUTO) >= AUTO_GRAPH_MAX_ENTRIES:
                _AUTO.pop(next(iter(_AUTO)))
                _AUTO_FAST.clear()
            ent = _AUTO[key] = _AutoEntry(refs, dict(tensors))
        ent.src = tensors
        if len(_AUTO_FAST) >= 4 * AUTO_GRAPH_MAX_ENTRIES:
            _AUTO_FAST.clear()
        _AUTO_FAST[fkey] = ent
    ent.calls += 1
    _AUTO_CLOCK[0] += 1
    ent.last_use = _AUTO_CLOCK[0]
    if ent.failed or ent.evicted or ent.calls < 2:
        return None
    if ent.run is None:
        before = torch.cuda.memory_reserved(graph.device)
        try:
            ent.run = GraphedRun(opgraph, stream, graph, ent.tensors, semantics, plan_chunk, warmup=1)
        except Exception:  # something in this stream is not capturable: stay eager for this key
            ent.failed = True
            torch.cuda.synchronize(graph.device)
            return None
        ent.pool_bytes = max(0, torch.cuda.memory_reserved(graph.device) - before)
        _evict_pools(keep=ent)
    return ent.run


def _evict_pools(keep):
    """Keep the captured graphs' pools within AUTO_GRAPH_MAX_POOL_BYTES (a Reddit / products-sized
    layer holds GBs of intermediates): drop the graphs of the least recently used entries other than
    `keep`, and mark those entries to stay eager.  (deleting the largest other entry made
    two large alternating layers evict each other on every capture and recapture two calls later --
    repeated captures and warm-ups instead of replays.  An evicted entry keeps its call history, so
    it is never recaptured.)  pool_bytes is the memory_reserved() growth across the capture: the
    caching allocator's view, which may under-count a pool that reused freed blocks."""
    total = sum(e.pool_bytes for e in _AUTO.values() if e.run is not None)
    while total > AUTO_GRAPH_MAX_POOL_BYTES:
        victims = [(e.last_use, i, e) for i, e in enumerate(_AUTO.values()) if e.run is not None and e is not keep]
        if not victims:
            break
        _, _, e = min(victims)
        total -= e.pool_bytes
        e.run, e.evicted = None, True


def run_stream(opgraph, stream, graph, tensors, semantics=None, plan_chunk=512, sync=True, trace=False):
    dev = graph.device
    if not AUTO_GRAPH and _AUTO:
        clear_auto_graphs()
    if AUTO_GRAPH and not trace and dev.type == "cuda" and graph.nnz <= AUTO_GRAPH_MAX_EDGES:
        gr = _auto_graph(opgraph, stream, graph, tensors, semantics, plan_chunk)
        if gr is not None:
            if sync:
                torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            outputs = gr.replay()
            if sync:
                torch.cuda.synchronize(dev)
            ex = gr.executor
            return ExecResult(ex.values, outputs, time.perf_counter() - t0, ex.alg_bytes, ex.launches), ex
    ex = Executor(opgraph, stream, graph, tensors, semantics, plan_chunk)
    ex.trace = trace
    sync = sync and dev.type == "cuda"
    if sync:
        torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    outputs = ex.run()
    if sync:
        torch.cuda.synchronize(dev)
    dt = time.perf_counter() - t0
    return ExecResult(ex.values, outputs, dt, ex.alg_bytes, ex.launches), ex


def _tiles_for(graph, sparse=True):
    """T -> the tile counts of graph for the cost model, cached on the graph object like its plans:
    sparse (tiles.sparse_counts, O(E)) for the closed-form per-instruction model, or the dense flat
    list (gta_tile_nnz on the GPU, row-major [ceil(N/T)][n_cols]) the cycle loop walks.  Like the
    reference's dense adjacency they count a repeated (dst, src) once when rows are column-sorted."""
    from . import tiles
    cache = graph.__dict__.setdefault("_tile_nnz_cache", {})

    def tiles_for(T):
        key = (T, sparse)
        if key not in cache:
            cache[key] = (tiles.sparse_counts(graph, int(T)) if sparse
                          else ops.tile_nnz(graph, int(T)).flatten().cpu().numpy().astype(np.int64))
        return cache[key]
    return tiles_for


def attach_model(res, stream_records, tile_size_list, graph, model="rw", isSinput=False, dataset=None):
    """The reference's modelled numbers for the stream just executed (simulate(), code/simulator.py:370-502):
      "rw"   res.model_rw, the closed form (one tile-count pass at T = N);
      "inst" also res.model_insts, the per-instruction model (costmodel.per_instruction: each
             instruction's rw_record bytes and unit-busy cycles, closed form over sparse tile counts:
             runs at Reddit / products scale), res.model_rw its sum;
      "full" also res.model_cycles and res.model_spans via the exact cycle-loop restatement
             (costmodel.simulate_stream with each instruction's first start / last end; Python
             speed: Cora / Flickr-sized graphs)."""
    from . import costmodel
    if model is None:
        return res
    n = graph.n_rows
    sp = SPARSITY.get(dataset, 1)
    if model == "rw":
        cache = graph.__dict__.setdefault("_tile_nnz_cache", {})
        if ("sum", n) not in cache:
            cache[("sum", n)] = int(ops.tile_nnz(graph, n).sum().item())
        res.model_rw = costmodel.model_rw(stream_records, n, cache[("sum", n)])
        return res
    res.model_insts = costmodel.per_instruction(stream_records, tile_size_list, n, _tiles_for(graph), isSinput, sp)
    res.model_rw = sum(r["rw_bytes"] for r in res.model_insts)
    if model == "full":
        res.model_cycles, rw, res.model_spans = costmodel.simulate_stream(
            stream_records, tile_size_list, n, _tiles_for(graph, sparse=False), isSinput, sp, record=True)
        assert rw == res.model_rw, (rw, res.model_rw)
    return res


def model_trace(res, events=None):
    """The modelled numbers beside the measured Chrome trace.  Every measured op event gets, in
    args.model, the stream instructions that execute it (by the op ids in their IDs) with their
    modelled bytes (rw_record) and unit-busy cycles / µs at the reference's 1 GHz clock
    (code/start.py:56 reports cycles/1e9 s).  With model="full" the modelled timeline is added as
    its own tracks: one event per instruction from its first start to its last end, pid
    "GTA model", tid = the reference's hardware unit (vTCAD/code/simulator.py:360-382 schema)."""
    insts = getattr(res, "model_insts", None) or []
    by_op = {}
    for r in insts:
        for op in {p[0] for p in ir.parse_id(r["ID"])}:
            by_op.setdefault(op, []).append({"TYPE": r["TYPE"], "ID": r["ID"], "bytes": r["record_bytes"],
                                             "busy_cycles": r["busy"], "model_us": r["busy"] / 1e3,
                                             "iterations": r["starts"]})
    out = []
    for e in events or []:
        e = dict(e, args=dict(e["args"]))
        e["args"]["model"] = by_op.get(e["args"]["op"], [])
        out.append(e)
    spans = getattr(res, "model_spans", None)
    if spans:
        for r in insts:
            sp = spans.get((r["block"], r["index"]))
            if sp is None:
                continue
            out.append({"name": r["TYPE"], "cat": r["ID"], "ph": "X", "ts": sp[0] / 1e3, "dur": (sp[2] - sp[0]) / 1e3,
                        "pid": "GTA model", "tid": r["unit"],
                        "args": {"bytes": r["record_bytes"], "busy_cycles": r["busy"], "iterations": r["starts"],
                                 "block": r["block"]}})
    return out


SPARSITY = {"cora": 0.012, "pubmed": 0.1, "flickr": 0.46, "reddit": 1}  # code/simulator.py:381-392


_LOADED = {}


def _load(network, reorder, semantics, op_path, inst_path):
    """(semantics, op graph, stream records, stream) of a layer, kept while its files are unchanged:
    repeated execute() calls then hand run_stream the same objects, so they replay one HIP graph."""
    def stamp(p):
        st = os.stat(p)
        return p, st.st_mtime_ns, st.st_size
    key = (network, bool(reorder), id(semantics), stamp(op_path), stamp(inst_path))
    hit = _LOADED.get(key)
    if hit is None or hit[0] is not semantics:
        sem = semantics or Semantics.for_network(network, reorder)
        g = ir.OpGraph.load(op_path, sem.inputs)
        records = ir.read_yaml(inst_path)
        if len(_LOADED) >= 64:
            _LOADED.clear()
        hit = _LOADED[key] = (semantics, sem, g, records, ir.Stream(records))
    return hit[1:]


ARCHITECTURES = ("GTA", "HyGCN", "GCNAX", "OPU")  # vTCAD/code/simulator.py:489-509


def execute(tile_size_list, dataset, network, layer, isReorder, isSinput=False, isFlexibleHardware=False,
            architecture_name="GTA", *, graph, tensors, inst_root="Results/Insts", op_root="Network", inst_path=None,
            op_path=None, semantics=None, plan_chunk=512, model="rw", trace=None):
    """Drop-in for simulate(tile_size_list, dataset, network, layer, isReorder, isSinput)
    (code/simulator.py:370): same leading arguments, same files, real execution.

    Returns ExecResult: the sink ops' device tensors, measured elapsed_s, and the
    reference's modelled numbers for the same stream (attach_model): model_rw (always, closed
    form), model_insts (model="inst" or "full": per instruction, the bytes simulate() records in
    rw_record and the unit-busy cycles, closed form at any graph size) and model_cycles /
    model_spans (model="full"; exact restatement of the cycle loop, Python-speed, meant for
    Cora/Flickr-sized graphs).  `res.simulate_tuple()` is what simulate() would have returned.
    trace: True (events in res.trace) or a path for a Chrome trace JSON of the measured per-op
    device time, as the reference's chrome_timeline.json, each op event carrying its
    instructions' modelled bytes and cycles (model_trace; model="full" adds the modelled timeline).

    Also takes vTCAD's call, simulate(tile_size_list, dataset, network, layer, isReorder, isSinput,
    isFlexibleHardware, architecture_name) (vTCAD/code/simulator.py:423, called positionally at
    vTCAD/code/test.py:15; bind() gives a callable that takes exactly that line).  The names are
    checked as vTCAD checks them (:489-510: an unknown architecture is an error -- vTCAD returns -1,
    this raises) and kept in res.model_arch.  They select the modelled ASIC, not the execution: the
    GPU runs the same kernels for every architecture, and the modelled numbers restate
    code/simulator.py's fixed-hardware GTA model; vTCAD's other presets and its per-block search
    over flexible unit counts are ASIC design-space models outside the hot path.

    From the second call with the same stream, CSR and input tensor objects on (graphs of at most
    AUTO_GRAPH_MAX_EDGES edges: every graph by default), the execution replays a captured HIP graph: the outputs are then
    the graph's own tensors and the next such call overwrites them -- clone what must outlive it
    (AUTO_GRAPH = False keeps every call eager, with fresh outputs)."""
    if architecture_name not in ARCHITECTURES:
        raise ValueError(f"architecture_name {architecture_name!r}: vTCAD knows {', '.join(ARCHITECTURES)} "
                         "(vTCAD/code/simulator.py:489-510)")
    if not isinstance(isFlexibleHardware, (bool, int)):
        raise TypeError("isFlexibleHardware must be a bool")
    op_path = op_path or ir.op_yaml_path(network, dataset, layer, isReorder, op_root)
    inst_path = inst_path or ir.inst_path(network, dataset, layer, isReorder, inst_root)
    sem, g, records, s = _load(network, isReorder, semantics, op_path, inst_path)
    res, ex = run_stream(g, s, graph, tensors, sem, plan_chunk, trace=trace is not None)
    # a trace carries the per-instruction model beside the measured ops
    attach_model(res, records, tile_size_list, graph, "inst" if (trace is not None and model == "rw") else model,
                 isSinput, dataset)
    if trace is not None:
        res.trace = model_trace(res, ex.trace_events)
        if isinstance(trace, str):
            save_chrome_trace(res.trace, trace)
    # vTCAD turns flexible hardware off for every preset but GTA (:493-507)
    res.model_arch = (architecture_name, bool(isFlexibleHardware) and architecture_name == "GTA")
    return res


def bind(graph, tensors, **kw):
    """A simulate()-shaped callable over one graph and its tensors: bind(g, t)(tile_size_list,
    dataset, network, layer, isReorder, isSinput[, isFlexibleHardware, architecture_name]) -- the
    reference callers' lines (code/start.py:51, code/genetic_algorithm.py:603, vTCAD/code/test.py:15)
    unchanged once `simulate` names it."""
    import functools
    return functools.partial(execute, graph=graph, tensors=tensors, **kw)


class GraphedRun:
    """A stream execution captured once as a HIP graph and replayed (torch.cuda.CUDAGraph is
    hipGraph on ROCm): every libgta launch of the layer is recorded, so a replay costs one graph
    launch instead of one Python-driven launch per op -- the launch-bound small graphs (Cora,
    Flickr) are where it matters.  Inputs are the tensors given here (static addresses: update
    them in place between replays); outputs are the same tensors after every replay.  The
    warm-up run builds every plan, workspace and W^T cache outside the capture.  The graph keeps
    the W^T tensors (and sibling-weight concatenations) it reads alive, and a weight changed in
    place (its version moved) is re-concatenated / re-transposed into them before the next replay."""

    def __init__(self, opgraph, stream, graph, tensors, semantics=None, plan_chunk=512, warmup=2):
        if graph.device.type != "cuda":
            raise RuntimeError("GraphedRun captures device launches: the graph must be on a HIP device")
        self.tensors = tensors
        side = torch.cuda.Stream(graph.device)
        side.wait_stream(torch.cuda.current_stream(graph.device))
        with torch.cuda.stream(side):
            for _ in range(max(1, warmup)):
                Executor(opgraph, stream, graph, tensors, semantics, plan_chunk).run()
        torch.cuda.current_stream(graph.device).wait_stream(side)
        torch.cuda.synchronize(graph.device)
        self.cuda_graph = torch.cuda.CUDAGraph()
        del ops._CAPTURED_WT[:]
        del _CAPTURED_WCAT[:]
        try:
            with torch.cuda.graph(self.cuda_graph):
                self.executor = Executor(opgraph, stream, graph, tensors, semantics, plan_chunk)
                self.outputs = self.executor.run()
        finally:
            taken, ops._CAPTURED_WT[:] = list(ops._CAPTURED_WT), []
            cats, _CAPTURED_WCAT[:] = list(_CAPTURED_WCAT), []
        # (sibling weights, their concatenation read by the graph, the versions it holds); refreshed
        # before the W^T below, so a re-concatenation moves Wc's version and re-transposes it too
        self._wcats = [[srcs, wc, tuple(w._version for w in srcs)]
                       for srcs, wc in {id(wc): (srcs, wc) for srcs, wc in cats}.values()]
        # (weight, its W^T read by the graph, the weight version that W^T holds)
        self._wts = [[w, wt, w._version] for w, wt in {id(wt): (w, wt) for w, wt in taken}.values()]

    def replay(self):
        for ent in self._wcats:
            srcs, wc, vers = ent
            now = tuple(w._version for w in srcs)
            if now != vers:  # a sibling weight changed in place: re-concatenate into the graph's copy
                wc.copy_(torch.cat(srcs, dim=1))
                ent[2] = now
        for ent in self._wts:
            w, wt, ver = ent
            if w._version != ver:  # changed in place since the capture: refresh the graph's W^T
                wt.copy_(w.t())
                ent[2] = w._version
        self.cuda_graph.replay()
        return self.outputs

