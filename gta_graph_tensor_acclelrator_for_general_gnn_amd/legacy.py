"""Legacy V2 path (BASELINE config 0): V2 op graph -> fused_template stream -> execution.

  lower_v2     restates V2/interpreter.py:13-271 (create_list): per op, the byte counts
               and shapes of its loads / computes / saves (template/fused_template.yaml
               schema), times_1/2/3 and isR.  Output is byte-identical under
               yaml.safe_dump to the reference's own files (tests/golden/v2/, made by
               running create_list; case 0 is the committed V2/fused.yaml).
  LegacyStream the per-op records as executor blocks (one block per op list entry).
  execute_v2   runs a V2 stream on the HIP executor.  V2 op graphs carry no COMP_TYPE;
               comp_types() assigns them from the op structure (the typing genGraphOP
               gives the same 14-op GAT, vTCAD/GraphOP/genGraphOP.py:51-60).

Reference quirks kept: the sparse_path prefix is the author's absolute path
(V2/interpreter.py:50); a scatter or gather with an empty output list indexes
output_list[0] and raises IndexError (:66-67, :131-132), as does a gather with an
empty input list (:92-93).
"""
import math

import yaml

from . import executor, ir
from .semantics import Semantics

_SPARSE = "/Users/sijin/Desktop/RA/MPAD/Eva/Compiler/data/adj_{}_{}_1.yaml"  # V2/interpreter.py:50


def _record(op, block, tile, node_num, dataset):
    """One create_list record (V2/interpreter.py:24-255) for op record `op` inside `block`."""
    kind, order = op["TYPE"], op["ORDER"]
    inp, out = op["INPUT"], op["OUTPUT"]
    gl, spf, osz, outs = inp["input_g_list"], inp["size_per_feature"], out["size_per_feature"], out["output_list"]
    r = dict(w_list=[], load_list=[], load_shape=[], compute_list=[], compute_shape=[], compute_type=[],
             save_list=[], save_shape=[], type=kind, sparse_path="", isR=1)
    edge_shape = [node_num, tile]
    outside = [o not in block for o in outs]

    def weights():
        if inp["input_nong_num"] != 0:
            r["compute_type"].append(0)
            r["w_list"] += [[inp["input_size"][w] / spf[w], spf[w]] for w in range(len(inp["input_size"]))]
        else:
            r["w_list"].append([0, 0])
            r["compute_type"].append(1)

    if kind == "scatter":  # :43-87
        r["w_list"].append([0, 0])
        r["compute_type"].append(-1)
        r["compute_list"].append(0)
        r["compute_shape"].append(0)
        r["sparse_path"] = _SPARSE.format(dataset, tile)
        for k, g in enumerate(gl):
            if g in block:
                r["load_list"].append(0)
                r["load_shape"].append([0, 0])
            elif order == "R":
                r["load_list"].append(spf[k])
                r["load_shape"].append([tile, 1])
            else:
                r["isR"] = 0
                r["load_list"].append(spf[k])
                r["load_shape"].append([1, 1])
        if not outs:
            raise IndexError("list index out of range")  # output_list[0] on an empty list, :66-67
        for o in outside:
            if not o:
                r["save_list"].append(0)
                r["save_shape"].append([0, 0])
                continue
            r["save_list"].append(osz)
            if order != "R":
                r["isR"] = 0
            r["save_shape"].append([node_num, tile] if order == "R" else [1, tile])
    elif kind == "gather":  # :88-160
        r["w_list"].append([0, 0])
        r["sparse_path"] = _SPARSE.format(dataset, tile)
        if not gl:
            raise IndexError("list index out of range")  # input_g_list[k] on an empty list, :92-93
        for k, g in enumerate(gl):
            if g in block:
                r["load_list"].append(0)
                r["load_shape"].append([0, 0])
                continue
            if order != "R":
                r["isR"] = 0
            r["load_list"] += [osz, spf[k] if order == "R" else spf[k] * tile]
            r["load_shape"] += [[tile, 1], list(edge_shape)]
        r["compute_type"].append(1)
        r["compute_list"].append(osz)
        if order != "R":
            r["isR"] = 0
        r["compute_shape"].append(list(edge_shape) if order == "R" else [1, tile])
        if not outs:
            raise IndexError("list index out of range")  # :131-132
        for o in outside:
            if not o:
                r["save_list"].append(0)
                r["save_shape"].append([0, 0])
                continue
            r["save_list"].append(osz)
            if order != "R":
                r["isR"] = 0
            r["save_shape"].append([1, tile] if order == "R" else [1, 1])
    else:  # applynode :162-206 / applyedge :208-255
        node = kind == "applynode"
        shape = [1, 1] if node else edge_shape
        if not node:
            r["sparse_path"] = _SPARSE.format(dataset, tile)
            r["type"] = "applyedge"
        weights()
        if not gl:
            r["load_list"].append(spf[0])
            r["load_shape"].append(list(shape))
        for k, g in enumerate(gl):
            r["load_list"].append(0 if g in block else spf[k])
            r["load_shape"].append([0, 0] if g in block else list(shape))
        r["compute_list"].append(inp["input_size"][0] / 4 if inp["input_nong_num"] != 0 else spf[0])
        r["compute_shape"].append(list(shape))
        if not outs:
            r["save_list"].append(osz)
            r["save_shape"].append(list(shape))
        for o in outside:
            r["save_list"].append(osz if o else 0)
            r["save_shape"].append(list(shape) if o else [0, 0])
    r["times_1"] = math.ceil(node_num / tile)
    r["times_2"] = node_num
    r["times_3"] = tile
    return r


def lower_v2(dataset, op_records, op_list, tile_size, node_num):
    """create_list (V2/interpreter.py:13-271) -> {record index: record}, in op_list order."""
    res = {}
    for i, block in enumerate(op_list):
        for no in block:
            rec = _record(op_records[no], block, tile_size[i], node_num, dataset)
            rec["OP_NO"] = no
            res[len(res)] = rec
    return res


def dump(res):
    """The reference writes with yaml.safe_dump (V2/interpreter.py:257-258)."""
    return yaml.safe_dump(res)


def comp_types(op_records):
    """COMP_TYPE per op of a V2 op graph (which has none): MM for weighted applies, NONE for
    scatters, ADD for gathers, SF for single-input applies, and for two-input applyedges ADD
    when both inputs are scatters (score sum) else MUL -- the typing genGraphOP gives the same
    graph (GAT: MM MM MM NONE NONE NONE ADD SF ADD MUL NONE MUL ADD SF)."""
    kinds = {r["OP_NO"]: r["TYPE"] for r in op_records}
    out = []
    for r in op_records:
        t, gl = r["TYPE"], r["INPUT"]["input_g_list"]
        if t == "scatter":
            out.append("NONE")
        elif t == "gather":
            out.append("ADD")
        elif r["INPUT"]["input_nong_num"] != 0:
            out.append("MM")
        elif len(gl) <= 1:
            out.append("SF")
        elif t == "applyedge" and all(kinds.get(g) == "scatter" for g in gl):
            out.append("ADD")
        else:
            out.append("ADD" if t == "applynode" else "MUL")
    return out


def typed_records(op_records):
    """Op records with COMP_TYPE: kept where the graph has it (genGraphOP's), inferred otherwise."""
    recs = []
    for r, c in zip(op_records, comp_types(op_records)):
        r = dict(r)
        r.setdefault("COMP_TYPE", c)
        recs.append(r)
    return recs


class _Block:
    def __init__(self, index, ops, stored):
        self.index, self.ops, self.stored, self.fused = index, sorted(ops), sorted(stored), []


class LegacyStream:
    """lower_v2 records grouped into executor blocks (op_list order; one block per op if
    op_list is not given).  V2 records carry no instruction fusion, so no block has fused COMPs."""

    def __init__(self, records, op_list=None):
        recs = [records[k] for k in sorted(records)]
        if op_list is None:
            op_list = [[r["OP_NO"]] for r in recs]
        stored = {r["OP_NO"] for r in recs if any(s for s in r["save_list"])}
        self.blocks = [_Block(i, b, [o for o in b if o in stored]) for i, b in enumerate(op_list)]
        self.records = recs

    def __iter__(self):
        return iter(self.blocks)

    def __len__(self):
        return len(self.blocks)


SEMANTICS = {  # the build's choices for the V2 graphs (cf. semantics.py)
    "GAT": Semantics(sf={7: "EXP_LEAKY_RELU", 13: "ELU"}, bin={9: "DIV"}),
    "simpletest": Semantics(sf={6: "EXP_LEAKY_RELU", 8: "ELU"}),
}


def execute_v2(op_records, stream_records, graph, tensors, network="GAT", op_list=None, plan_chunk=512,
               reorder=False):
    """Run a V2 stream (lower_v2 output) on the HIP executor -> (ExecResult, Executor).  network names
    the V2 graphs ("GAT" = V2/GAT_Cora.yaml, "simpletest") or any genGraphOP network."""
    sem = SEMANTICS.get(network) or Semantics.for_network(network, reorder)
    g = ir.OpGraph(typed_records(op_records), sem.inputs)
    return executor.run_stream(g, LegacyStream(stream_records, op_list), graph, tensors, sem, plan_chunk)


# ---------------------------------------------------------------------------------------------
# The legacy execution boundary: pipeline(data, op_fused, isCycle) -> (total_p, record, rw)
# ---------------------------------------------------------------------------------------------
V2_HARDWARE = {  # V2/simulator.py:213-222 (the module's __main__ sets these globals before pipeline)
    "bw": 128 * (1024 ** 3) * (10 ** (-9)),  # bytes per cycle (128 GB/s at 1 cycle = 1 ns)
    "compute_perfom": [[16, 16], [16, 16]],  # [mm, ele-wise] x [pl_in, pl_out]
}


def v2_sparsity(graph, T, C=1):
    """The sparse table V2's pipeline reads from `sparse_path` (adj_<dataset>_<T>_<C>.yaml), from a
    CSR: V2/preprocessing.py:11-38 pads the dense adjacency (rows = destination, cols = source) to
    whole T x C blocks and counts, per block, the entries EQUAL to zero (`count_nonzero(block ==
    0)`: the zeros, not the edges -- a reference quirk kept here), with self loops and padding
    included.  -> list of lists [ceil(N / T)][ceil(n_cols / C)]."""
    import numpy as np
    ip, ix = graph.numpy()
    n, m = len(ip) - 1, int(graph.n_cols)
    rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(ip))
    key = np.unique(rows * m + ix.astype(np.int64))  # a dense matrix holds each (dst, src) once
    r, c = key // m, key % m
    nr, nc = -(-n // T), -(-m // C)
    nnz = np.bincount((r // T) * nc + c // C, minlength=nr * nc).reshape(nr, nc)
    return (T * C - nnz).tolist()


class _V2Model:
    """V2/simulator.py:18-209 restated: one in-order load / compute / save timeline per call,
    state starting at zero as the module's __main__ leaves it (:224-230)."""

    def __init__(self, sparse, hardware=None):
        hw = dict(V2_HARDWARE, **(hardware or {}))
        self.bw, self.perf = hw["bw"], hw["compute_perfom"]
        self.sparse = sparse
        self.load_p = self.save_p = self.save_start_p = self.c_p = self.total_p = 0
        self.compute_p = [0, 0]
        self.rw = 0

    def _lat(self, x, isCycle):
        return math.ceil(x) * (10 ** (-9)) if isCycle == 0 else math.ceil(x)

    def load(self, data, isCycle):  # :18-40 (the position compare adds bytes to a time: kept)
        self.rw += data
        latency = self._lat(data / self.bw, isCycle)
        if self.load_p + data > self.save_start_p and self.save_start_p != 0:
            self.load_p = self.save_p + latency
        else:
            self.load_p += latency
        if self.load_p > self.c_p and self.load_p > self.save_p:
            self.total_p = self.load_p

    def compute(self, data, t, isCycle):  # :42-71
        p = self.perf[t]
        if isCycle == 0:
            latency = math.ceil(data[0] / p[0]) * math.ceil(data[1] / p[1]) * (10 ** (-9))
        else:
            latency = math.ceil(data[0] / p[0]) * math.ceil(data[1] / p[1])
        if t in (0, 1):
            if self.load_p < self.compute_p[t]:
                self.compute_p[t] += latency
            else:
                self.compute_p[t] = self.load_p + latency
        self.c_p = self.compute_p[0] if self.compute_p[0] > self.compute_p[1] else self.compute_p[1]
        if self.c_p > self.load_p and self.c_p > self.save_p:
            self.total_p = self.c_p

    def save(self, data, isCycle):  # :73-96
        self.rw += data
        latency = self._lat(data / self.bw, isCycle)
        if self.c_p < self.save_p:
            self.save_p += latency
        else:
            self.save_start_p = self.c_p
            self.save_p = self.c_p + latency
        if self.save_p > self.load_p and self.save_p > self.c_p:
            self.total_p = self.save_p

    def decode(self, d, kind, isCycle, optype, t1, t2, sp):  # :98-149
        if kind == "load":
            # :108-117 appends a 0 and skips the entry when it is 0: decode never loads anything
            return
        if kind == "compute":
            for j in range(len(d["compute_list"])):
                ct, w = d["compute_type"][j], d["w_list"][j]
                if optype in ("gather", "applyedge"):
                    cd = [w[1] / 4, sp[t1][t2]] if ct == 1 else [w[0], w[1] / 4 * sp[t1][t2]]
                else:
                    cs = d["compute_shape"][j]
                    cd = [w[1] / 4, cs[0] * cs[1]] if ct == 1 else [w[0], w[1] / 4 * cs[0] * cs[1]]
                self.compute(cd, ct, isCycle)
            return
        for j in range(len(d["save_list"])):
            if d["save_list"][j] == 0:
                continue
            if optype in ("scatter", "applyedge"):
                self.save(d["save_list"][j] * sp[t1][t2], isCycle)
            else:
                self.save(d["save_list"][j] * d["save_shape"][j][1], isCycle)

    def run(self, data, op_fused, isCycle):  # :152-209
        record, sp = [], []
        for blk in op_fused:
            head = data[blk[0]]
            for t1 in range(int(head["times_1"])):
                for op in blk:
                    d = data[op]
                    record.append(self.total_p)
                    kind = d["type"]
                    if kind in ("scatter", "gather", "applyedge"):
                        sp = self.sparse(d["sparse_path"])
                    if kind == "scatter":
                        for t2 in range(int(head["times_2"])):
                            self.decode(d, "save", isCycle, "scatter", t1, t2, sp)
                    elif kind == "gather" and d["isR"] == 1:
                        for t2 in range(int(head["times_2"])):
                            self.decode(d, "compute", isCycle, "gather", t1, t2, sp)
                        self.decode(d, "save", isCycle, "gather", t1, -1, sp)
                    elif kind == "gather":
                        for t2 in range(int(head["times_2"])):
                            self.decode(d, "compute", isCycle, "gather", t1, t2, sp)
                            self.decode(d, "save", isCycle, "gather", t1, t2, sp)
                    elif kind == "applynode":
                        if t1 == 0:
                            for w in d["w_list"]:
                                self.load(w[0] * w[1], isCycle)
                        for t3 in range(int(head["times_3"])):
                            self.decode(d, "compute", isCycle, "applynode", t1, t3, sp)
                            self.decode(d, "save", isCycle, "applynode", t1, t3, sp)
                    else:
                        if t1 == 0:
                            for w in d["w_list"]:
                                self.load(w[0] * w[1], isCycle)
                        for t2 in range(int(head["times_2"])):
                            self.decode(d, "compute", isCycle, "applyedge", t1, t2, sp)
                            self.decode(d, "save", isCycle, "applyedge", t1, t2, sp)
        return self.total_p, record, self.rw


def sparse_reader(graph=None, tables=None):
    """path -> sparse table, as V2's read(sparse_path): a table given for that path, else the file if
    it exists, else (graph given) v2_sparsity(graph, T, C) with T and C taken from the reference's
    file name pattern adj_<dataset>_<T>_<C>.yaml (V2/interpreter.py:50)."""
    import os
    import re
    cache = dict(tables or {})

    def read(path):
        if path not in cache:
            if os.path.exists(path):
                with open(path) as f:
                    cache[path] = yaml.safe_load(f)
            else:
                m = re.search(r"_(\d+)_(\d+)\.yaml$", path)
                if graph is None or m is None:
                    raise FileNotFoundError(path)
                cache[path] = v2_sparsity(graph, int(m.group(1)), int(m.group(2)))
        return cache[path]
    return read


def pipeline_model(data, op_fused, isCycle, sparse, hardware=None):
    """V2/simulator.py pipeline(data, op_fused, isCycle) -> (total_p, record, rw), exactly, with
    `sparse(path)` standing for its read(sparse_path).  isCycle 1: cycles; 0: seconds."""
    return _V2Model(sparse, hardware).run(data, op_fused, isCycle)


class V2Result(tuple):
    """(total_p, record, rw) -- what V2's pipeline returns, so `total_p, record, rw = pipeline(...)`
    keeps working -- plus the executed layer: .outputs (sink op -> tensor), .result (ExecResult),
    .executor."""

    def __new__(cls, triple, result=None, ex=None):
        self = super().__new__(cls, triple)
        self.result, self.executor = result, ex
        self.outputs = result.outputs if result is not None else {}
        return self


def bind_v2(op_records, graph, tensors, network="GAT", sparse=None, hardware=None, execute=True):
    """The legacy boundary as a drop-in: a callable with V2's signature pipeline(data, op_fused,
    isCycle) (V2/simulator.py:152) that EXECUTES the stream `data` (create_list / fused.yaml
    records, keyed by record index; op_fused = blocks of record indices) on libgta over `graph` /
    `tensors`, and returns the reference's modelled (total_p, record, rw) for the same call as a
    V2Result carrying the outputs.  op_records: the V2 op graph the stream was lowered from (the
    records name ops only by OP_NO).  sparse: {sparse_path: table} overriding the reader."""
    read = sparse_reader(graph, sparse)

    def pipeline(data, op_fused, isCycle):
        data = {int(k): v for k, v in data.items()}
        triple = pipeline_model(data, op_fused, isCycle, read, hardware)
        if not execute:
            return V2Result(triple)
        op_list = [[data[k]["OP_NO"] for k in blk] for blk in op_fused]
        res, ex = execute_v2(op_records, data, graph, tensors, network, op_list=op_list)
        return V2Result(triple, res, ex)
    return pipeline
