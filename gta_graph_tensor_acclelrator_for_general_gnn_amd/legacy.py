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
