"""Op-graph front end: GNN layer -> op-graph records (the op_template of the IR).

Restates vTCAD/GraphOP/genGraphOP.py:27-154 (gen_yaml) as data: each network is a
table of op rows with symbolic sizes, expanded per layer.  Pinned byte-for-byte
against the reference's YAML for all 7 networks x 3 layers x original/trans
(tests/test_frontend.py).  Sizes are bytes of fp32 features, as in the reference:
  fin  = [0, F, 128, 64, 16][layer]   input width      (genGraphOP.py:31)
  fout = [0, 128, 64, 16][layer]      output width     (genGraphOP.py:32)
  fh   = 16 (weight_size[3])          attention width; `heads` overrides it
The reference's quirks are part of the data (GAT row 2 carries OP_NO 1; GCN-trans
ops 1/2 list themselves as outputs; PNA-trans ops 0/1 list themselves as inputs;
GAT-original op 10 lists input 7).
"""
import yaml

# row: (op_no, comp, type, order, fnum, inputs, g_num, nong, wsize, in_sizes, outputs, onum, osize)
#   fnum/onum: "N"/"E" symbols; wsize/in_sizes/osize: products of fin/fout/fh (bytes = 4 * product)
_N, _E = "N", "E"


def _r(no, comp, kind, order, fnum, ins, g, nong, w, isz, outs, onum, osz):
    return (no, comp, kind, order, fnum, ins, g, nong, w, isz, outs, onum, osz)


_AGG_IN = ("fin",)
TABLE = {
    ("GCN", False): [
        _r(0, "NONE", "scatter", "C", [_N], [], 1, 0, None, ["fin"], [1], _E, "fin"),
        _r(1, "MUL", "applyedge", "R", [_E, _E], [0, -1], 2, 0, None, ["fin", "fin"], [2], _E, "fin"),
        _r(2, "ADD", "gather", "R", [_E], [1], 1, 0, None, ["fin"], [3], _N, "fin"),
        _r(3, "MM", "applynode", "R", [_N], [2], 1, 1, "fin*fout", ["fin"], [], _N, "fout"),
    ],
    ("GCN", True): [
        _r(0, "MM", "applynode", "R", [_N], [], 1, 1, "fin*fout", ["fin"], [1], _N, "fout"),
        _r(1, "NONE", "scatter", "C", [_N], [0], 1, 0, None, ["fout"], [1], _E, "fout"),
        _r(2, "MUL", "applyedge", "R", [_E], [1, -1], 2, 0, None, ["fout", "fout"], [2], _E, "fout"),
        _r(3, "ADD", "gather", "R", [_E], [2], 1, 0, None, ["fout"], [], _N, "fout"),
    ],
    ("GAT", False): [
        _r(0, "MM", "applynode", "R", [_N], [], 1, 1, "fout*fin", ["fin"], [1, 2, 3], _N, "fout"),
        _r(1, "MM", "applynode", "R", [_N], [0], 1, 1, "fout*fh", ["fout"], [4], _N, "fh"),
        _r(1, "MM", "applynode", "R", [_N], [0], 1, 1, "fout*fh", ["fout"], [5], _N, "fh"),
        _r(3, "NONE", "scatter", "C", [_N], [0], 1, 0, None, ["fout"], [11], _E, "fout"),
        _r(4, "NONE", "scatter", "R", [_N], [1], 1, 0, None, ["fh"], [6], _E, "fh"),
        _r(5, "NONE", "scatter", "C", [_N], [2], 1, 0, None, ["fh"], [6], _E, "fh"),
        _r(6, "ADD", "applyedge", "R", [_E, _E], [4, 5], 2, 0, None, ["fh", "fh"], [7], _E, "fh"),
        _r(7, "SF", "applyedge", "R", [_E], [6], 1, 0, None, ["fh"], [8, 9], _E, "fh"),
        _r(8, "ADD", "gather", "R", [_E], [7], 1, 0, None, ["fh"], [10], _N, "fh"),
        _r(9, "MUL", "applyedge", "R", [_E, _E], [7, 10], 2, 0, None, ["fh", "fh"], [11], _E, "fh"),
        _r(10, "NONE", "scatter", "R", [_N], [7], 1, 0, None, ["fh"], [9], _E, "fh"),
        _r(11, "MUL", "applyedge", "R", [_E, _E], [3, 9], 2, 0, None, ["fout", "fh"], [12], _E, "fout"),
        _r(12, "ADD", "gather", "R", [_E], [11], 1, 0, None, ["fout"], [13], _N, "fout"),
        _r(13, "SF", "applynode", "R", [_N], [12], 1, 0, None, ["fout"], [], _N, "fout"),
    ],
    ("GAT", True): [
        _r(0, "MM", "applynode", "R", [_N], [], 1, 1, "fout*fin", ["fin"], [1, 2, 3], _N, "fout"),
        _r(1, "MM", "applynode", "R", [_N], [0], 1, 1, "fout*fh", ["fout"], [4], _N, "fh"),
        _r(1, "MM", "applynode", "R", [_N], [0], 1, 1, "fout*fh", ["fout"], [5], _N, "fh"),
        _r(3, "NONE", "scatter", "C", [_N], [0], 1, 0, None, ["fout"], [11], _E, "fout"),
        _r(4, "NONE", "scatter", "R", [_N], [1], 1, 0, None, ["fh"], [6], _E, "fh"),
        _r(5, "NONE", "scatter", "C", [_N], [2], 1, 0, None, ["fh"], [6], _E, "fh"),
        _r(6, "ADD", "applyedge", "R", [_E, _E], [4, 5], 2, 0, None, ["fh", "fh"], [7], _E, "fh"),
        _r(7, "MUL", "applyedge", "R", [_E, _E], [3, 8], 2, 0, None, ["fout", "fh"], [10], _E, "fout"),
        _r(8, "SF", "applyedge", "R", [_E], [6], 1, 0, None, ["fh"], [9], _E, "fh"),
        _r(9, "ADD", "gather", "R", [_E], [8], 1, 0, None, ["fh"], [11], _N, "fh"),
        _r(10, "ADD", "gather", "R", [_E], [7], 1, 0, None, ["fout"], [11], _N, "fout"),
        _r(11, "MUL", "applynode", "R", [_N, _N], [9, 10], 2, 0, None, ["fh", "fout"], [12], _N, "fout"),
        _r(12, "SF", "applynode", "R", [_N], [11], 1, 0, None, ["fout"], [], _N, "fout"),
    ],
    "SGC": [
        _r(0, "NONE", "scatter", "C", [_N], [], 1, 0, None, ["fin"], [1], _E, "fin"),
        _r(1, "MUL", "applyedge", "R", [_E, _E], [0, -1], 2, 0, None, ["fin", "fin"], [2], _E, "fin"),
        _r(2, "ADD", "gather", "R", [_E], [1], 1, 0, None, ["fin"], [3], _N, "fin"),
        _r(3, "NONE", "scatter", "C", [_N], [2], 1, 0, None, ["fin"], [4], _E, "fin"),
        _r(4, "MUL", "applyedge", "R", [_E, _E], [3, -1], 2, 0, None, ["fin", "fin"], [5], _E, "fin"),
        _r(5, "ADD", "gather", "R", [_E], [4], 1, 0, None, ["fin"], [6], _N, "fin"),
        _r(6, "MM", "applynode", "R", [_N], [5], 1, 1, "fin*fout", ["fin"], [], _N, "fout"),
    ],
    "GraphSAGE": [
        _r(0, "NONE", "scatter", "C", [_N], [], 1, 0, None, ["fin"], [1], _E, "fin"),
        _r(1, "MUL", "applyedge", "R", [_E, _E], [0, -1], 2, 0, None, ["fin", "fin"], [2], _E, "fin"),
        _r(2, "ADD", "gather", "R", [_E], [1], 1, 0, None, ["fin"], [3], _N, "fin"),
        _r(3, "MM", "applynode", "R", [_N], [2], 1, 1, "fin*fout", ["fin"], [5], _N, "fout"),
        _r(4, "MM", "applynode", "R", [_N], [], 1, 1, "fin*fout", ["fin"], [5], _N, "fout"),
        _r(5, "ADD", "applynode", "R", [_N, _N], [3, 4], 2, 0, None, ["fout", "fout"], [6], _N, "fout"),
        _r(6, "SF", "applynode", "R", [_N], [5], 1, 0, None, ["fout"], [], _N, "fout"),
    ],
    "GIN": [
        _r(0, "NONE", "scatter", "C", [_N], [], 1, 0, None, ["fin"], [1], _E, "fin"),
        _r(1, "MUL", "applyedge", "R", [_E, _E], [0, -1], 2, 0, None, ["fin", "fin"], [2], _E, "fin"),
        _r(2, "ADD", "gather", "R", [_E], [1], 1, 0, None, ["fin"], [3], _N, "fin"),
        _r(3, "MUL", "applynode", "R", [_N, _N], [-1, -1], 2, 0, None, ["fin", "1"], [4], _N, "fin"),
        _r(4, "ADD", "applynode", "R", [_N, _N], [2, 3], 2, 0, None, ["fin", "fin"], [5], _N, "fin"),
        _r(5, "MM", "applynode", "R", [_N], [4], 1, 1, "fin*fout", ["fin"], [6], _N, "fout"),
        _r(6, "SF", "applynode", "R", [_N], [5], 1, 0, None, ["fout"], [7], _N, "fout"),
        _r(7, "MM", "applynode", "R", [_N], [6], 1, 1, "fout*fout", ["fout"], [8], _N, "fout"),
        _r(8, "SF", "applynode", "R", [_N], [7], 1, 0, None, ["fout"], [], _N, "fout"),
    ],
    "DGN": [
        _r(0, "NONE", "scatter", "C", [_N], [], 1, 0, None, ["fin"], [2], _E, "fin"),
        _r(1, "NONE", "scatter", "R", [_N], [], 1, 0, None, ["fin"], [2], _E, "fin"),
        _r(2, "ADD", "applyedge", "R", [_E, _E], [0, 1], 2, 0, None, ["fin", "fin"], [3], _E, "fin"),
        _r(3, "MM", "applyedge", "R", [_E], [2], 1, 1, "fin*fout", ["fin"], [7], _E, "fout"),
        _r(4, "NONE", "scatter", "C", [_N], [], 1, 0, None, ["fout"], [6], _E, "fout"),
        _r(5, "NONE", "scatter", "R", [_N], [], 1, 0, None, ["fout"], [6], _E, "fout"),
        _r(6, "ADD", "applyedge", "R", [_E, _E], [4, 5], 2, 0, None, ["fout", "fout"], [7], _E, "fout"),
        _r(7, "ADD", "applyedge", "R", [_E, _E], [3, 6], 2, 0, None, ["fout", "fout"], [8], _E, "fout"),
        _r(8, "ADD", "gather", "R", [_E], [7], 1, 0, None, ["fout"], [9], _N, "fout"),
        _r(9, "MUL", "applynode", "R", [_N], [8], 1, 0, None, ["fout"], [10], _N, "fout"),
        _r(10, "SF", "applynode", "R", [_N], [9], 1, 0, None, ["fout"], [], _N, "fout"),
    ],
    ("PNA", False): [
        _r(0, "NONE", "scatter", "C", [_N], [], 1, 0, None, ["fin"], [3], _E, "fin"),
        _r(1, "NONE", "scatter", "R", [_N], [], 1, 0, None, ["fin"], [4], _E, "fin"),
        _r(2, "MM", "applyedge", "R", [_E], [], 1, 1, "fin*fout", ["fin"], [6], _E, "fout"),
        _r(3, "MM", "applyedge", "R", [_E], [0], 1, 1, "fin*fout", ["fin"], [5], _E, "fout"),
        _r(4, "MM", "applyedge", "R", [_E], [1], 1, 1, "fin*fout", ["fin"], [5], _E, "fout"),
        _r(5, "ADD", "applyedge", "R", [_E, _E], [3, 4], 2, 0, None, ["fout", "fout"], [6], _E, "fout"),
        _r(6, "ADD", "applyedge", "R", [_E, _E], [2, 5], 2, 0, None, ["fout", "fout"], [7], _E, "fout"),
        _r(7, "SF", "applyedge", "R", [_E], [6], 1, 0, None, ["fout"], [8], _E, "fout"),
        _r(8, "ADD", "gather", "R", [_E], [7], 1, 0, None, ["fout"], [9], _N, "fout"),
        _r(9, "MUL", "applynode", "R", [_N], [8], 1, 0, None, ["fout"], [10], _N, "fout"),
        _r(10, "MM", "applynode", "R", [_N], [9], 1, 1, "fout*fout", ["fout"], [], _N, "fout"),
    ],
    ("PNA", True): [
        _r(0, "MM", "applynode", "R", [_N], [0], 1, 1, "fin*fout", ["fin"], [3], _N, "fout"),
        _r(1, "MM", "applynode", "R", [_N], [1], 1, 1, "fin*fout", ["fin"], [4], _N, "fout"),
        _r(2, "MM", "applyedge", "R", [_E], [], 1, 1, "fin*fout", ["fin"], [6], _E, "fout"),
        _r(3, "NONE", "scatter", "C", [_N], [], 1, 0, None, ["fout"], [5], _E, "fout"),
        _r(4, "NONE", "scatter", "R", [_N], [], 1, 0, None, ["fout"], [5], _E, "fout"),
        _r(5, "ADD", "applyedge", "R", [_E, _E], [3, 4], 2, 0, None, ["fout", "fout"], [6], _E, "fout"),
        _r(6, "ADD", "applyedge", "R", [_E, _E], [2, 5], 2, 0, None, ["fout", "fout"], [7], _E, "fout"),
        _r(7, "SF", "applyedge", "R", [_E], [6], 1, 0, None, ["fout"], [8], _E, "fout"),
        _r(8, "ADD", "gather", "R", [_E], [7], 1, 0, None, ["fout"], [9], _N, "fout"),
        _r(9, "MUL", "applynode", "R", [_N], [8], 1, 0, None, ["fout"], [10], _N, "fout"),
        _r(10, "MM", "applynode", "R", [_N], [9], 1, 1, "fout*fout", ["fout"], [], _N, "fout"),
    ],
}
NETWORKS = ["GCN", "GAT", "SGC", "GraphSAGE", "GIN", "DGN", "PNA"]


def _size(sym, env):
    v = 1
    for part in sym.split("*"):
        v *= env[part] if part in env else int(part)
    return v * 4


def gen_ops(network, layer, node_num, edge_num, feature, reorder=False, heads=16):
    """Op-graph records for one layer (what gen_yaml writes, genGraphOP.py:27-154)."""
    key = (network, bool(reorder))
    rows = TABLE.get(key, TABLE.get(network))
    if rows is None:
        raise ValueError(f"no such network {network}")
    env = {"fin": [0, feature, 128, 64, 16][layer], "fout": [0, 128, 64, 16][layer], "fh": heads}
    count = {_N: node_num, _E: edge_num}
    out = []
    for no, comp, kind, order, fnum, ins, g, nong, w, isz, outs, onum, osz in rows:
        out.append({
            "OP_NO": no, "COMP_TYPE": comp, "TYPE": kind, "ORDER": order,
            "INPUT": {"input_g_list": list(ins), "input_g_num": g, "input_nong_num": nong, "input_nong_list": [],
                      "input_size": [] if w is None else [_size(w, env)],
                      "feature_number": [count[f] for f in fnum],
                      "size_per_feature": [_size(s, env) for s in isz]},
            "OUTPUT": {"output_list": list(outs), "output_number": count[onum], "size_per_feature": _size(osz, env)},
        })
    return out


def gen_yaml(path, node_num, edge_num, size_per_feature, network, layer, isReorder, heads=16):
    """Same call and output as genGraphOP.gen_yaml (+ optional attention width `heads`)."""
    import os
    data = gen_ops(network, layer, node_num, edge_num, size_per_feature, isReorder, heads)
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, "w") as f:
        yaml.safe_dump(data, f)
    return path


def dumps(records):
    return yaml.safe_dump(records)
