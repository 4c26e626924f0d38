"""The op graphs' data flow, read twice and pinned to the reference.

ir.OpGraph (the product's reader) and oracle/opgraph_ref (the oracle's own reader) must give the
same producer edges for every golden op YAML, and both must match what the reference's lowering
wrote into the golden streams: interpret() turns an in-block input into a RAW dependency on the
producer's COMP (code/interpreter.py:399-402), a fused COMP pair names producer then consumer in
its ID (inst_fusion_x2, :575-636), and fuse_fetch re-points a removed FETCH's consumers at the
scatter's LOAD (:764-802).  The per-network input patches of semantics.py are the only departures
from the YAML, and they are listed here.
"""
import os

import pytest

from gta_graph_tensor_acclelrator_for_general_gnn_amd import ir
from gta_graph_tensor_acclelrator_for_general_gnn_amd.semantics import TABLE, Semantics
from oracle import opgraph_ref

from .conftest import load_manifest

M = load_manifest()
OPS = M["ops"]
STREAMS = [s for s in M["streams"] if "file" in s]

# the documented departures from the YAML (semantics.py): GAT-original op 10 reads op 8's
# per-destination sums (template/GAT_op.png, op 8's output_list) where genGraphOP.py:59 lists [7]
PATCHED = {("GAT", "original"): {10: [8]}}


def _key(rec):
    return rec["network"], "trans" if rec["reorder"] else "original"


@pytest.mark.parametrize("rec", OPS, ids=[r["file"][:-5] for r in OPS])
def test_product_and_oracle_readers_agree(golden_dir, rec):
    records = ir.read_yaml(os.path.join(golden_dir, "ops", rec["file"]))
    patches = Semantics.for_network(rec["network"], rec["reorder"]).inputs
    g = ir.OpGraph(records, patches)
    ref = opgraph_ref.producers(records, patches)
    for i in range(len(records)):
        assert g.producers(i) == ref[i], (rec["file"], i)
        kinds = [s.kind for s in g.inputs[i]]
        assert kinds == [k for k, _ in opgraph_ref.slots(records[i], i, patches.get(i))], (rec["file"], i)
    assert g.topo() == opgraph_ref.topo(records, patches)
    # the patches are the only difference from the YAML as written, and they are the listed ones
    plain = opgraph_ref.producers(records)
    diff = {i: ref[i] for i in ref if ref[i] != plain[i]}
    assert diff == PATCHED.get(_key(rec), {})


def test_patch_table_is_the_documented_one():
    assert {k: v["inputs"] for k, v in TABLE.items() if v.get("inputs")} == PATCHED


def _stream_evidence(blocks):
    """Per block: (ops in the block, [(producer ops, consumer ops)] the stream states).  A fused COMP
    pair names producer then consumer; a RAW of any instruction on another op's instruction in the
    same block says one of that instruction's ops feeds one of this instruction's (a fused COMP on
    either side holds several ops: the edge is one of their pairs; a scatter whose FETCH fuse_fetch
    removed has its STORE_E read the producer's COMP directly)."""
    out = []
    for blk in blocks:
        ops_in = {p[0] for inst in blk for p in ir.parse_id(inst["ID"])}
        stated = []
        for inst in blk:
            parts = [p[0] for p in ir.parse_id(inst["ID"])]
            for a, b in zip(parts, parts[1:]):
                stated.append(({a}, {b}))
            for d in inst["Dependency"]["RAW"]:
                src = {q[0] for q in ir.parse_id(d["ID"])} - set(parts)
                if src and src <= ops_in:
                    stated.append((src, set(parts)))
        out.append((ops_in, stated))
    return out


@pytest.mark.parametrize("rec", STREAMS, ids=[r["file"][:-5] for r in STREAMS])
def test_stream_dependencies_are_the_yaml_data_flow(golden_dir, rec):
    """Every producer edge the reference's stream states is an edge of the oracle's reading of the
    YAML, and every YAML edge inside a fused block is stated by the stream."""
    records = ir.read_yaml(os.path.join(golden_dir, "ops", rec["op_yaml"]))
    blocks = ir.read_yaml(os.path.join(golden_dir, "streams", rec["file"]))
    prod = opgraph_ref.producers(records)  # as written: the stream follows the YAML
    for ops_in, stated in _stream_evidence(blocks):
        for P, C in stated:
            assert any(p in prod[c] for p in P for c in C), (rec["file"], P, C)
        for c in ops_in:
            for p in prod[c]:
                if p in ops_in and p != c:
                    assert any(p in P and c in C for P, C in stated), (rec["file"], "edge not in the stream", p, c)
