"""Data flow of a GTA op-graph YAML, read without the product's ir.OpGraph (TEST ORACLE ONLY, see
oracle/__init__.py).

exec_ref evaluates an op graph with the slots this module resolves, so a misreading of
input_g_list in the product (ir.OpGraph._resolve) cannot hide in the oracle too; and
tests/test_dataflow.py pins both readers to the producer edges the reference's own lowering wrote
into the 157+ golden streams.

How the reference reads an op's inputs (code/interpreter.py:313-430, gen_inst):
  * input_g_list entries are POSITIONS in the YAML list (op_info[current_input_op], :401), not OP_NO
    (GAT position 2 carries OP_NO 1, genGraphOP.py:51);
  * an entry naming another op is a producer: a RAW on its COMP when both sit in one fused block
    (:399-402), else a LOAD of the stored value (:403-430);
  * an empty list means the op reads the model input (the LOADs of :364-393);
  * entry -1, or a slot beyond the list up to input_g_num, is an input from outside the graph (the
    "outside" LOAD_E / LOAD_N of :344-352: GCN/SAGE/GIN op 1's edge weight, GIN op 3's eps);
  * an op naming itself (PNA-trans ops 0/1, genGraphOP.py:137-138) reads the model input;
  * scatter, gather and MM / SF ops take one graph operand (their COMPUTE rules,
    template/ISA_defination.yaml:1-61); MM's second operand is the LOAD_W weight.
The per-network patches (semantics.py: GAT-original op 10 reads op 8's sums, GAT_op.png) are given
by the caller, as the only documented departures from the YAML.
"""


def slots(rec, idx, patch=None):
    """[("op", j) | ("x", s) | ("ext", s)] for the op at position idx (rec: its YAML record)."""
    inp = rec["INPUT"]
    lst = list(patch if patch is not None else (inp.get("input_g_list") or []))
    num = int(inp.get("input_g_num") or 0)
    out = []
    for s in range(max(num, len(lst), 1)):
        if s < len(lst):
            j = int(lst[s])
            out.append(("ext", s) if j == -1 else (("x", s) if j == idx else ("op", j)))
        elif not lst and s == 0:
            out.append(("x", s))
        else:
            out.append(("ext", s))
    single = rec["TYPE"] in ("scatter", "gather") or rec.get("COMP_TYPE", "NONE") in ("MM", "SF")
    return out[:1] if single else out


def dataflow(records, patches=None):
    """{position: slots} for every op of the YAML list."""
    patches = patches or {}
    return {i: slots(r, i, patches.get(i)) for i, r in enumerate(records)}


def producers(records, patches=None):
    """{position: [producer positions, slot order]}."""
    return {i: [j for k, j in ss if k == "op"] for i, ss in dataflow(records, patches).items()}


def topo(records, patches=None):
    """Positions in data-flow order (Kahn, lowest position first); raises on a cycle."""
    prod = producers(records, patches)
    left = {i: len(p) for i, p in prod.items()}
    order, ready = [], sorted(i for i, c in left.items() if c == 0)
    while ready:
        i = ready.pop(0)
        order.append(i)
        for k, p in prod.items():
            if i in p:
                left[k] -= p.count(i)
                if left[k] == 0:
                    ready.append(k)
                    ready.sort()
    if len(order) != len(records):
        raise ValueError("op graph has a cycle")
    return order
