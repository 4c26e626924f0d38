"""Numeric semantics the op YAML leaves open, per network (the build's written choices).

The reference never computes values, so three things are not fixed by its files:
  * which special function an SF op is (COMP_TYPE "SF", unit SF_ALU, code/interpreter.py:7);
  * GAT op 9 is typed MUL in genGraphOP.py:58 but drawn as "/" in
    template/GAT_op.png (alpha = exp / sum exp); GAT-trans op 11 divides the
    aggregated numerator (op 10) by the aggregated denominator (op 9);
  * a few YAML data-flow quirks: GAT-original op 10 lists input [7]
    (genGraphOP.py:59) while GAT_op.png and op 8's output_list route the
    per-destination sums (op 8) into it.
Everything else follows the YAML literally (ADD/MUL element-wise with head
broadcast of the narrower operand, MM = x . W, scatter/gather per ORDER).
"""

DEFAULT = {"sf": {}, "bin": {}, "inputs": {}}

TABLE = {
    ("GAT", "original"): {"sf": {7: "EXP_LEAKY_RELU", 13: "ELU"}, "bin": {9: "DIV"}, "inputs": {10: [8]}},
    ("GAT", "trans"): {"sf": {8: "EXP_LEAKY_RELU", 12: "ELU"}, "bin": {11: "RDIV"}},
    ("GCN", "original"): {},
    ("GCN", "trans"): {},
    ("SGC", "original"): {},
    ("SGC", "trans"): {},
    ("GraphSAGE", "original"): {"sf": {6: "RELU"}},
    ("GraphSAGE", "trans"): {"sf": {6: "RELU"}},
    ("GIN", "original"): {"sf": {6: "RELU", 8: "RELU"}},
    ("GIN", "trans"): {"sf": {6: "RELU", 8: "RELU"}},
    ("DGN", "original"): {"sf": {10: "RELU"}},
    ("DGN", "trans"): {"sf": {10: "RELU"}},
    ("PNA", "original"): {"sf": {7: "RELU"}},
    ("PNA", "trans"): {"sf": {7: "RELU"}},
}


class Semantics:
    def __init__(self, sf=None, bin=None, inputs=None, default_sf="RELU"):
        self.sf = dict(sf or {})
        self.bin = dict(bin or {})
        self.inputs = dict(inputs or {})
        self.default_sf = default_sf

    @classmethod
    def for_network(cls, network, reorder=False):
        t = TABLE.get((network, "trans" if reorder else "original"), {})
        return cls(t.get("sf"), t.get("bin"), t.get("inputs"))

    def sf_of(self, op):
        return self.sf.get(op.idx, self.default_sf)

    def bin_of(self, op):
        """ADD / MUL / DIV / RDIV (b / a) for a binary element-wise op."""
        return self.bin.get(op.idx, op.comp)
