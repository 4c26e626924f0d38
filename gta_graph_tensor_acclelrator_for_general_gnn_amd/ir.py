"""GTA IR: op-graph YAML, instruction-stream YAML and the fused-instruction menu.

Formats (reference):
  op graph   -- list of op records {OP_NO, COMP_TYPE, TYPE, ORDER, INPUT{input_g_list,
                input_g_num, input_nong_num, input_nong_list, input_size, feature_number,
                size_per_feature}, OUTPUT{output_list, output_number, size_per_feature}}
                (vTCAD/GraphOP/genGraphOP.py:4-25; template/op_template.yaml:1-19).
                Ops are addressed by POSITION in the list (interpreter op_info[op_id],
                code/interpreter.py:134), not by OP_NO (GAT index 2 carries OP_NO 1,
                genGraphOP.py:51).
  stream     -- list of fused blocks, each a list of instruction records {TYPE, ID,
                Hardware_Unit, Tile_Times, Tile_Size, Feature_Length, [Weight_Size],
                Dependency{RAW,WAR}, Enable{RAW,WAR}} (code/interpreter.py:145-161,
                244-259, 281-296, 617-632); fused COMPs have TYPE 'COMP_A_COMP_B' and ID
                '<op>_<type>_<k>_<op>_<type>_<k>' (:608-609).
  fused menu -- hardware_info.yaml Inst_fused ("FinalVersion For Paper/hardware_info.yaml":11-68).
Sizes in the op YAML are bytes of fp32 features (genGraphOP multiplies by 4).
"""
import re

import yaml

# hardware_info.yaml Inst_fused, restated: (pattern, compute types) -> (Is_Fused, Buffer_Type)
INST_FUSED = {
    (("scatter", "gather"), ("NONE", "ADD")): (True, "Edge"),
    (("gather", "scatter"), ("ADD", "NONE")): (False, "Node"),
    (("scatter", "applyedge"), ("NONE", "MM")): (True, "Edge"),
    (("scatter", "applyedge"), ("NONE", "ADD")): (True, "Edge"),
    (("applyedge", "gather"), ("MM", "ADD")): (True, "Edge"),
    (("applyedge", "gather"), ("MUL", "ADD")): (True, "Edge"),
    (("applyedge", "gather"), ("ELE", "ELE")): (False, "Edge"),
    (("applyedge", "applyedge"), ("MM", "MM")): (False, "Edge"),
    (("applyedge", "applyedge"), ("MM", "ELE")): (False, "Edge"),
    (("applyedge", "applyedge"), ("ELE", "ELE")): (False, "Edge"),
    (("applynode", "applynode"), ("MM", "MM")): (False, "Node"),
    (("applynode", "applynode"), ("MM", "ELE")): (False, "Node"),
    (("applynode", "applynode"), ("ELE", "ELE")): (False, "Node"),
}


def is_fused(pattern, comp_types):
    v = INST_FUSED.get((tuple(pattern), tuple(comp_types)))
    return bool(v and v[0])


def read_yaml(path):
    with open(path) as f:
        return yaml.safe_load(f)


class Op:
    __slots__ = ("idx", "op_no", "type", "comp", "order", "in_list", "in_num", "in_sizes", "w_sizes",
                 "nong_num", "out_list", "out_size", "out_number", "feature_number")

    def __init__(self, idx, rec):
        self.idx = idx
        self.op_no = rec["OP_NO"]
        self.type = rec["TYPE"]
        self.comp = rec.get("COMP_TYPE", "NONE")
        self.order = rec.get("ORDER", "R")
        inp, out = rec["INPUT"], rec["OUTPUT"]
        self.in_list = list(inp.get("input_g_list") or [])
        self.in_num = int(inp.get("input_g_num") or 0)
        self.in_sizes = list(inp.get("size_per_feature") or [])
        self.w_sizes = list(inp.get("input_size") or [])
        self.nong_num = int(inp.get("input_nong_num") or 0)
        self.feature_number = list(inp.get("feature_number") or [])
        self.out_list = list(out.get("output_list") or [])
        self.out_size = int(out.get("size_per_feature") or 0)
        self.out_number = int(out.get("output_number") or 0)

    @property
    def out_width(self):
        return self.out_size // 4

    def in_width(self, slot):
        return self.in_sizes[slot] // 4 if slot < len(self.in_sizes) else None

    def __repr__(self):
        return f"Op({self.idx}:{self.type}/{self.comp}/{self.order} in={self.in_list} out={self.out_list})"


class Source:
    """Where an op input slot comes from: another op, the model input x, or an external tensor."""
    __slots__ = ("kind", "op", "slot")

    def __init__(self, kind, op=None, slot=None):
        self.kind, self.op, self.slot = kind, op, slot

    def __repr__(self):
        return {"op": f"op{self.op}", "x": "x", "ext": f"ext{self.slot}"}[self.kind]


class OpGraph:
    """Op graph with resolved data flow.

    Resolution rules (the reference YAML's inputs are authoritative, as in
    interpret()'s loads and RAW deps, code/interpreter.py:394-430):
      * input_g_list entry j >= 0, j != self -> output of op j
      * entry -1 -> external tensor for that slot ("ext:<op>:<slot>")
      * empty input_g_list, or an op naming itself (PNA trans op 0/1,
        genGraphOP.py:137-138) -> the model input x
      * slots beyond len(input_g_list) up to input_g_num -> external
      * `patches` (from the network semantics table) override slots.
    """

    def __init__(self, records, patches=None):
        self.records = records  # the YAML list as read (the oracle resolves its own data flow from it)
        self.ops = [Op(i, r) for i, r in enumerate(records)]
        self.patches = dict(patches or {})
        self.inputs = [self._resolve(op) for op in self.ops]

    @classmethod
    def load(cls, path, patches=None):
        return cls(read_yaml(path), patches)

    def __len__(self):
        return len(self.ops)

    def _resolve(self, op):
        lst = self.patches.get(op.idx, op.in_list)
        n = max(op.in_num, len(lst), 1)
        srcs = []
        for s in range(n):
            if s < len(lst):
                j = lst[s]
                if j == -1:
                    srcs.append(Source("ext", slot=s))
                elif j == op.idx:
                    srcs.append(Source("x", slot=s))
                else:
                    srcs.append(Source("op", op=j, slot=s))
            elif not lst:
                srcs.append(Source("x", slot=s) if s == 0 else Source("ext", slot=s))
            else:
                srcs.append(Source("ext", slot=s))
        if op.type in ("scatter", "gather") or (op.comp in ("MM", "SF")):
            srcs = srcs[:1]
        return srcs

    def producers(self, i):
        return [s.op for s in self.inputs[i] if s.kind == "op"]

    def topo(self, subset=None):
        """Topological order of `subset` (default all ops), ties by op index."""
        subset = sorted(range(len(self.ops)) if subset is None else subset)
        sset = set(subset)
        indeg = {i: sum(1 for p in self.producers(i) if p in sset) for i in subset}
        ready = [i for i in subset if indeg[i] == 0]
        out = []
        while ready:
            ready.sort()
            i = ready.pop(0)
            out.append(i)
            for j in subset:
                if i in self.producers(j):
                    indeg[j] -= self.producers(j).count(i)
                    if indeg[j] == 0:
                        ready.append(j)
        if len(out) != len(subset):
            raise ValueError(f"op graph has a cycle among {subset}")
        return out


_TRIPLE = re.compile(r"(\d+)_(scatter|gather|applyedge|applynode)_(\d+)")


def parse_id(inst_id):
    """'3_scatter_0' -> [(3,'scatter',0)]; fused '11_applyedge_0_12_gather_0' -> two triples."""
    return [(int(a), b, int(c)) for a, b, c in _TRIPLE.findall(inst_id)]


class Inst:
    __slots__ = ("type", "id", "unit", "tile_times", "tile_size", "feature_length", "weight_size", "raw", "war",
                 "parts", "rec")

    def __init__(self, rec):
        self.rec = rec
        self.type = rec["TYPE"]
        self.id = rec["ID"]
        self.unit = rec.get("Hardware_Unit")
        self.tile_times = rec.get("Tile_Times")
        self.tile_size = rec.get("Tile_Size")
        self.feature_length = rec.get("Feature_Length")
        self.weight_size = rec.get("Weight_Size")
        dep = rec.get("Dependency") or {}
        self.raw = [(d["TYPE"], d["ID"], list(d["Times"])) for d in dep.get("RAW") or []]
        self.war = [(d["TYPE"], d["ID"], list(d["Times"])) for d in dep.get("WAR") or []]
        self.parts = parse_id(self.id)

    @property
    def kind(self):
        t = self.type
        if t.startswith("LOAD"):
            return "load"
        if t.startswith("STORE"):
            return "store"
        if t == "FETCH":
            return "fetch"
        return "comp"

    @property
    def comp_types(self):
        """'COMP_MUL_COMP_ADD' -> ['MUL', 'ADD']."""
        return re.findall(r"COMP_([A-Z]+)", self.type)

    def __repr__(self):
        return f"{self.type}:{self.id}"


class Block:
    def __init__(self, index, recs):
        self.index = index
        self.insts = [Inst(r) for r in recs]
        ops = set()
        for ins in self.insts:
            for op, _, _ in ins.parts:
                ops.add(op)
        self.ops = sorted(ops)
        self.stored = sorted({ins.parts[0][0] for ins in self.insts if ins.kind == "store"})
        self.fused = []  # [(producer op, consumer op, [ctype, ctype])]
        for ins in self.insts:
            if ins.kind == "comp" and len(ins.parts) >= 2:
                ct = ins.comp_types
                for k in range(len(ins.parts) - 1):
                    self.fused.append((ins.parts[k][0], ins.parts[k + 1][0], ct[k:k + 2]))
        # tile sizes: an R-ordered op's LOAD_N/STORE_N/COMP Tile_Size is SR
        self.tile_size = None
        for ins in self.insts:
            if ins.kind == "comp" and ins.tile_size:
                self.tile_size = ins.tile_size
                break

    def __repr__(self):
        return f"Block{self.index}(ops={self.ops}, fused={self.fused})"


class Stream:
    def __init__(self, blocks):
        self.blocks = [Block(i, b) for i, b in enumerate(blocks)]

    @classmethod
    def load(cls, path):
        return cls(read_yaml(path))

    def __iter__(self):
        return iter(self.blocks)

    def __len__(self):
        return len(self.blocks)


def op_yaml_path(network, dataset, layer, reorder, root="Network"):
    """interpreter.py:817-821 path convention."""
    m = "trans" if reorder else "original"
    return f"{root}/{network}/{network}-{dataset}/{network}-{m}/{network}-{layer}-{m}.yaml"


def inst_path(network, dataset, layer, reorder, root="Results/Insts"):
    """simulator.py:398 / interpreter.py:823 path convention."""
    m = "trans" if reorder else "original"
    return f"{root}/{network}-{dataset}-{layer}-{m}.yaml"
