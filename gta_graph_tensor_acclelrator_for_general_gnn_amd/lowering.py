"""ISA lowering: op graph + fusion partition + tile sizes -> GTA instruction stream.

A behavioural restatement of the reference's `interpret()` (code/interpreter.py:805-849),
pinned byte-for-byte against the reference-emitted streams in tests/golden/streams
(tests/test_lowering.py).  The stream feeds executor.execute(), so shapes the
reference cannot lower (interpret() hard-codes N for four dataset names,
code/interpreter.py:807-815, e.g. ogbn-products) get their stream from here.

Stages (reference line ranges):
  per op   gen_inst           :313-479  loads / COMP (FETCH for scatter) / store + RAW/WAR records
  links    gen_link           :487-495  WAR successor index of every instruction
  pairs    gen_inst_fused_list:540-573  COMP->COMP pairs allowed by the Inst_fused menu
  fuse     update_inst        :737-756  inst_fusion_x2/x3 :575-715, rename via update_fused_dependency :717-734
  fetch    fuse_fetch         :764-802  drop FETCH, splice its RAW/WAR through
Quirks kept on purpose (they change the bytes): dependency records are shared
between a fused instruction and its parents and renamed in place by SUBSTRING
match of ID and TYPE; the load tile lookup receives the compute type where a
load type is expected (so LOAD_W tiles come from the later override); fused
instructions carry no Weight_Size; unsupported op pairs raise (TypeError) where
the reference raises.
"""
import math
import os

import yaml

from . import ir

UNIT_OF = {"ADD": "VEC_ALU", "SF": "SF_ALU", "MUL": "VEC_ALU", "LOAD": "Memory_Access_Unit",
           "LOAD_N": "Virtual_Loader", "STORE": "Memory_Access_Unit", "MM": "MM", "Fused": "MM"}


class _NoAlias(yaml.SafeDumper):
    def ignore_aliases(self, data):
        return True


def dump(stream_blocks):
    """YAML text exactly as the reference writes it (code/interpreter.py:33-47)."""
    return yaml.dump(stream_blocks, Dumper=_NoAlias)


# ------------------------------------------------------------------ records
def _record(typ, ident, unit, times, size, flen, weight=None):
    r = {"TYPE": typ, "ID": ident, "Hardware_Unit": unit, "Tile_Times": times, "Tile_Size": size,
         "Feature_Length": flen, "Dependency": {"RAW": [], "WAR": []}, "Enable": {"RAW": [], "WAR": []}}
    if weight is not None:
        r["Weight_Size"] = weight
    return r


def _ref(inst, times):
    return {"TYPE": inst["TYPE"], "ID": inst["ID"], "Times": times}


def _flip(t):
    return [t[1], t[0]]


def _feed(load, comp, times):
    """load -> COMP: `times` is stated from the load's side; the COMP holds it flipped."""
    load["Dependency"]["WAR"].append(_ref(comp, times))
    load["Enable"]["RAW"].append(_ref(comp, times))
    comp["Dependency"]["RAW"].append(_ref(load, _flip(times)))
    comp["Enable"]["WAR"].append(_ref(load, _flip(times)))


def _drain(comp, store, times):
    """COMP -> store: `times` is stated from the store's side; the COMP holds it flipped."""
    store["Dependency"]["RAW"].append(_ref(comp, times))
    store["Enable"]["WAR"].append(_ref(comp, times))
    comp["Dependency"]["WAR"].append(_ref(store, _flip(times)))
    comp["Enable"]["RAW"].append(_ref(store, _flip(times)))


class _Lower:
    def __init__(self, records, node_num, fused_menu=None):
        self.ops = records
        self.N = node_num
        self.menu = fused_menu or ir.INST_FUSED

    # ---- tile arithmetic (code/interpreter.py:55-129)
    @staticmethod
    def _load_tile(kind, order, TR, TC, SR, SC):
        if kind == "scatter":
            return (TR, SR) if order == "R" else (TR * TC, SC)
        if kind in ("gather", "applyedge"):
            return TR * TC, SR * SC
        if kind == "applynode":
            return (TR, SR) if order == "R" else (TC, SC)
        return -1, -1

    @staticmethod
    def _comp_tile(kind, order, TR, TC, SR, SC):
        if kind in ("scatter", "gather", "applyedge"):
            return TR * TC, SR * SC
        if kind == "applynode":
            return (TR, SR) if order == "R" else (TC, SC)
        return -1, -1

    @staticmethod
    def _store_tile(kind, order, TR, TC, SR, SC):
        if kind in ("scatter", "applyedge"):
            return TR * TC, SR * SC
        if kind in ("gather", "applynode"):
            return (TR, SR) if order == "R" else (TR * TC, SC)
        return -1, -1

    @staticmethod
    def _dep_times(kind, order, consumer_kind, TR, TC):
        """Tile-count ratio between a producer and an in-block consumer (code/interpreter.py:165-194)."""
        if kind == "scatter":
            if consumer_kind in ("gather", "applyedge"):
                return [1, 1]
            return None
        if kind == "gather":
            if consumer_kind == "applynode":
                return [TC, 1] if order == "R" else [TR, 1]
            return None
        if kind == "applyedge":
            if consumer_kind in ("gather", "applyedge"):
                return [1, 1]
            return None
        if kind == "applynode":
            if consumer_kind == "scatter":
                return [1, TC] if order == "R" else [1, TR]
            if consumer_kind == "applynode":
                return [1, 1]
            return None
        return [-1, -1]

    def _in_block_ref(self, other, kind, order, consumer_kind, TR, TC, SR, SC, reverse):
        t = self._dep_times(kind, order, consumer_kind, TR, TC)
        if t is None:
            raise TypeError("'NoneType' object is not subscriptable "
                            f"(no tile relation {kind}->{consumer_kind}, code/interpreter.py:165-194)")
        times = [t[1], t[0]] if reverse else [t[0], t[1]]
        return _ref(self._comp(other, TR, TC, SR, SC), times)

    # ---- instruction builders (code/interpreter.py:132-298)
    def _comp(self, i, TR, TC, SR, SC):
        op = self.ops[i]
        kind, ctype, order = op["TYPE"], op["COMP_TYPE"], op["ORDER"]
        tt, ts = self._comp_tile(kind, order, TR, TC, SR, SC)
        typ = "FETCH" if kind == "scatter" else "COMP_" + ctype
        return _record(typ, f"{i}_{kind}_0", UNIT_OF.get(ctype), tt, ts, op["INPUT"]["size_per_feature"][0], 0)

    def _load(self, i, slot, load_type, TR, TC, SR, SC):
        op = self.ops[i]
        kind, order = op["TYPE"], op["ORDER"]
        tt, ts = self._load_tile(kind, order, TR, TC, SR, SC)
        unit = UNIT_OF["LOAD"]
        g_num = op["INPUT"]["input_g_num"]
        if load_type == "LOAD_W":
            flen, ident, tt, ts = op["INPUT"]["input_size"][0], f"{i}_{kind}_{g_num}", 1, 1
        elif load_type == "LOAD_N" and kind == "gather":
            flen, ident = op["OUTPUT"]["size_per_feature"], f"{i}_{kind}_{g_num}"
            if order == "R":
                unit, tt = UNIT_OF["LOAD_N"], TR
            else:
                tt = TC
        else:
            flen, ident = op["INPUT"]["size_per_feature"][slot], f"{i}_{kind}_{slot}"
        return _record(load_type, ident, unit, tt, ts, flen)

    def _store(self, i, TR, TC, SR, SC):
        op = self.ops[i]
        kind, order = op["TYPE"], op["ORDER"]
        tt, ts = self._store_tile(kind, order, TR, TC, SR, SC)
        dt = "E" if kind in ("scatter", "applyedge") else "N"
        return _record("STORE_" + dt, f"{i}_{kind}_0", UNIT_OF["STORE"], tt, ts, op["OUTPUT"]["size_per_feature"])

    @staticmethod
    def _input_loads(kind, order, ctype, n_inputs, TR, TC):
        """(load types, times) for inputs read from memory (code/interpreter.py:364-421)."""
        if kind == "scatter":
            return ["LOAD_N"], ([1, TC] if order == "R" else [1, 1])
        if kind == "gather":
            return ["LOAD_E"], [1, 1]
        letter = "LOAD_" + kind[5].upper()
        if ctype == "MM":
            return [letter], [1, 1]
        return [letter] * n_inputs, [1, 1]

    def gen(self, i, block_ops, TR, TC, SR, SC):
        op = self.ops[i]
        kind, order, ctype = op["TYPE"], op["ORDER"], op["COMP_TYPE"]
        ins, g_num, outs = op["INPUT"]["input_g_list"], op["INPUT"]["input_g_num"], op["OUTPUT"]["output_list"]
        comp = self._comp(i, TR, TC, SR, SC)
        loads, store = [], None

        # operand the op brings itself: accumulator, weights, or missing graph inputs (:326-361)
        extra, times = None, None
        if kind == "gather":
            extra, times = "LOAD_N", ([1, TC] if order == "R" else [1, 1])
        elif ctype == "MM" and kind == "applyedge":
            extra, times = "LOAD_W", [1, TR * TC]
        elif ctype == "MM" and kind == "applynode":
            extra, times = "LOAD_W", ([1, TR] if order == "R" else [1, TC])
        elif kind == "applyedge" and len(ins) != g_num:
            extra, times = "LOAD_E", [1, 1]
        elif kind == "applynode" and len(ins) != g_num:
            extra, times = "LOAD_N", ([1, TR] if order == "R" else [1, TC])
        if extra:
            ld = self._load(i, g_num - 1, extra, TR, TC, SR, SC)
            loads.append(ld)
            if extra == "LOAD_W":
                comp["Weight_Size"] = ld["Feature_Length"]
            _feed(ld, comp, times)

        # graph inputs (:363-430)
        if not ins:
            types, times = self._input_loads(kind, order, ctype, len(ins), TR, TC)
            for slot, lt in enumerate(types):
                ld = self._load(i, slot, lt, TR, TC, SR, SC)
                loads.append(ld)
                _feed(ld, comp, times)
        else:
            for slot, src in enumerate(ins):
                if src in block_ops:
                    s = self.ops[src]
                    for lst in (comp["Dependency"]["RAW"], comp["Enable"]["WAR"]):
                        lst.append(self._in_block_ref(src, s["TYPE"], s["ORDER"], kind, TR, TC, SR, SC, True))
                else:
                    types, times = self._input_loads(kind, order, ctype, len(ins), TR, TC)
                    ld = self._load(i, slot, types[slot], TR, TC, SR, SC)
                    loads.append(ld)
                    _feed(ld, comp, times)

        # outputs (:432-477)
        st_times = [1, TC] if (kind == "gather" and order == "R") else [1, 1]
        if not outs:
            store = self._store(i, TR, TC, SR, SC)
            _drain(comp, store, st_times)
        else:
            for dst in outs:
                if dst in block_ops:
                    d = self.ops[dst]
                    for lst in (comp["Dependency"]["WAR"], comp["Enable"]["RAW"]):
                        lst.append(self._in_block_ref(dst, kind, order, d["TYPE"], TR, TC, SR, SC, False))
                elif store is None:
                    store = self._store(i, TR, TC, SR, SC)
                    _drain(comp, store, st_times)
        return loads, comp, store


# ---------------------------------------------------------------- stream passes
def _find(blocks, typ, ident):
    """Position of the first instruction with this TYPE/ID in ANY block (code/interpreter.py:481-485)."""
    for blk in blocks:
        for j, inst in enumerate(blk):
            if inst["TYPE"] == typ and inst["ID"] == ident:
                return j
    return None


def _successors(blocks):
    return [[[_find(blocks, d["TYPE"], d["ID"]) for d in inst["Dependency"]["WAR"]] for inst in blk]
            for blk in blocks]


def _is_comp(inst):
    return inst["TYPE"].split("_")[0] == "COMP"


def _second(s):
    parts = s.split("_")
    return parts[1] if len(parts) > 1 else None


def _pair_allowed(a, b, menu):
    if not (_is_comp(a) and _is_comp(b)):
        return False
    key = ((_second(a["ID"]), _second(b["ID"])), (_second(a["TYPE"]), _second(b["TYPE"])))
    v = menu.get(key)
    return bool(v and v[0])


def _fusion_groups(succ, blocks, menu):
    """COMP pairs (and would-be triples) per block, in scan order (code/interpreter.py:540-573)."""
    groups = []
    for b, blk in enumerate(blocks):
        links = succ[b]
        undecided = list(range(len(blk)))
        groups.append([])
        cur = 0
        while undecided:
            inst = blk[cur]
            if not _is_comp(inst) or len(links[cur]) != 1:
                undecided.remove(cur)
            else:
                nxt = links[cur][0]
                if _pair_allowed(inst, blk[nxt], menu):
                    groups[-1].append([cur, nxt])
                    undecided.remove(cur)
                    if len(links[nxt]) == 1:
                        third = links[nxt][0]
                        if _pair_allowed(blk[nxt], blk[third], menu):
                            groups[-1][-1].append(blk[third])  # the reference appends the record, not its index
                            undecided.remove(nxt)
                else:
                    undecided.remove(cur)
            cur += 1
    return groups


def _rename_refs(blk, fused):
    """update_fused_dependency (code/interpreter.py:717-734): substring match on ID and TYPE."""
    for inst in blk:
        for lst in (inst["Dependency"]["RAW"], inst["Dependency"]["WAR"], inst["Enable"]["RAW"], inst["Enable"]["WAR"]):
            for d in lst:
                if d["ID"] in fused["ID"] and d["TYPE"] in fused["TYPE"]:
                    d["ID"], d["TYPE"] = fused["ID"], fused["TYPE"]


def _fuse(blk, members):
    """inst_fusion_x2 / x3 (code/interpreter.py:575-715) for member indices in order."""
    insts = [blk[m] for m in members]
    raw = list(insts[0]["Dependency"]["RAW"])
    for prev, inst in zip(insts, insts[1:]):
        raw += [d for d in inst["Dependency"]["RAW"] if not (d["TYPE"] == prev["TYPE"] and d["ID"] == prev["ID"])]
    war = []
    for inst, nxt in zip(insts, insts[1:]):
        war += [d for d in inst["Dependency"]["WAR"] if not (d["TYPE"] == nxt["TYPE"] and d["ID"] == nxt["ID"])]
    war += list(insts[-1]["Dependency"]["WAR"])
    head = insts[0]
    fused = {"TYPE": "_".join(i["TYPE"] for i in insts), "ID": "_".join(i["ID"] for i in insts),
             "Hardware_Unit": UNIT_OF["Fused"], "Tile_Times": head["Tile_Times"], "Tile_Size": head["Tile_Size"],
             "Feature_Length": head["Feature_Length"],
             "Dependency": {"RAW": raw, "WAR": war}, "Enable": {"RAW": war, "WAR": raw}}
    _rename_refs(blk, fused)
    return fused


def _apply_fusion(blocks, groups):
    """update_inst (code/interpreter.py:737-756): build every fused record, then splice per block."""
    built = []
    for b, gs in enumerate(groups):
        built.append([])
        for g in gs:
            if len(g) not in (2, 3):
                continue
            built[-1].append(_fuse(blocks[b], g))  # a triple holds a record -> TypeError, as in the reference
    for b, blk in enumerate(blocks):
        if not built[b]:
            continue
        for j in range(len(groups[b]) - 1, -1, -1):
            for k in sorted(groups[b][j], reverse=True):
                del blk[k]
            blk.append(built[b][j])


def _index_of(inst, refs):
    for k, d in enumerate(refs):
        if inst["ID"] == d["ID"] and inst["TYPE"] == d["TYPE"]:
            return k
    return None


def _drop_fetch(blocks):
    """fuse_fetch (code/interpreter.py:764-802): route around every FETCH, then delete it."""
    gone = []
    for b, blk in enumerate(blocks):
        for j, inst in enumerate(blk):
            if inst["TYPE"] != "FETCH":
                continue
            gone.append((b, j))
            f_raw, f_war, fid = inst["Dependency"]["RAW"], inst["Dependency"]["WAR"], inst["ID"]
            for other in blk:
                for k, d in enumerate(other["Dependency"]["RAW"]):
                    twin = other["Enable"]["WAR"][k]
                    if d["ID"] == fid and d["TYPE"] == "FETCH":
                        src = f_raw[_index_of(other, f_war)]
                        for rec in (d, twin):
                            rec["ID"], rec["TYPE"], rec["Times"] = src["ID"], src["TYPE"], src["Times"]
                for k, d in enumerate(other["Dependency"]["WAR"]):
                    twin = other["Enable"]["RAW"][k]
                    if d["ID"] == fid and d["TYPE"] == "FETCH":
                        dst = f_war[_index_of(other, f_raw)]
                        for rec in (d, twin):
                            rec["ID"], rec["TYPE"] = dst["ID"], dst["TYPE"]
    for b, j in sorted(gone, reverse=True):
        del blocks[b][j]


def lower(op_records, node_num, op_array, tile_size_list, fused_menu=None):
    """Instruction stream (list of blocks of records) for a fusion partition and its tiles."""
    L = _Lower(op_records, node_num, fused_menu)
    blocks = []
    for ops_b, (SR, SC) in zip(op_array, tile_size_list):
        TR, TC = math.ceil(node_num / SR), math.ceil(node_num / SC)
        blk = []
        for i in ops_b:
            loads, comp, store = L.gen(i, ops_b, TR, TC, SR, SC)
            blk.extend(loads)
            blk.append(comp)
            if store is not None:
                blk.append(store)
        blocks.append(blk)
    succ = _successors(blocks)
    groups = _fusion_groups(succ, blocks, L.menu)
    _apply_fusion(blocks, groups)
    _drop_fetch(blocks)
    return blocks


DATASET_NODES = {"cora": 2708, "pubmed": 19717, "flickr": 89250, "reddit": 232965}


def interpret(data_set, network, isReorder, layer, op_array, tile_size_list, node_num=None,
              op_root="Network", out_root="Results/Insts"):
    """Same call and files as the reference interpret(); node_num may be given for other graphs."""
    n = node_num if node_num is not None else DATASET_NODES.get(data_set, 0)
    path = ir.op_yaml_path(network, data_set, layer, isReorder, op_root)
    records = ir.read_yaml(path)
    blocks = lower(records, n, op_array, tile_size_list)
    out = ir.inst_path(network, data_set, layer, isReorder, out_root)
    os.makedirs(os.path.dirname(out), exist_ok=True)
    with open(out, "w") as f:
        f.write(dump(blocks))
    return out
