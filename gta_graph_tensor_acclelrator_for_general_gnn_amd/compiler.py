"""Fusion + tiling search: op graph -> ranked (fusion partition, tile sizes, modelled DRAM bytes).

Behavioural restatement of the reference's compile() (code/compiler.py:475-510),
pinned against its candidate lists in tests/golden/manifest.json
(tests/test_compiler.py).  Together with lowering.lower() it makes the whole
upstream (op graph -> stream) available without the reference, so the executor
can run shapes the reference never lowered.

Search (reference line ranges):
  op-edge list, break points   gen_op_connected_info :451-468 (edges keyed by OP_NO,
                               so GAT's duplicate OP_NO 1 yields edge (1,5), not (2,5))
  every bitmask of fused edges generate_all_binaries :382-442 (masks touching a break
                               point skipped; cyclic partitions rejected, :349-371)
  mask -> blocks               trans_binary_to_fused_array :29-62 (connected components,
                               sorted by (size, members))
  block buffer need + bytes    cal_size :132-258; largest tile that fits the 2 MiB buffer
                               (x2 ping-pong) by binary search over the tile sizes :67-110
Candidates are returned sorted by modelled bytes (stable), as the reference does.
"""
import math

from . import ir

BUFFER_BYTES = 2 * 1024 * 1024  # code/compiler.py:479


def op_edges(ops):
    """(edge list keyed by OP_NO, op count, skip bit positions, break points)."""
    edges, brk = [], []
    for op in ops:
        a = op["OP_NO"]
        for b in op["OUTPUT"]["output_list"]:
            edges.append([a, b])
            src, dst = ops[a], ops[b]
            if (src["TYPE"] == "gather" and dst["TYPE"] == "scatter") or \
                    (src["ORDER"] != dst["ORDER"] and dst["TYPE"] == "scatter"):
                brk.append([a, b])
    skip = sorted(len(edges) - edges.index(p) for p in brk)
    return edges, len(ops), skip, brk


def blocks_of(edges, mask, n_ops):
    """Connected components of the ops joined by the '1' bits of mask."""
    adj = {i: [] for i in range(n_ops)}
    for bit, (u, v) in zip(mask, edges):
        if bit == "1":
            adj[u].append(v)
            adj[v].append(u)
    seen, comps = set(), []
    for s in range(n_ops):
        if s in seen:
            continue
        comp, todo = [], [s]
        while todo:
            u = todo.pop()
            if u in seen:
                continue
            seen.add(u)
            comp.append(u)
            todo.extend(w for w in adj[u] if w not in seen)
        comps.append(sorted(comp))
    return sorted(comps, key=lambda c: (len(c), c))


def pick_tile(pingpang, sizes, buffer_bytes, max_tiles, weight, edge_b, row_b, col_b, node_num):
    """Largest tile size (rows) whose buffer need fits; (-1, -1) if none."""
    k = 2 if pingpang else 1
    lo, hi = 0, len(sizes) - 1
    for i, s in enumerate(sizes):
        if s > node_num:
            hi = i
            break

    def need(j):
        return weight + (row_b * sizes[j] + col_b + edge_b * max_tiles[j]) * k
    while lo < hi:
        mid = (lo + hi + 1) // 2
        if need(mid) < buffer_bytes:
            lo = mid
        else:
            hi = mid - 1
    if need(lo) > buffer_bytes:
        return -1, -1
    return sizes[lo], 1


def block_cost(ops, block, menu, sizes, max_tiles, node_num, pingpang=True, sinput=False,
               buffer_bytes=BUFFER_BYTES):
    """(modelled DRAM bytes, row tile, col tile) of one fused block."""
    weight = inp = outp = special = 0
    edge_b = row_b = col_b = 0

    def add_buf(kind, order, amount):
        nonlocal edge_b, row_b, col_b
        if kind in ("scatter", "applynode"):
            if order == "R":
                row_b += amount
            else:
                col_b += amount
        else:
            edge_b += amount

    for i in block:
        op = ops[i]
        kind, order, comp = op["TYPE"], op["ORDER"], op["COMP_TYPE"]
        I, O = op["INPUT"], op["OUTPUT"]
        in_sz, out_sz = I["size_per_feature"], O["size_per_feature"]
        if I["input_nong_num"] != 0:
            weight += sum(I["input_size"])
        if kind == "gather":  # the accumulator's node read
            inp += O["output_number"] * out_sz
        sinput_skip = kind == "applynode" and comp == "MM" and sinput and op["OP_NO"] == 0
        srcs = I["input_g_list"]
        if not srcs:
            if sinput_skip:
                pass
            elif kind == "scatter" and order == "C":
                special += I["feature_number"][0] * in_sz[0]
            else:
                inp += I["feature_number"][0] * in_sz[0]
            add_buf(kind, order, in_sz[0])
        else:
            for s, src in enumerate(srcs):
                add_buf(kind, order, in_sz[s])
                if src not in block:
                    if sinput_skip:
                        pass
                    elif kind == "scatter" and order == "C":
                        special += I["feature_number"][s] * in_sz[s]
                    else:
                        inp += I["feature_number"][s] * in_sz[s]
                else:
                    prod = ops[src]
                    v = menu.get(((prod["TYPE"], kind), (prod["COMP_TYPE"], comp)))
                    if v and v[0]:  # fused pair: the intermediate never needs a buffer of its own
                        if v[1] == "Edge":
                            edge_b -= out_sz
                        elif order == "R":
                            row_b -= out_sz
                        else:
                            col_b -= out_sz
        # output buffer and stores
        if kind in ("scatter", "applyedge"):
            edge_b += out_sz
        elif order == "R":
            row_b += out_sz
        else:
            col_b += out_sz
        if not O["output_list"] or any(d not in block for d in O["output_list"]):
            outp += O["output_number"] * out_sz
    row, col = pick_tile(pingpang, sizes, buffer_bytes, max_tiles, weight, edge_b, row_b, col_b, node_num)
    rw = weight + inp + outp + special * math.ceil(node_num / row)
    return rw, row, col


def _returns_to(graph, block):
    """Does any path leaving the block come back into it (code/compiler.py:318-347)?"""
    members = set(block)

    def dfs(u, seen):
        if u in seen:
            return False
        if u in members:
            return True
        seen.add(u)
        for w in graph.get(u, []):
            if dfs(w, seen):
                return True
        seen.remove(u)
        return False

    for u in block:
        seen = set()
        for w in graph.get(u, []):
            if w not in members and dfs(w, seen):
                return True
    return False


def has_cycle(ops, blocks):
    graph = {}
    for op in ops:  # keyed by OP_NO: a duplicate OP_NO keeps the LAST op's outputs
        graph[op["OP_NO"]] = list(op["OUTPUT"]["output_list"])
    return any(_returns_to(graph, b) for b in blocks)


def search(ops, node_num, sizes, max_tiles, pingpang=True, sinput=False, menu=None, buffer_bytes=BUFFER_BYTES):
    """All feasible (blocks, tile sizes, bytes, mask) sorted by bytes -- compile()'s result list."""
    menu = menu or ir.INST_FUSED
    edges, n_ops, skip, brk = op_edges(ops)
    k = len(edges)
    out = []
    for number in range(1 << k):
        mask = bin(number)[2:].zfill(k) if k else ""
        if skip and any(mask[k - b] == "1" for b in skip):
            continue
        blocks = blocks_of(edges, mask, n_ops)
        total, tiles, ok = 0, [], True
        for blk in blocks:
            rw, row, col = block_cost(ops, blk, menu, sizes, max_tiles, node_num, pingpang, sinput, buffer_bytes)
            if row == -1:
                ok = False
                break
            total += rw
            tiles.append([row, col])
        if not ok:
            continue
        if brk:
            if any(a in blk and b in blk for blk in blocks for a, b in brk):
                continue
            if has_cycle(ops, blocks):
                continue
        out.append((blocks, tiles, total, mask))
    out.sort(key=lambda r: r[2])
    return out


def compile(dataset_name, network_name, layer_name, isReorder, isSinput, isPingpang, *, node_num, sizes, max_tiles,
            op_root="Network"):
    """Same result list as the reference compile()[0]; node_num / tile lists passed explicitly
    (the reference reads dataset/<ds>/maxlist_*, sizelist_* and hard-codes N per name)."""
    ops = ir.read_yaml(ir.op_yaml_path(network_name, dataset_name, layer_name, isReorder, op_root))
    return search(ops, node_num, sizes, max_tiles, isPingpang, isSinput)
