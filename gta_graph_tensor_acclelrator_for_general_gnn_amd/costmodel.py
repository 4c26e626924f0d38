"""The reference's modelled (cycles, rw) for a stream -- restated, exact, and fast.

The reference's only "result" of executing a stream is simulate()'s pair
(modelled cycles, modelled DRAM bytes) (code/simulator.py:370-502).  This
module reproduces both numbers exactly so the executor can report them next to
the measured run (ExecResult.model_cycles / model_rw).  It is pinned against the
reference's simulate() outputs in tests/golden/manifest.json (tests/test_costmodel.py).

Semantics restated from code/simulator.py:
  * units Memory_Access_Unit, VEC_ALU, SF_ALU, MM, Virtual_Loader, one instruction each (:51-58, :206-249)
  * every instruction runs Tile_Times iterations; an iteration may start when
    its RAW/WAR credits suffice and its unit is idle; credits: WAR edges start at
    2*Times[0]*Times[1], starting consumes Times[1] per edge, finishing grants
    Times[1] to the other side (:171-233)
  * one modelled cycle per loop iteration, instructions visited in order; an
    iteration that started this cycle is not decremented this cycle; it finishes
    when its counter reaches 0 or -1 (:430-488)
  * iteration cost (:272-327): LOAD_E/STORE_E ceil(nnz(tile)*FL/BW);
    LOAD_W/LOAD_N/STORE_N ceil(Tile_Size*FL/BW) with a tail tile for the last
    LOAD_N/STORE_N iteration; COMP_MM ceil(FL/16)*ceil((W/FL)/8); edge COMPs
    ceil(nnz/8)*ceil(FL/16); node COMPs ceil(TS/8)*ceil(FL/16); BW = 128 GiB/s
    at 1 GHz = 137.438953472 B/cycle.
The cycle loop here skips runs of cycles in which nothing can start or finish
(state is then invariant, so every skipped cycle is a no-op in the reference);
the result is identical, and a Cora layer takes ~1 s instead of ~20 s.
tile nnz data = calculate_sparsity(SR, 1) of the graph flattened row-major (:425-426),
from ops.tile_nnz (GPU) or a CPU restatement.

Per instruction (per_instruction): the bytes every instruction appends to simulate()'s rw_record
(:282-309; aggregated per TYPE by aggregate_rw_record, :107-125) and the unit-busy cycles of its
iterations (the durations update_timeline records, :329-330), in closed form over the tile-nnz
array with NumPy -- no cycle loop, so it runs at Reddit scale (the metric block's 106 M-iteration
instructions) in seconds.  The cycle loop (simulate_stream(..., record=True)) adds each
instruction's first start and last end; timeline_info restates aggregate_timeline (:127-146).
"""
import math

import numpy as np

BW = 128 * (1024 ** 3) * (10 ** (-9))
UNITS = ["Memory_Access_Unit", "VEC_ALU", "SF_ALU", "MM", "Virtual_Loader"]
PERF = {"VEC_ALU": (8, 16), "SF_ALU": (8, 16), "MM": (8, 16)}


def _find(blocks, typ, ident):
    for blk in blocks:
        for j, inst in enumerate(blk):
            if inst["TYPE"] == typ and inst["ID"] == ident:
                return j
    raise KeyError(f"dependency on missing instruction {typ} {ident}")


class _Sim:
    def __init__(self, node_num, tiles_for, sinput=False, sparsity=1.0, record=False):
        self.N = node_num
        self.tiles_for = tiles_for  # SR -> flat list of tile nnz (row-major [ceil(N/SR)][N])
        self.sinput = sinput
        self.sparsity = sparsity
        self.rw = 0
        self.spans = {} if record else None  # (block, index) -> [first start, its cost, last end]

    def cost(self, inst, remain, data):
        t = inst["TYPE"]
        fl = inst["Feature_Length"]
        if t in ("LOAD_E", "STORE_E"):
            size = data[len(data) - remain] * fl
            self.rw += size
            return math.ceil(size / BW)
        if t in ("LOAD_W", "LOAD_N", "STORE_N"):
            if t == "LOAD_N" and "0_applynode" in inst["ID"] and self.sinput:
                if any(d["TYPE"] == "COMP_MM" and d["ID"].split("_")[0] == inst["ID"].split("_")[0]
                       for d in inst["Dependency"]["WAR"]):
                    v = math.ceil(inst["Tile_Size"] * fl * self.sparsity)
                    self.rw += v
                    return math.ceil(inst["Tile_Size"] * fl * self.sparsity / BW)
            ts = inst["Tile_Size"]
            if t in ("LOAD_N", "STORE_N") and remain == 1:
                block = self.N - math.floor(self.N / ts) * ts
                size = (block if block else ts) * fl
            else:
                size = ts * fl
            self.rw += math.ceil(size)
            return math.ceil(size / BW)
        perf = PERF[inst["Hardware_Unit"]]
        if t == "COMP_MM":
            if "0_applynode" in inst["ID"] and self.sinput:
                return math.ceil(inst["Tile_Size"] * self.sparsity / PERF["VEC_ALU"][0]) * math.ceil(fl / PERF["VEC_ALU"][1])
            return math.ceil(math.ceil(fl / perf[1]) * math.ceil((inst["Weight_Size"] / fl) / perf[0]))
        if "applyedge" in inst["ID"] or "gather" in inst["ID"]:
            return math.ceil(data[len(data) - remain] / perf[0]) * math.ceil(fl / perf[1])
        return math.ceil(inst["Tile_Size"] / perf[0]) * math.ceil(fl / perf[1])

    def run(self, blocks, tile_sizes):
        prev = [[[_find(blocks, d["TYPE"], d["ID"]) for d in inst["Dependency"]["RAW"]] for inst in blk]
                for blk in blocks]
        nxt = [[[_find(blocks, d["TYPE"], d["ID"]) for d in inst["Dependency"]["WAR"]] for inst in blk]
               for blk in blocks]
        unit_busy = [False] * len(UNITS)
        cycle = 0
        data = None
        for b, blk in enumerate(blocks):
            if b == 0 or tile_sizes[b][0] != tile_sizes[b - 1][0]:
                data = self.tiles_for(tile_sizes[b][0])
                if isinstance(data, TileCounts):
                    data = data.dense()
                if isinstance(data, np.ndarray):
                    data = data.tolist()
            n = len(blk)
            credit = [[0] * n for _ in range(n)]
            for j, inst in enumerate(blk):
                for k, d in enumerate(inst["Dependency"]["WAR"]):
                    credit[j][nxt[b][j][k]] = 2 * d["Times"][0] * d["Times"][1]
            raw_need = [[d["Times"][1] for d in inst["Dependency"]["RAW"]] for inst in blk]
            war_need = [[d["Times"][1] for d in inst["Dependency"]["WAR"]] for inst in blk]
            unit_of = [UNITS.index(inst["Hardware_Unit"]) for inst in blk]
            state = [0] * n  # 0 waiting, 1 running, 2 finished
            remain_times = [inst["Tile_Times"] for inst in blk]
            remain_cycle = [0] * n
            P, Q = prev[b], nxt[b]
            while True:
                busy_change = False
                unfinished = False
                for j in range(n):
                    st = state[j]
                    if st == 0:
                        unfinished = True
                        if unit_busy[unit_of[j]]:
                            continue
                        row = credit[j]
                        if any(row[P[j][i]] < raw_need[j][i] for i in range(len(P[j]))):
                            continue
                        if any(row[Q[j][i]] < war_need[j][i] for i in range(len(Q[j]))):
                            continue
                        for i in range(len(Q[j])):
                            row[Q[j][i]] -= war_need[j][i]
                        for i in range(len(P[j])):
                            row[P[j][i]] -= raw_need[j][i]
                        unit_busy[unit_of[j]] = True
                        state[j] = 1
                        remain_cycle[j] = self.cost(blk[j], remain_times[j], data)
                        if self.spans is not None:
                            sp = self.spans.setdefault((b, j), [cycle, remain_cycle[j], 0])
                            sp[2] = cycle + remain_cycle[j]
                        busy_change = True
                    elif st == 1:
                        unfinished = True
                        remain_cycle[j] -= 1
                        if remain_cycle[j] == 0 or remain_cycle[j] == -1:
                            for i in range(len(Q[j])):
                                credit[Q[j][i]][j] += war_need[j][i]
                            for i in range(len(P[j])):
                                credit[P[j][i]][j] += raw_need[j][i]
                            unit_busy[unit_of[j]] = False
                            remain_times[j] -= 1
                            state[j] = 2 if remain_times[j] == 0 else 0
                            busy_change = True
                if not unfinished:  # block done; the reference counts the switch cycle except after the last
                    if b + 1 < len(blocks):
                        cycle += 1
                    break
                cycle += 1
                if not busy_change:
                    running = [max(remain_cycle[j], 1) for j in range(n) if state[j] == 1]
                    if not running:
                        raise RuntimeError(f"cost model deadlock in block {b} at cycle {cycle}")
                    skip = min(running) - 1
                    if skip > 0:
                        for j in range(n):
                            if state[j] == 1:
                                remain_cycle[j] -= skip
                        cycle += skip
        return cycle - 1, self.rw


def simulate_stream(blocks, tile_size_list, node_num, tiles_for, sinput=False, sparsity=1.0, record=False):
    """(cycles, rw) exactly as code/simulator.py:370-502 computes them for this stream.  record=True:
    (cycles, rw, spans) with spans[(block, index)] = [first start cycle, that iteration's cost, last
    end cycle] per instruction -- the first and last entries update_timeline (:329-330) records."""
    sim = _Sim(node_num, tiles_for, sinput, sparsity, record)
    cycles, rw = sim.run(blocks, tile_size_list)
    return (cycles, rw, sim.spans) if record else (cycles, rw)


def model_rw(blocks, node_num, edges_in_tiles):
    """Closed form of simulate()'s rw (timing-free): every LOAD_E/STORE_E sweeps all tiles once
    (sum nnz = edges_in_tiles), node/weight loads move Tile_Size*FL per iteration with a tail."""
    rw = 0
    for blk in blocks:
        for inst in blk:
            t, fl, tt, ts = inst["TYPE"], inst.get("Feature_Length"), inst.get("Tile_Times"), inst.get("Tile_Size")
            if t in ("LOAD_E", "STORE_E"):
                rw += edges_in_tiles * fl
            elif t in ("LOAD_N", "STORE_N"):
                block = node_num - math.floor(node_num / ts) * ts
                rw += (tt - 1) * math.ceil(ts * fl) + math.ceil((block if block else ts) * fl)
            elif t == "LOAD_W":
                rw += tt * math.ceil(ts * fl)
    return rw


class TileCounts:
    """calculate_sparsity(T, 1)'s flat [ceil(N/T) * n_cols] list without its zeros: the nonzero
    tile counts (any order), the list's length and its first entry (tile (0, 0)) -- all the
    per-instruction model needs when an instruction sweeps every tile (Tile_Times == length, which
    interpret()'s TR*TC is), at the size of the edge list rather than the tile grid (ogbn-products'
    dense grid at T = 512 would hold 1.2e10 entries).  dense() rebuilds the list (small graphs)."""
    __slots__ = ("length", "values", "first", "_dense")

    def __init__(self, length, values, first, dense=None):
        self.length, self.values, self.first, self._dense = int(length), np.asarray(values, np.int64), int(first), dense

    def __len__(self):
        return self.length

    def dense(self):
        if self._dense is None:
            raise ValueError("TileCounts: no dense form available")
        return np.asarray(self._dense(), dtype=np.int64)


def _first(data, tt):
    """data[len(data) - tt]: the tile of an instruction's first iteration."""
    if isinstance(data, TileCounts):
        if tt == data.length:
            return data.first
        data = data.dense()
    return int(_data_slice(data, tt)[0])


def _data_slice(data, tt):
    """data[len(data) - remain] for remain = tt .. 1 (the iteration order of :282 and :324), as an
    array; Python's negative-index wrap for remain > len(data) kept."""
    n = len(data)
    if tt <= n:
        return data[n - tt:]
    idx = n - np.arange(tt, 0, -1, dtype=np.int64)
    return data[np.where(idx < 0, idx + n, idx)]


def _edge_sums(cache, data, tt, fl):
    """(sum nnz, sum ceil(nnz/8), sum ceil(nnz*fl/BW)) over the instruction's iterations, cached per
    (tt, fl): the metric block's three edge instructions share one 106 M-entry pass each.  The entry
    holds `data` itself, so the id in its key cannot be reused by another array while it lives
    (a freed per-tile-size array's id could otherwise alias the next one's)."""
    key = (id(data), tt)
    if key in cache and cache[key]["data"] is not data:
        del cache[key]
    if key not in cache:
        if isinstance(data, TileCounts):
            d = data.values if tt == data.length else _data_slice(data.dense(), tt)  # zeros add nothing
        else:
            d = _data_slice(data, tt)
        # one histogram pass over the (106 M-entry) slice, then every sum over its distinct values:
        # the same per-value expression as the element-wise form, times each value's count
        d = np.asarray(d, dtype=np.int64)
        lo, hi = (int(d.min()), int(d.max())) if d.size else (0, 0)
        if 0 <= lo and hi < (1 << 22):  # tile counts are at most a tile's rows
            cnt = np.bincount(d, minlength=1)
            v = np.arange(cnt.size, dtype=np.int64)
            keep = cnt > 0
            v, cnt = v[keep], cnt[keep]
        else:  # a negative or huge count (never from a tile list): the element-wise form
            v, cnt = d, np.ones_like(d)
        cache[key] = {"nnz": int((v * cnt).sum()), "c8": int((((v + 7) // 8) * cnt).sum()), "v": v, "cnt": cnt,
                      "data": data}
    ent = cache[key]
    if fl not in ent:
        ent[fl] = int((np.ceil((ent["v"] * fl) / BW).astype(np.int64) * ent["cnt"]).sum())
    return ent["nnz"], ent["c8"], ent[fl]


def per_instruction(blocks, tile_size_list, node_num, tiles_for, sinput=False, sparsity=1.0):
    """Closed-form per-instruction model of simulate() (code/simulator.py:272-327) for a stream.

    Returns one dict per instruction, in stream order:
      block, index, TYPE, ID, unit   -- where it is and which modelled unit runs it
      starts                          -- iterations (= Tile_Times = timeline entries)
      rw_bytes                        -- its contribution to simulate()'s rw
      record_bytes, records, nnz      -- what it appends to rw_record: summed bytes, count, and the
                                         summed edge-tile nnz of its LOAD_E/STORE_E records
      busy                            -- summed unit-busy cycles of its iterations (timeline durations)
      first_cost                      -- the cost of its first iteration
    Equal to the records simulate() keeps, bit for bit (tests/golden/simulate_records.json)."""
    out = []
    cache = {}
    data = None
    for b, blk in enumerate(blocks):
        if b == 0 or tile_size_list[b][0] != tile_size_list[b - 1][0]:
            data = tiles_for(tile_size_list[b][0])
            if not isinstance(data, TileCounts):
                data = np.asarray(data, dtype=np.int64)
        for j, inst in enumerate(blk):
            t, fl, tt, ts, unit = (inst["TYPE"], inst["Feature_Length"], inst["Tile_Times"], inst["Tile_Size"],
                                   inst["Hardware_Unit"])
            r = {"block": b, "index": j, "TYPE": t, "ID": inst["ID"], "unit": unit, "starts": tt, "rw_bytes": 0,
                 "record_bytes": 0, "records": 0, "nnz": 0, "busy": 0, "first_cost": 0}
            if tt <= 0:
                out.append(r)
                continue
            if t in ("LOAD_E", "STORE_E"):
                nnz, _, cyc = _edge_sums(cache, data, tt, fl)
                d0 = _first(data, tt)
                r.update(rw_bytes=nnz * fl, record_bytes=nnz * fl, records=tt, nnz=nnz, busy=cyc,
                         first_cost=math.ceil(d0 * fl / BW))
            elif t in ("LOAD_W", "LOAD_N", "STORE_N"):
                sp = (t == "LOAD_N" and "0_applynode" in inst["ID"] and sinput and any(
                    d["TYPE"] == "COMP_MM" and d["ID"].split("_")[0] == inst["ID"].split("_")[0]
                    for d in inst["Dependency"]["WAR"]))
                if sp:  # the sparse-input path adds to rw but records nothing (:292-295)
                    v = math.ceil(ts * fl * sparsity)
                    c = math.ceil(ts * fl * sparsity / BW)
                    r.update(rw_bytes=tt * v, busy=tt * c, first_cost=c)
                else:
                    full = ts * fl
                    last = full
                    if t != "LOAD_W":
                        blk_rows = node_num - math.floor(node_num / ts) * ts
                        last = (blk_rows if blk_rows else ts) * fl
                    cf, cl = math.ceil(full / BW), math.ceil(last / BW)
                    tot = (tt - 1) * math.ceil(full) + math.ceil(last)
                    r.update(rw_bytes=tot, record_bytes=(tt - 1) * full + last, records=tt,
                             busy=(tt - 1) * cf + cl, first_cost=cl if tt == 1 else cf)
            else:
                perf = PERF[unit]
                if t == "COMP_MM":
                    if "0_applynode" in inst["ID"] and sinput:
                        c = math.ceil(ts * sparsity / PERF["VEC_ALU"][0]) * math.ceil(fl / PERF["VEC_ALU"][1])
                    else:
                        c = math.ceil(math.ceil(fl / perf[1]) * math.ceil((inst["Weight_Size"] / fl) / perf[0]))
                    r.update(busy=tt * c, first_cost=c)
                elif "applyedge" in inst["ID"] or "gather" in inst["ID"]:
                    _, c8, _ = _edge_sums(cache, data, tt, fl)
                    f16 = math.ceil(fl / perf[1])
                    d0 = _first(data, tt)
                    r.update(busy=c8 * f16, first_cost=math.ceil(d0 / perf[0]) * f16)
                else:
                    c = math.ceil(ts / perf[0]) * math.ceil(fl / perf[1])
                    r.update(busy=tt * c, first_cost=c)
            out.append(r)
    return out


def rw_info(insts):
    """aggregate_rw_record (code/simulator.py:107-125): ({TYPE: summed bytes}, {TYPE: records})."""
    val, cnt = {}, {}
    for r in insts:
        if r["records"]:
            val[r["TYPE"]] = val.get(r["TYPE"], 0) + r["record_bytes"]
            cnt[r["TYPE"]] = cnt.get(r["TYPE"], 0) + r["records"]
    return val, cnt


def timeline_info(insts, spans):
    """aggregate_timeline (code/simulator.py:127-146): ({TYPE: entries}, {TYPE: summed durations}).
    Restated with its quirk: a type's first entry met (blocks in order, units in UNITS order, then
    time order) initialises the total with its duration and is then added again."""
    count, total = {}, {}
    order = sorted(insts, key=lambda r: (r["block"], UNITS.index(r["unit"]), spans[(r["block"], r["index"])][0]))
    for r in order:
        if r["starts"] <= 0:
            continue
        t = r["TYPE"]
        if t not in count:
            count[t] = 0
            total[t] = r["first_cost"]
        count[t] += r["starts"]
        total[t] += r["busy"]
    return count, total
