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
"""
import math

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
    def __init__(self, node_num, tiles_for, sinput=False, sparsity=1.0):
        self.N = node_num
        self.tiles_for = tiles_for  # SR -> flat list of tile nnz (row-major [ceil(N/SR)][N])
        self.sinput = sinput
        self.sparsity = sparsity
        self.rw = 0

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


def simulate_stream(blocks, tile_size_list, node_num, tiles_for, sinput=False, sparsity=1.0):
    """(cycles, rw) exactly as code/simulator.py:370-502 computes them for this stream."""
    return _Sim(node_num, tiles_for, sinput, sparsity).run(blocks, tile_size_list)


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
