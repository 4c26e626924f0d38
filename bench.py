"""Headline benchmark: GAT neighbour AGGREGATE on Reddit-shaped CSR (BASELINE.json metric).

One "step" = one pass of the hot path over the whole graph: the fused
COMP_MUL_COMP_ADD block [3, 11, 12] of GAT layer 1 (scatter C -> applyedge MUL
-> gather ADD, reference code/interpreter.py:575-636, 764-802), i.e.
    Y[i, :] = sum_{e -> i} alpha[e, head(c)] * X1[src(e), :]
with N = 232,965, E = 114,615,892, F = 128 fp32 = 8 heads x 16, alpha [E, 8]
fp32.  Inputs are synthetic (seeded lognormal-degree CSR, uniform sources,
X ~ N(0,1), alpha = softmax over in-edges of N(0,1) logits) and resident in
HBM before the timed region.

--gpus N (launched by torch.distributed.run): the edges are cut into a grid of
tiles -- pr row groups (destination rows, nnz-balanced) x pc column groups
(source columns, nnz-balanced), the reference's row-tile x column blocking
(code/preprocessing.py:26-38).  Default pr = N, pc = 1: each rank aggregates
the in-edges of its destination-row tile (X replicated, 119 MB of 288 GB) in
one launch and ends with its rows of Y; row tiles are independent, so there is
no data-path collective.  Per-rank compute of a row tile equals that of a 2-D
tile of the same edge count (profiles/r01_grid_sweep.json), so column groups
would only add their exchange.  --grid PRxPC (pc > 1) gives the 2-D form: the
pc ranks of a row group sum their partial aggregates with one RCCL
reduce-scatter per row chunk, overlapped with the next chunk.  --layout chunked
keeps 1-D source-column shards with per-row-chunk collectives (--collective
all_reduce | reduce_scatter).  Total work fixed: "strong".

Printed JSON (rank 0): value = edges/s of the whole job; roofline = the
aggregate kernel's algorithmic HBM bytes (548 B/edge + 520 B/node, SURVEY.md
§8d) per launch / its HIP-event-timed duration vs 8 TB/s; cpu_baseline = the
oracle's C restatement (OpenMP) on a bounded row sample on the host cores.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed, graph as G, ops, partition  # noqa: E402

N_REDDIT, E_REDDIT = 232965, 114615892
F, HEADS = 128, 8
PEAK_HBM_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def alg_bytes(n_rows, nnz, f=F, heads=HEADS):
    """per edge 4 (col idx) + 4*H (alpha) + 4*F (gathered X row); per node 8 (indptr) + 4*F (Y)."""
    return nnz * (4 + 4 * heads + 4 * f) + n_rows * (8 + 4 * f)


def make_inputs(n, e, device, seed=0):
    g = G.synthetic(n, e, seed=seed, device=device)
    gen = torch.Generator(device=device)
    gen.manual_seed(seed + 100)
    x = torch.randn(n, F, generator=gen, device=device)
    logits = torch.randn(g.nnz, HEADS, generator=gen, device=device)
    # alpha = softmax over each destination's in-edges, per head (GAT ops 6-10), computed with libgta
    ex = torch.exp(logits)
    s = ops.gather_add(g, ex)
    alpha = ops.apply_edge(g, "DIV", None, ex, "edge", s, "dst")
    del logits, ex, s
    return g, x, alpha


def grid_chunks(pc):
    """Row chunks per rank tile: the reduce-scatter of chunk k overlaps chunk k+1's aggregate."""
    return 1 if pc == 1 else 2


def auto_blocks(graph, f):
    return ops.BlockedPlan.auto_blocks(graph, f)


def cpu_baseline(g, x, alpha, target_s=12.0):
    """Oracle C aggregate (OpenMP) on the first rows of the same workload, ~target_s of CPU work."""
    from oracle import cbase
    cbase.load()
    try:
        cores = min(len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", "16")))
    except AttributeError:
        cores = os.cpu_count()
    ip = g.indptr.cpu().numpy()
    ix = g.indices.cpu().numpy()
    xh = x.cpu().numpy()

    def run(rows):
        e1 = int(ip[rows])
        a = alpha[:e1].cpu().numpy()
        t0 = time.perf_counter()
        cbase.aggregate(ip[: rows + 1], ix[:e1], xh, a, 0, rows, threads=cores)
        return time.perf_counter() - t0, e1

    rows = min(g.n_rows, 2000)
    dt, ecount = run(rows)  # calibration
    rate = ecount / max(dt, 1e-6)
    want_edges = min(int(rate * target_s / 3), g.nnz)
    rows = int(min(g.n_rows, max(1, np.searchsorted(ip, want_edges))))
    times = []
    for _ in range(3):
        dt, ecount = run(rows)
        times.append(dt)
    best = float(np.median(times))
    return {"value": ecount / best, "unit": "edges/s", "cores": cores, "kind": "port",
            "sample": f"rows [0,{rows}) = {ecount} edges of the same graph/X/alpha, median of 3, "
                      f"oracle/spmm_ref.c fp32 OpenMP"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--chunk", type=int, default=512, help="aggregate plan row-chunk (edges)")
    ap.add_argument("--row-chunks", type=int, default=0, help="row chunks for comm overlap (0 = auto)")
    ap.add_argument("--lpe", type=int, default=0, help="force lanes-per-edge variant (32 or 64)")
    ap.add_argument("--impl", choices=["blocked", "plan"], default="blocked",
                    help="blocked: column-blocked aggregate (L2-resident X slices); plan: row-chunked single pass")
    ap.add_argument("--blocks", type=int, default=0,
                    help="column blocks of the blocked aggregate (0 = auto: ~7.5 MB X slices, >= 24 edges/row/block)")
    ap.add_argument("--n", "--graph-nodes", dest="n", type=int, default=N_REDDIT)
    ap.add_argument("--e", "--graph-edges", dest="e", type=int, default=E_REDDIT)
    ap.add_argument("--collective", choices=["reduce_scatter", "all_reduce"], default="reduce_scatter",
                    help="N>1 exchange: reduce-scatter hands each rank the summed rows of its own node range "
                         "(distributed.py layout, half the bytes); all-reduce gives every rank all of Y")
    ap.add_argument("--layout", choices=["grid", "chunked"], default="grid",
                    help="N>1: grid = 2-D edge tiles (row groups x column groups, distributed.GridShard), one "
                         "aggregate launch per rank, reduce-scatter inside each row group; chunked = 1-D source-"
                         "column shards over all rows, per-row-chunk collectives overlapped with compute")
    ap.add_argument("--grid", default="auto", help="PRxPC rank grid for --layout grid (auto: 1x2, 2x2, 4x2 ...)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # rehearsal knobs for a 1-GPU box: GTA_DIST_BACKEND=gloo GTA_SINGLE_DEVICE=1 (all ranks on cuda:0)
    backend = os.environ.get("GTA_DIST_BACKEND", "nccl")
    if os.environ.get("GTA_SINGLE_DEVICE"):
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    if args.lpe:
        ops.set_debug("agg_lpe", args.lpe)

    verbose = bool(os.environ.get("GTA_BENCH_VERBOSE"))

    def note(msg):
        if verbose:
            print(f"[rank {rank}] {time.strftime('%H:%M:%S')} {msg}", file=sys.stderr, flush=True)

    note("building inputs")
    g, x, alpha = make_inputs(args.n, args.e, dev)
    nnz_total = g.nnz
    note("inputs ready")
    grid = world > 1 and args.layout == "grid"
    rs = world > 1 and args.collective == "reduce_scatter" and not grid
    if grid:
        pr, pc = distributed.grid_shape(world) if args.grid == "auto" else map(int, args.grid.lower().split("x"))
        if pr * pc != world:
            raise SystemExit(f"--grid {pr}x{pc} does not match {world} ranks")
        n_chunks = args.row_chunks or grid_chunks(pc)
        shard = distributed.GridShard(g, rank, pr, pc, chunks=n_chunks)
        note(f"grid shard {shard.i},{shard.j}: {shard.graph.nnz} edges, {n_chunks} row chunks")
        groups = distributed.row_groups(pr, pc)
        note("row groups ready")
        gl = shard.graph
        xl = x[shard.c0:shard.c1].contiguous()
        wl = alpha[shard.edge_ids].contiguous()
    elif world > 1:
        n_chunks = args.row_chunks or 8
        if rs:
            shard = distributed.DistShard(g, rank, world, chunks=n_chunks)
        else:
            shard = partition.make_shard(g, rank, world)
        gl = shard.graph
        xl = x[shard.c0:shard.c1].contiguous()
        wl = alpha[shard.edge_ids].contiguous()
    else:
        shard, gl, xl, wl = None, g, x, alpha
        n_chunks = args.row_chunks or 1

    def make_chunks(chunk):
        if grid:  # one launch per row chunk of the rank's tile (one launch over the tile at 1 chunk)
            c = partition.ChunkedRows.__new__(partition.ChunkedRows)
            c.graph, c.parts = gl, []
            for k in range(shard.chunks):
                r0, r1 = shard.chunk_rows(k)
                gg = gl if shard.chunks == 1 else partition.sub_rows(gl, r0, r1)
                c.parts.append((r0, r1, gg, gg.plan(chunk) if chunk else None))
            return c
        if not rs:
            return partition.ChunkedRows(gl, n_chunks=n_chunks, chunk=chunk)
        parts = []  # chunk k = padded rows [k*W*mk, (k+1)*W*mk): one part per rank
        for k in range(shard.chunks):
            r0, r1 = shard.chunk_rows(k)
            gg = partition.sub_rows(gl, r0, r1)
            parts.append((r0, r1, gg, gg.plan(chunk) if chunk else None))
        c = partition.ChunkedRows.__new__(partition.ChunkedRows)
        c.graph, c.parts = gl, parts
        return c
    chunked = make_chunks(args.chunk if args.impl == "plan" else 0)
    impl = args.impl
    if impl == "blocked" and not args.blocks:
        args.blocks = auto_blocks(gl, F)
        if args.blocks < 4:  # slices already L2/MALL-friendly and segments short: single pass wins
            impl = "plan"
    if impl == "blocked":
        for _, _, gg, _ in chunked.parts:
            if not (ops.BlockedPlan.supports(F, HEADS) and gg.blocked_plan(args.blocks).sorted):
                impl = "plan"
        if impl == "plan":
            chunked = make_chunks(args.chunk)
    y = torch.empty(gl.n_rows if (rs or grid) else g.n_rows, F, device=dev)
    y_own = torch.empty(shard.chunks * shard.mk, F, device=dev) if rs else None  # this rank's reduced rows
    if grid:
        y_own = y if pc == 1 else torch.empty(shard.out_rows(), F, device=dev)
        my_group = groups[shard.i]
    stream = torch.cuda.current_stream(dev)

    def agg_chunk(gg, xx, ww, out, plan):
        if impl == "blocked":
            return ops.aggregate_blocked(gg, xx, ww, out=out, blocks=args.blocks)
        return ops.aggregate(gg, xx, "src", ww, out=out, plan=plan)

    def step():
        if grid:  # chunk k's reduce-scatter runs while chunk k+1 aggregates
            mk, works = shard.mk, []
            for k, (r0, r1, gg, plan) in enumerate(chunked.parts):
                agg_chunk(gg, xl, wl, y[r0:r1], plan)
                if pc == 1:  # row tile: the rows are complete, y is the rank's output
                    continue
                own = y_own[k * mk:(k + 1) * mk]
                if backend == "nccl":  # RCCL reduce-scatter among the pc ranks of this row group
                    works.append(dist.reduce_scatter_tensor(own, y[r0:r1], group=my_group, async_op=True))
                else:  # gloo (1-GPU rehearsal): no reduce-scatter
                    dist.all_reduce(y[r0:r1], group=my_group)
                    own.copy_(y[r0 + shard.j * mk:r0 + (shard.j + 1) * mk])
            for wk in works:
                wk.wait()
            return
        if not rs:
            partition.distributed_aggregate(chunked, xl, wl, y, aggregate_fn=agg_chunk)
            return
        works = []
        for k, (r0, r1, gg, plan) in enumerate(chunked.parts):
            agg_chunk(gg, xl, wl, y[r0:r1], plan)
            own = y_own[k * shard.mk:(k + 1) * shard.mk]
            if backend == "nccl":  # RCCL reduce-scatter of chunk k while chunk k+1 computes
                works.append(dist.reduce_scatter_tensor(own, y[r0:r1], async_op=True))
            else:  # gloo (1-GPU rehearsal): no reduce-scatter
                dist.all_reduce(y[r0:r1])
                own.copy_(y[r0 + rank * shard.mk:r0 + (rank + 1) * shard.mk])
        for wk in works:
            wk.wait()

    note(f"impl {impl}, warmup")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    note("timing")

    # kernel-only timing (HIP events on the launch stream) for the roofline
    n_evt = min(args.steps, 10)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_evt)]
    for a, b in evs:
        a.record(stream)
        for r0, r1, gg, plan in chunked.parts:
            agg_chunk(gg, xl, wl, y[r0:r1], plan)
        b.record(stream)
    torch.cuda.synchronize()
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))

    # timed region: K steps, barrier + sync on both sides, max over ranks
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt * 1e3 / args.steps
    value = nnz_total / (ms_per_step / 1e3)

    # size-independent parity checks on the full workload (outside the timed region):
    # N=1: a repeat run is bitwise identical; N>1: the all-reduced Y equals the 1-GPU aggregate
    y_mine = y.clone()
    if world > 1:
        ref = ops.aggregate(g, x, "src", alpha, plan=args.chunk)
        if grid:  # reassemble Y from every rank's reduced rows (row groups may differ in m: pad)
            mmax = max(len(shard.owned_rows(q)) for q in range(world))
            mine = torch.zeros(mmax, F, device=dev)
            mine[:y_own.shape[0]] = y_own
            parts = [torch.empty_like(mine) for _ in range(world)]
            dist.all_gather(parts, mine)
            full = torch.empty_like(ref)
            for q in range(world):
                rows = shard.owned_rows(q).to(dev)
                ok = rows >= 0
                full[rows[ok]] = parts[q][:rows.numel()][ok]
            y_mine, what = full, (f"{pr}x{pc} grid tiles" + (", reduce-scattered per row group" if pc > 1 else "") +
                                  " (reassembled) vs 1-GPU")
        elif rs:  # reassemble Y from every rank's reduced rows
            parts = [torch.empty_like(y_own) for _ in range(world)]
            dist.all_gather(parts, y_own)
            full = torch.empty_like(ref)
            for q in range(world):
                rows = shard.global_rows(q).to(dev)
                ok = rows >= 0
                full[rows[ok]] = parts[q][ok]
            y_mine, what = full, "reduce-scattered shards (reassembled) vs 1-GPU aggregate"
        else:
            what = "allreduced shards vs 1-GPU aggregate"
        err = float((y_mine - ref).abs().max().item())
        scale = float(ref.abs().max().item())
        parity = {"check": what, "max_abs_err": err, "max_abs_ref": scale, "ok": err <= 1e-4 * scale + 1e-5}
    else:
        step()
        parity = {"check": "repeat run bitwise identical", "ok": bool(torch.equal(y, y_mine))}

    # roofline of the dominant kernel (this rank's shard)
    ab = alg_bytes(gl.n_rows, gl.nnz)
    achieved = ab / (kern_ms / 1e3) / 1e9
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(pmc_path) and world == 1:
        try:
            pm = json.load(open(pmc_path))
            if pm.get("n") == args.n and pm.get("e") == args.e and pm.get("impl", "plan") == impl:
                traffic = pm.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    result = {
        "metric": "edges/sec + achieved HBM GB/s, GAT aggregate on Reddit, 1/2/4/8 MI355X",
        "value": value,
        "unit": "edges/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic: seeded lognormal-degree CSR (mean deg 492), uniform sources, X~N(0,1), "
                "alpha=per-head softmax over in-edges",
        "config": {"workload": "GAT layer-1 aggregate block [3,11,12] (scatter C -> applyedge MUL -> gather ADD)",
                   "graph": "reddit-shaped", "N": args.n, "E": nnz_total, "F": F, "heads": HEADS,
                   "parallelism": ("one GPU, whole graph" if world == 1 else
                                   f"destination-row tiles x{pr} (X replicated, no data-path collective)"
                                   if grid and pc == 1 else
                                   f"2-D edge tiles {pr}x{pc} (row groups x source-column groups), RCCL reduce-scatter "
                                   f"of the partial aggregates inside each row group" if grid else
                                   f"edge-partition by source column x{world}" + (
                                       (" + RCCL reduce-scatter per row chunk (each rank ends with its node "
                                        "range's rows)" if rs else " + RCCL all-reduce per row chunk")
                                       if world > 1 else "")),
                   "impl": impl, "blocks": args.blocks if impl == "blocked" else None,
                   "plan_chunk": args.chunk if impl == "plan" else None, "row_chunks": n_chunks},
        "achieved_GBps": nnz_total and alg_bytes(g.n_rows, nnz_total) / (ms_per_step / 1e3) / 1e9,
        "parity": parity,
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
                     "frac": achieved / PEAK_HBM_GBS, "traffic": traffic,
                     "kernel_ms": kern_ms, "alg_bytes_per_launch": ab,
                     # PMC bytes (L2 <-> fabric, incl. Infinity-Cache hits) per launch over the same time
                     "traffic_GBps": traffic and traffic / (kern_ms / 1e3) / 1e9,
                     "traffic_frac": traffic and traffic / (kern_ms / 1e3) / 1e9 / PEAK_HBM_GBS,
                     "kernels": ("k_agg_h32 + k_seg_reduce" if impl == "blocked" else "k_aggregate + combine")},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = cpu_baseline(g, x, alpha)
    elif rank == 0:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
