"""Interleaved sweep of the blocked aggregate's item length (BlockedPlan item_edges) on the
Reddit-shaped metric workload and on single rank tiles of 2-D grids (rank (0, 0)'s tile timed
alone on one GPU, as bench.py --gpus N would run it).  All variants of one shape run in one
process, round-robin; prints median kernel ms per variant, writes gpurun_out/item_sweep.json.

  python scripts/item_sweep.py --grids 1x1,2x2,4x2,8x1 --items 64,128,256,512,0 --blocks 0
  (item 0 = unbounded: one item per (block, row) segment; blocks 0 = auto per tile)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed, ops, partition  # noqa: E402

UNBOUNDED = 1 << 30


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grids", default="1x1")
    ap.add_argument("--items", default="64,128,256,512,0")
    ap.add_argument("--blocks", default="0", help="comma list; 0 = bench's auto choice for the tile")
    ap.add_argument("--rowedges", default="0", help="comma list of light-row merge targets (BlockedPlan row_edges)")
    ap.add_argument("--chunks", default="1", help="comma list of row chunks per tile (one launch per chunk, "
                                                   "chunk-major padded rows as bench.py --row-chunks)")
    ap.add_argument("--knobs", default="", help="';'-separated libgta debug settings per variant, e.g. "
                                              "'seg_lean=0;seg_lean=1' (each a ','-list of key=value)")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n", type=int, default=bench.N_REDDIT)
    ap.add_argument("--e", type=int, default=bench.E_REDDIT)
    ap.add_argument("--slices", type=int, default=1, help="confine sources to n/slices nodes (L2-only probe)")
    ap.add_argument("--plan-knobs", default="", help="libgta settings applied before any plan is built, "
                                                     "e.g. 'rows_cap=1024'")
    args = ap.parse_args()
    for kv in filter(None, args.plan_knobs.split(",")):
        k_, v_ = kv.split("=")
        ops.set_debug(k_, int(v_))
    dev = torch.device("cuda:0")
    t0 = time.time()
    g, x, alpha = bench.make_inputs(args.n, args.e, dev)
    if args.slices > 1:  # every gather hits a table of n/slices rows (columns kept sorted within rows)
        from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G
        cols = torch.remainder(g.indices.long(), args.n // args.slices)
        rows = g.row_of_edge().long()
        order = torch.sort(rows * args.n + cols).indices
        g = G.Graph(g.indptr, cols[order].to(torch.int32).contiguous())
        alpha = alpha[order].contiguous()
    print(f"inputs {time.time() - t0:.1f} s", flush=True)
    defaults = {"seg_lean": 1, "seg_lanes": 32, "seg_u": 8, "seg_nt": 2, "seg_quarter": 1, "seg_lean_w1": 1, "slab_rows": 0}
    out = {}
    for grid in args.grids.split(","):
        pr, pc = map(int, grid.lower().split("x"))
        variants = []
        for ch in map(int, args.chunks.split(",")):
            if pr * pc == 1 and ch == 1:
                gg, xl, wl, parts = g, x, alpha, [(0, g.n_rows)]
            else:
                s = distributed.GridShard(g, 0, pr, pc, chunks=ch)
                gg, xl, wl = s.graph, x[s.c0:s.c1].contiguous(), alpha[s.edge_ids].contiguous()
                parts = [s.chunk_rows(c) for c in range(s.chunks)]
            subs = [gg if len(parts) == 1 else partition.sub_rows(gg, a, b) for a, b in parts]
            y = torch.empty(gg.n_rows, bench.F, device=dev)
            for b in args.blocks.split(","):
                B = int(b) or bench.auto_blocks(gg, bench.F)
                for it in args.items.split(","):
                    ie = int(it) or UNBOUNDED
                    for re_ in map(int, args.rowedges.split(",")):
                        plans = [sg.blocked_plan(B, ie, re_) for sg in subs]
                        for kn in (args.knobs.split(";") if args.knobs else [""]):
                            kv = dict(p_.split("=") for p_ in kn.split(",") if p_)
                            tag = f"{grid}:c{ch}:B{B}:i{it}:r{re_}" + (f":{kn}" if kn else "")
                            variants.append((tag, B, plans, subs, parts, gg, xl, wl, y, kv))
        times = {v[0]: [] for v in variants}
        ref = {}
        for r in range(args.rounds):
            for name, B, plans, subs, parts, gg, xl, wl, y, kv in variants:
                for k_, v_ in kv.items():
                    ops.set_debug(k_, int(v_))

                def run():
                    for (a, b), sg, plan in zip(parts, subs, plans):
                        ops.aggregate_blocked(sg, xl, wl, out=y[a:b], plan=plan, blocks=B)
                run()
                a, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(args.reps):
                    run()
                e.record()
                torch.cuda.synchronize()
                times[name].append(a.elapsed_time(e) / args.reps)
                if r == 0:  # same sums per layout (chunked layouts differ only in padded row order)
                    key = len(parts)
                    if key not in ref:
                        ref[key] = y.clone()
                    else:
                        d = (y - ref[key]).abs().max().item()
                        print(f"  {name}: max |y - first variant| = {d}", flush=True)
                        assert d < 1e-3, f"variant {name} differs from the first by {d}"
                for k_ in kv:
                    ops.set_debug(k_, defaults[k_])
        for name, B, plans, subs, parts, gg, xl, wl, y, kv in variants:
            ab = bench.alg_bytes(gg.n_rows, gg.nnz)
            med = float(np.median(times[name]))
            n_items = sum(p.n_items for p in plans)
            out[name] = {"rows": gg.n_rows, "edges": gg.nnz, "items": n_items, "launches": len(plans),
                         "median_ms": med, "min_ms": float(np.min(times[name])),
                         "alg_GBps": ab / (med / 1e3) / 1e9, "edges_per_s": gg.nnz / (med / 1e3)}
            print(f"{name:22s} items {n_items:9d}  median {med:7.3f} ms  min {out[name]['min_ms']:7.3f}  "
                  f"{out[name]['alg_GBps']:7.0f} GB/s alg  {out[name]['edges_per_s'] / 1e9:6.2f} Gedges/s", flush=True)
        del variants
        torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "item_sweep.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
