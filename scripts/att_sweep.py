"""Interleaved timing of the fused GAT attention aggregate (gta_gat_aggregate_blocked: GAT ops 6-12,
alpha never materialised) on the Reddit-shaped metric graph, 8 heads, F = 128, per libgta knob
setting; prints median ms per variant and writes gpurun_out/att_sweep.json.

  python scripts/att_sweep.py --knobs "att_lean=0;att_lean=1;att_lean=2" --blocks 20
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--knobs", default="att_lean=0;att_lean=1")
    ap.add_argument("--blocks", default="20")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g = G.synthetic(bench.N_REDDIT, bench.E_REDDIT, seed=0, device=dev)
    gen = torch.Generator(device=dev)
    gen.manual_seed(7)
    x = torch.randn(g.n_rows, bench.F, generator=gen, device=dev)
    ab = torch.randn(g.n_rows, 2 * bench.HEADS, generator=gen, device=dev)  # [a | b] as the sibling GEMM makes them
    a, b = ab[:, :bench.HEADS], ab[:, bench.HEADS:]
    y = torch.empty(g.n_rows, bench.F, device=dev)
    variants = []
    for bl in map(int, args.blocks.split(",")):
        plan = g.blocked_plan(bl)
        for kn in args.knobs.split(";"):
            kv = dict(p.split("=") for p in kn.split(",") if p)
            variants.append((f"B{bl}:{kn}", plan, kv))
    times = {v[0]: [] for v in variants}
    ref = {}  # per block count (B changes the sum order)
    for r in range(args.rounds):
        for name, plan, kv in variants:
            for k, v in kv.items():
                ops.set_debug(k, int(v))
            run = lambda: ops.gat_aggregate_blocked(g, x, a, b, out=y, plan=plan)  # noqa: E731
            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            times[name].append(e0.elapsed_time(e1) / args.reps)
            if r == 0:
                key = plan.blocks
                if key not in ref:
                    ref[key] = y.clone()
                else:
                    assert torch.equal(y, ref[key]), f"{name} differs from the first variant of its B"
            ops.set_debug("att_lean", 2)
    out = {}
    for name, plan, kv in variants:
        med = float(np.median(times[name]))
        out[name] = {"median_ms": med, "min_ms": float(np.min(times[name])), "edges_per_s": g.nnz / (med / 1e3),
                     "items": plan.n_items}
        print(f"{name:28s} median {med:7.3f} ms  min {out[name]['min_ms']:7.3f}  "
              f"{out[name]['edges_per_s'] / 1e9:6.2f} Gedges/s", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "att_sweep.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
