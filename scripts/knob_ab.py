"""Interleaved A/B of libgta tuning knobs on the metric workload (bench.py's exact call).

Each variant is a ';'-free list of knob=value pairs (gta_debug_set keys), variants separated by
'/', e.g.  --variants "seg_fuse=0/seg_fuse=1/seg_fuse=1,plan_len_sort=0".
All variants run in ONE process, round-robin over R rounds (cdna_hip_programming.md §5.4 rule 24);
every variant's output must be bitwise equal to the first's (--tol to relax).  Prints median/min
ms per variant and writes gpurun_out/knob_ab.json.
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

from gta_graph_tensor_acclelrator_for_general_gnn_amd import metric, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="seg_fuse=0/seg_fuse=1")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--blocks", type=int, default=0)
    ap.add_argument("--n", type=int, default=metric.N_REDDIT)
    ap.add_argument("--e", type=int, default=metric.E_REDDIT)
    ap.add_argument("--tol", type=float, default=0.0)
    ap.add_argument("--out", default="knob_ab.json")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    t0 = time.time()
    sh = metric.Shard(args.n, args.e, 0, 1, 1, 1, dev, keep_rows=False)
    g = sh.graph
    B = args.blocks or ops.BlockedPlan.auto_blocks(g, metric.F)
    plan = g.blocked_plan(B)
    print(f"inputs ready in {time.time() - t0:.1f} s, B={B}, items={plan.n_items}", flush=True)
    variants = []
    for v in args.variants.split("/"):
        kv = [p.split("=") for p in v.split(",") if p]
        variants.append((v, [(k, int(val)) for k, val in kv]))
    y = torch.empty(g.n_rows, metric.F, device=dev)
    times = {name: [] for name, _ in variants}
    ref = None
    for r in range(args.rounds):
        for name, kv in variants:
            for k, val in kv:
                ops.set_debug(k, val)
            y.fill_(float("nan"))
            ops.aggregate_blocked(g, sh.x, sh.alpha, out=y, plan=plan)  # warm + checked output
            torch.cuda.synchronize()
            if r == 0:
                if ref is None:
                    ref = y.clone()
                else:
                    d = (y - ref).abs().max().item()
                    same = torch.equal(y, ref)
                    print(f"  {name}: bitwise {'equal' if same else 'DIFFERENT'} (max |d| {d:.3g})", flush=True)
                    assert same or d <= args.tol, f"variant {name} differs from the first"
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.reps):
                ops.aggregate_blocked(g, sh.x, sh.alpha, out=y, plan=plan)
            e.record()
            torch.cuda.synchronize()
            times[name].append(s.elapsed_time(e) / args.reps)
            for k, _ in kv:  # back to the defaults
                ops.set_debug(k, DEFAULTS.get(k, 0))
        print(f"round {r}: " + ", ".join(f"{n} {times[n][-1]:.3f}" for n in times), flush=True)
    out = {}
    for name in times:
        med = float(np.median(times[name]))
        out[name] = {"median_ms": med, "min_ms": float(np.min(times[name])), "edges_per_s": g.nnz / (med / 1e3)}
        print(f"{name:40s} median {med:7.3f} ms  min {out[name]['min_ms']:7.3f}  "
              f"{out[name]['edges_per_s'] / 1e9:6.2f} G edges/s", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", args.out), "w") as f:
        json.dump({"n": args.n, "e": args.e, "blocks": B, "variants": out}, f, indent=1)


DEFAULTS = {"seg_fuse": 0, "seg_lean": 1, "seg_nt": 3, "plan_len_sort": 1, "seg_lanes": 32, "seg_u": 8,
            "seg_quarter": 1, "seg_lean_w1": 1}

if __name__ == "__main__":
    main()
