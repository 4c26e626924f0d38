"""Interleaved A/B sweep of aggregate-kernel variants on the Reddit-shaped metric workload.

All variants run in ONE process, round-robin over R rounds (cdna_hip_programming.md
§5.4 rule 24); prints median/min kernel ms per variant and writes JSON to gpurun_out/.
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
from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--variants", default="lpe64:c512,lpe64:c512:nt,lpe32:c512,lpe32:c512:nt,lpe64:c1024,"
                                             "lpe64:c1024:nt,lpe64:c256")
    ap.add_argument("--n", type=int, default=bench.N_REDDIT)
    ap.add_argument("--e", type=int, default=bench.E_REDDIT)
    ap.add_argument("--slices", type=int, default=1, help="confine sources to n/slices nodes (L2 probe)")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    g, x, alpha = bench.make_inputs(args.n, args.e, dev)
    if args.slices > 1:
        from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G
        cols = torch.remainder(g.indices.long(), args.n // args.slices)
        rows = g.row_of_edge().long()
        order = torch.sort(rows * args.n + cols).indices  # keep columns sorted within rows (blocked plans)
        g = G.Graph(g.indptr, cols[order].to(torch.int32).contiguous())
        alpha = alpha[order].contiguous()
    y = torch.empty(g.n_rows, bench.F, device=dev)
    variants = []
    for v in args.variants.split(","):
        parts = v.split(":")
        if parts[0].startswith("blk"):  # column-blocked path, B = blk<B>[:w<persistent waves>]
            wv = int(parts[1][1:]) if len(parts) > 1 and parts[1].startswith("w") else 0
            single = 0 if "multi" in parts[1:] else 1
            quarter = 0 if "q0" in parts[1:] else 1  # q0: one item per wave (k_agg_seg2d)
            us = [int(p_[1:]) for p_ in parts[1:] if p_.startswith("u")]
            quarter = quarter * (us[0] if us else 8)  # u<U>: edges per step of the quarter-wave form
            lanes = 32 if "h" in parts[1:] else 16  # h: half-wave items (32 lanes each)
            wv = wv + 10000000 * (lanes // 16 - 1)
            nts = [int(p_[2:]) for p_ in parts[1:] if p_.startswith("nt")]
            wv = wv + 1000 * (nts[0] if nts else 0)  # nt<bits>: non-temporal loads (1) / slab stores (2)
            variants.append((v, -int(parts[0][3:]), quarter, wv, single))
            continue
        lpe = int(parts[0].replace("lpe", ""))
        chunk = None if parts[1] == "none" else int(parts[1].replace("c", ""))
        nt = int("nt" in parts[2:])
        lean = 0 if "lean0" in parts[2:] else 1
        variants.append((v, lpe, chunk, nt, lean))
    plans = {v[2]: (g.plan(v[2]) if v[2] else None) for v in variants if v[1] > 0}
    for v in variants:
        if v[1] < 0:
            g.blocked_plan(-v[1])
    times = {v[0]: [] for v in variants}
    ref = None
    for r in range(args.rounds):
        for name, lpe, chunk, nt, lean in variants:
            if lpe < 0:
                ops.set_debug("seg_lanes", 32 if nt >= 10000000 else 16)
                nt = nt % 10000000
                ops.set_debug("seg_waves", nt % 1000)
                ops.set_debug("seg_nt", nt // 1000)
                ops.set_debug("seg_quarter", 1 if chunk else 0)
                ops.set_debug("seg_u", chunk or 8)

                def run(lpe=lpe, lean=lean):
                    ops.aggregate_blocked(g, x, alpha, out=y, blocks=-lpe, single_launch=bool(lean))
            else:
                ops.set_debug("agg_lpe", lpe)
                ops.set_debug("agg_nt", nt)
                ops.set_debug("agg_lean", lean)

                def run(chunk=chunk):
                    ops.aggregate(g, x, "src", alpha, out=y, plan=plans[chunk])
            run()  # warm
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(args.reps):
                run()
            e.record()
            torch.cuda.synchronize()
            times[name].append(s.elapsed_time(e) / args.reps)
            if r == 0:
                if ref is None:
                    ref = y.clone()
                else:
                    d = (y - ref).abs().max().item()
                    assert d < 1e-3, f"variant {name} differs from the first by {d}"
    ab = bench.alg_bytes(g.n_rows, g.nnz)
    out = {}
    for name in times:
        med = float(np.median(times[name]))
        out[name] = {"median_ms": med, "min_ms": float(np.min(times[name])),
                     "alg_GBps": ab / (med / 1e3) / 1e9, "edges_per_s": g.nnz / (med / 1e3)}
        print(f"{name:16s} median {med:7.3f} ms  min {out[name]['min_ms']:7.3f}  "
              f"{out[name]['alg_GBps']:7.0f} GB/s alg  {out[name]['edges_per_s']/1e9:6.2f} Gedges/s", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"agg_sweep_s{args.slices}.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
