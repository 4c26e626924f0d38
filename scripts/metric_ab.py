"""A/B of the metric aggregate's kernel forms on bench.py's exact inputs, in one process.

Builds the Reddit metric shard once (metric.Shard, one rank), then times every (knob set, block
count) variant with HIP events over back-to-back launches of ops.aggregate_blocked -- the item
launch and the ordered reduce apart (knob seg_phase) and the pair -- in interleaved rounds, and
checks each variant's output bitwise against the first variant's at the same block count.
Prints one JSON line per variant (median over rounds).

Usage: python scripts/metric_ab.py [--rounds R] [--reps K] VARIANT ...
  VARIANT = B[:knob=v[,knob=v...]], e.g.  20  16  20:seg_lean=0
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import metric, ops  # noqa: E402


def parse(v):
    b, _, kn = v.partition(":")
    knobs = dict((k, int(x)) for k, x in (p.split("=") for p in kn.split(",") if p))
    return int(b), knobs


def timed(fn, reps, stream):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(stream)
        fn()
        b.record(stream)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    args = sys.argv[1:]
    rounds, reps = 3, 10
    if "--rounds" in args:
        i = args.index("--rounds")
        rounds = int(args[i + 1])
        del args[i:i + 2]
    if "--reps" in args:
        i = args.index("--reps")
        reps = int(args[i + 1])
        del args[i:i + 2]
    variants = [parse(v) for v in (args or ["20", "20:seg_lean=0"])]
    dev = torch.device("cuda", 0)
    sh = metric.Shard(metric.N_REDDIT, metric.E_REDDIT, 0, 1, 1, 1, dev, keep_rows=False)
    g, x, a = sh.graph, sh.x, sh.alpha
    stream = torch.cuda.current_stream(dev)
    outs, ref = {}, {}
    res = {i: {"pair": [], "items": [], "reduce": []} for i in range(len(variants))}
    for B, _ in variants:
        g.blocked_plan(B)
    for r in range(rounds):
        for i, (B, knobs) in enumerate(variants):
            y = outs.setdefault(i, torch.empty(g.n_rows, metric.F, device=dev))
            old = {k: ops.get_debug(k) for k in knobs}
            try:
                for k, v in knobs.items():
                    ops.set_debug(k, v)
                run = lambda: ops.aggregate_blocked(g, x, a, out=y, blocks=B)  # noqa: E731
                run()
                torch.cuda.synchronize()
                if r == 0:
                    if B in ref:
                        res[i]["bitwise_vs_first"] = bool(torch.equal(y, ref[B]))
                    else:
                        ref[B] = y.clone()
                res[i]["pair"].append(timed(run, reps, stream))
                for ph, name in ((1, "items"), (2, "reduce")):
                    ops.set_debug("seg_phase", ph)
                    res[i][name].append(timed(run, reps, stream))
                ops.set_debug("seg_phase", 0)
            finally:
                ops.set_debug("seg_phase", 0)
                for k, v in old.items():
                    ops.set_debug(k, v)
    for i, (B, knobs) in enumerate(variants):
        d = res[i]
        rec = {"blocks": B, "knobs": knobs, "n_items": g.blocked_plan(B).n_items,
               "pair_ms": round(float(np.median(d["pair"])), 4), "items_ms": round(float(np.median(d["items"])), 4),
               "reduce_ms": round(float(np.median(d["reduce"])), 4), "pair_all": [round(v, 4) for v in d["pair"]],
               "bitwise_vs_first": d.get("bitwise_vs_first")}
        rec["G_edges_per_s"] = round(metric.E_REDDIT / (rec["pair_ms"] / 1e3) / 1e9, 2)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
