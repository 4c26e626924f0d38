"""Row-chunked metric aggregate with each chunk's ordered reduce overlapped with the next chunk's
item launch (a second stream), against the one-launch form, interleaved in one process.

The rows are cut into C chunks of equal edge count, each with its own column-blocked plan (B as
bench.py picks); variant 'seq' runs chunk after chunk (items + reduce), 'overlap' runs the item
launches back to back on the main stream (knob seg_phase = 1) and chunk c's reduce (seg_phase = 2)
on a side stream once chunk c's items are done.  Every variant's output must equal the one-launch
form bitwise (the per-row reduce order does not depend on the chunking).  Writes
gpurun_out/overlap_probe.json."""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, metric, ops  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="2,4")
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    t0 = time.time()
    sh = metric.Shard(metric.N_REDDIT, metric.E_REDDIT, 0, 1, 1, 1, dev, keep_rows=False)
    g = sh.graph
    B = ops.BlockedPlan.auto_blocks(g, metric.F)
    plan = g.blocked_plan(B)
    ip = g.indptr
    parts = {}
    for C in (int(c) for c in args.chunks.split(",")):
        cuts = torch.searchsorted(ip, torch.arange(C + 1, device=dev, dtype=torch.int64) * g.nnz // C).tolist()
        cuts[0], cuts[-1] = 0, g.n_rows
        pc = []
        for a, b in zip(cuts[:-1], cuts[1:]):
            gg = G.Graph(ip[a:b + 1], g.indices, n_cols=g.n_cols)
            pc.append((a, b, gg, gg.blocked_plan(B)))
        parts[C] = pc
    print(f"inputs ready in {time.time() - t0:.1f} s, B={B}", flush=True)
    side = torch.cuda.Stream(dev)
    main_s = torch.cuda.current_stream(dev)
    y = torch.empty(g.n_rows, metric.F, device=dev)

    def one():
        ops.aggregate_blocked(g, sh.x, sh.alpha, out=y, plan=plan)

    def seq(C):
        for a, b, gg, pl in parts[C]:
            ops.aggregate_blocked(gg, sh.x, sh.alpha, out=y[a:b], plan=pl)

    def overlap(C):
        for a, b, gg, pl in parts[C]:
            ops.set_debug("seg_phase", 1)
            ops.aggregate_blocked(gg, sh.x, sh.alpha, out=y[a:b], plan=pl)
            ev = torch.cuda.Event()
            ev.record(main_s)
            side.wait_event(ev)
            with torch.cuda.stream(side):
                ops.set_debug("seg_phase", 2)
                ops.aggregate_blocked(gg, sh.x, sh.alpha, out=y[a:b], plan=pl)
        ops.set_debug("seg_phase", 0)
        main_s.wait_stream(side)

    variants = [("one launch", one)]
    for C in parts:
        variants += [(f"seq C={C}", lambda C=C: seq(C)), (f"overlap C={C}", lambda C=C: overlap(C))]
    times = {n: [] for n, _ in variants}
    ref = None
    for r in range(args.rounds):
        for name, fn in variants:
            y.fill_(float("nan"))
            fn()
            torch.cuda.synchronize()
            if r == 0:
                if ref is None:
                    ref = y.clone()
                else:
                    same = torch.equal(y, ref)
                    print(f"  {name}: bitwise {'equal' if same else 'DIFFERENT'}", flush=True)
                    assert same, name
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record(main_s)
            for _ in range(args.reps):
                fn()
            e.record(main_s)
            torch.cuda.synchronize()
            times[name].append(s.elapsed_time(e) / args.reps)
        print(f"round {r}: " + ", ".join(f"{n} {times[n][-1]:.3f}" for n in times), flush=True)
    out = {}
    for name in times:
        med = float(np.median(times[name]))
        out[name] = {"median_ms": med, "min_ms": float(np.min(times[name])), "edges_per_s": g.nnz / (med / 1e3)}
        print(f"{name:16s} median {med:7.3f} ms  min {out[name]['min_ms']:7.3f}  "
              f"{out[name]['edges_per_s'] / 1e9:6.2f} G edges/s", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "overlap_probe.json"), "w") as f:
        json.dump({"blocks": B, "variants": out}, f, indent=1)


if __name__ == "__main__":
    main()
