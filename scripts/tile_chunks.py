"""One rank's tile of the multi-GPU metric bench, rebuilt alone on one GPU, timed per row chunk,
and the step it would take on the 8-GPU node modelled from those times.

For each --chunk-fracs variant the tile of rank R on the PRxPC grid (bench.build with the
whole-graph column histogram from metric.column_counts, as bench's PMC child does) is built; every
chunk's launch pair is timed alone with HIP events (median of reps), and so is the whole step's
launch sequence.  The exchange is modelled, not measured (one GPU here): chunk c's reduce-scatter
inside a row group of pc ranks moves (pc - 1) / pc of the chunk's partial rows each way,
rows_c x 512 B x (pc - 1) / pc, at an assumed per-direction link rate.  A chunk's exchange starts
when its launch and the previous exchange are done; the step ends when the last exchange ends.
Prints one JSON line per variant: chunk ms, exchange MB, modelled step and speed-up over the
1-GPU step (--one-gpu-ms) at each link rate.

Usage: python scripts/tile_chunks.py [--grid 4x2] [--rank 0] [--one-gpu-ms 4.90] [--rates 64,32]
       [--reps 20] FRACS ...   (FRACS: 1 | 0.5,0.5 | 0.7,0.3 | 0.55,0.3,0.15 ...)
"""
import argparse
import json
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gta_graph_tensor_acclelrator_for_general_gnn_amd import metric  # noqa: E402


def model(chunk_ms, xfer_mb, rate_gbs):
    t_comp, t_comm = 0.0, 0.0
    for c, x in zip(chunk_ms, xfer_mb):
        t_comp += c
        t_comm = max(t_comp, t_comm) + x / rate_gbs  # MB / (GB/s) = ms
    return max(t_comp, t_comm)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--grid", default="4x2")
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--one-gpu-ms", type=float, default=4.90)
    ap.add_argument("--rates", default="64,32", help="per-direction GB/s of the reduce-scatter")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("fracs", nargs="*", default=["1", "0.5,0.5", "0.7,0.3", "0.55,0.3,0.15"])
    a = ap.parse_args()
    pr, pc = (int(v) for v in a.grid.split("x"))
    world = pr * pc
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    counts = metric.column_counts(metric.N_REDDIT, metric.E_REDDIT, dev) if pc > 1 else None
    rates = [float(v) for v in a.rates.split(",")]
    stream = torch.cuda.current_stream(dev)
    for fr in a.fracs:
        parts = [float(v) for v in fr.split(",")]
        chunks = len(parts)
        args = types.SimpleNamespace(mode="edges", grid=a.grid, row_chunks=chunks,
                                     chunk_fracs="equal" if chunks == 1 else fr, n=metric.N_REDDIT,
                                     e=metric.E_REDDIT, blocks=0, impl="blocked")
        shard, agg, *_ = bench.build(args, world, a.rank, dev, "none", lambda m: None, col_counts=counts)
        live = [c for c, (x0, x1, _) in enumerate(agg.parts) if x1 > x0]
        for _ in range(3):
            for c in live:
                agg.launch(c)
        torch.cuda.synchronize()

        def t(fn):
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.reps)]
            for s, e in ev:
                s.record(stream)
                fn()
                e.record(stream)
            torch.cuda.synchronize()
            return float(np.median([s.elapsed_time(e) for s, e in ev]))

        chunk_ms = [t(lambda c=c: agg.launch(c)) for c in live]
        step_ms = t(lambda: [agg.launch(c) for c in live])
        rows = [agg.parts[c][1] - agg.parts[c][0] for c in live]
        xfer_mb = [r * metric.F * 4 * (pc - 1) / pc / 1e6 for r in rows]
        rec = {"grid": a.grid, "rank": a.rank, "fracs": parts, "tile_edges": int(shard.graph.nnz), "blocks": agg.blocks,
               "chunk_ms": [round(v, 4) for v in chunk_ms], "step_compute_ms": round(step_ms, 4),
               "chunk_rows": rows, "exchange_MB": [round(v, 2) for v in xfer_mb]}
        for r in rates:
            # chunk times scaled to the measured back-to-back step (launch gaps included)
            scale = step_ms / max(sum(chunk_ms), 1e-9)
            st = model([c * scale for c in chunk_ms], xfer_mb, r)
            rec[f"model_step_ms@{r:g}GBps"] = round(st, 4)
            rec[f"model_speedup@{r:g}GBps"] = round(a.one_gpu_ms / st, 2)
        print(json.dumps(rec), flush=True)
        del shard, agg
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
