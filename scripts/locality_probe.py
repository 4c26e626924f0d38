"""The metric aggregate (Reddit shape, F = 128, 8 head weights) on SURVEY §8(d)'s "locality" variant of
the synthetic graph: sources within +-W of the destination row instead of uniform over [0, N).
For each W: the column-blocked pair (B = 20, the bench's form, and any --blocks) against
the single-pass row-chunked aggregate (512-edge plan), HIP events, interleaved rounds; the two
outputs agree to fp32 rounding (different fold orders).

Usage: python scripts/locality_probe.py [--rounds R] [--widths W1,W2,...] [--blocks B1,B2,...]
(width 0 = uniform sources; blocks default 20)"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, ops  # noqa: E402

N, E = 232965, 114615892


def main():
    argv = sys.argv[1:]
    rounds = int(argv[argv.index("--rounds") + 1]) if "--rounds" in argv else 3
    widths = [int(v) for v in argv[argv.index("--widths") + 1].split(",")] if "--widths" in argv else [0, 65536, 8192, 1024]
    blocks = [int(v) for v in argv[argv.index("--blocks") + 1].split(",")] if "--blocks" in argv else [20]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.current_stream(dev)
    for W in widths:
        g = G.synthetic(N, E, seed=0, device=dev, locality_width=W or None)
        x = torch.randn(N, 128, device=dev)
        a = torch.rand(g.nnz, 8, device=dev)
        forms = {f"blocked_B{b}": (lambda b=b: ops.aggregate_blocked(g, x, a, blocks=b))
                 for b in blocks}
        forms["row_chunked"] = lambda: ops.aggregate(g, x, "src", a, plan=512)
        times = {k: [] for k in forms}
        outs = {}
        for r in range(rounds):
            for k, fn in forms.items():
                outs[k] = fn().clone()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(10)]
                for s0, s1 in ev:
                    s0.record(stream)
                    fn()
                    s1.record(stream)
                torch.cuda.synchronize()
                times[k].append(float(np.median([s0.elapsed_time(s1) for s0, s1 in ev])))
        d = max(float((outs[k] - outs["row_chunked"]).abs().max()) for k in outs)
        ms = {k: round(float(np.median(v)), 4) for k, v in times.items()}
        print(json.dumps({"locality_width": W or "uniform", "E": g.nnz, "ms": ms,
                          "G_edges_per_s": {k: round(g.nnz / v / 1e6, 2) for k, v in ms.items()},
                          "max_abs_diff": d, "max_abs_out": float(outs["row_chunked"].abs().max())}), flush=True)
        del g, x, a, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
