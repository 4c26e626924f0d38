"""Probe: the GIN products aggregate (bf16 200-B rows, F = 100, self term: gta_aggregate_self, the
layer's launch) when every gathered source lies in 1/B of the table -- what column blocking would
buy if each block's slice stayed Infinity-Cache (B >= 2: <= 245 MB) or L2 resident.

Same kernel, same N, E, F; only the source range shrinks (B = 1 is the real workload).  Prints one
JSON line per B: median ms of HIP-event-timed launches and the sector-level rate (4 x 64-B sectors
per gathered 200-B row)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, ops  # noqa: E402


def main(reps=7):
    dev = torch.device("cuda:0")
    g0 = G.dataset_graph("products", seed=0, device=dev)
    n, F = g0.n_rows, 100
    x = torch.randn(n, F, device=dev).to(torch.bfloat16)
    s = torch.full((1,), 1.25, device=dev)
    y = torch.empty(n, F, device=dev)
    for B in [int(v) for v in (sys.argv[1:] or ["1", "2", "3", "4", "8", "64"])]:
        g = g0 if B == 1 else G.Graph(g0.indptr, torch.remainder(g0.indices, n // B).to(torch.int32).contiguous())
        plan = g.plan(512)
        for _ in range(2):
            ops.aggregate(g, x, "src", None, out=y, plan=plan, self_term=(x, s))
        ts = []
        for _ in range(reps):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            ops.aggregate(g, x, "src", None, out=y, plan=plan, self_term=(x, s))
            b.record()
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        ms = float(np.median(ts))
        print(json.dumps({"B": B, "slice_MB": round(n // B * F * 2 / 1e6, 1), "E": g.nnz, "ms": round(ms, 4),
                          "sector_TBps": round(g.nnz * 256 / (ms / 1e3) / 1e12, 3),
                          "alg_TBps": round(g.nnz * (4 + 2 * F) / (ms / 1e3) / 1e12, 3)}), flush=True)
        del g, plan


if __name__ == "__main__":
    main()
