"""Probe: aggregate-kernel rate when all gathered sources lie in a slice of 1/B of X.

Same kernel, same E, N, F, H as the metric; only the source range shrinks
(B=1 is the metric workload).  Tells how fast gathers run once the X slice fits
an XCD's 4 MB L2 -- the premise of a column-blocked aggregate.
"""
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
    dev = torch.device("cuda:0")
    n, e = bench.N_REDDIT, bench.E_REDDIT
    out = {}
    for B in (1, 4, 16, 32, 64, 128):
        g = G.synthetic(n, e, seed=0, device=dev)
        if B > 1:
            span = n // B
            g = G.Graph(g.indptr, torch.remainder(g.indices, span).to(torch.int32).contiguous())
            g.indices, _ = g.indices, None
        gen = torch.Generator(device=dev)
        gen.manual_seed(5)
        x = torch.randn(n, bench.F, generator=gen, device=dev)
        w = torch.rand(g.nnz, bench.HEADS, generator=gen, device=dev)
        y = torch.empty(n, bench.F, device=dev)
        plan = g.plan(512)
        for _ in range(2):
            ops.aggregate(g, x, "src", w, out=y, plan=plan)
        s, t = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(5):
            ops.aggregate(g, x, "src", w, out=y, plan=plan)
        t.record()
        torch.cuda.synchronize()
        ms = s.elapsed_time(t) / 5
        ab = bench.alg_bytes(n, e)
        out[B] = {"slice_MB": n // B * 512 / 1e6, "ms": ms, "alg_TBps": ab / ms / 1e9}
        print(B, json.dumps(out[B]), flush=True)
        del g, x, w, y, plan
        torch.cuda.empty_cache()
    with open(os.path.join(ROOT, "gpurun_out", "l2_probe.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
