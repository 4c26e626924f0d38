"""Fused attention aggregate (gta_gat_aggregate_blocked) at B = 1 vs the unfused edge-softmax +
aggregate + divide path on a low-degree graph (Flickr shape, 8 heads, F = 128)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, ops  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        t.append(a.elapsed_time(b) / reps)
    return float(np.median(t))


def main():
    dev = torch.device("cuda:0")
    for ds in ("flickr", "cora"):
        g = G.dataset_graph(ds, device=dev)
        torch.manual_seed(0)
        x = torch.randn(g.n_rows, 128, device=dev)
        a = torch.randn(g.n_rows, 8, device=dev)
        b = torch.randn(g.n_rows, 8, device=dev)
        res = {}
        for B in (1, 2):
            res[f"fused B={B}"] = timed(lambda B=B: ops.gat_aggregate_blocked(g, x, a, b, blocks=B))

        def unfused():
            v, s = ops.edge_softmax(g, a, b, "EXP_LEAKY_RELU", normalize=False, want_sums=True)
            y = ops.aggregate(g, x, "src", v, plan=512)
            return y, s
        res["softmax(v) + aggregate"] = timed(unfused)
        y1, _ = ops.gat_aggregate_blocked(g, x, a, b, blocks=1)
        alpha = ops.edge_softmax(g, a, b, "EXP_LEAKY_RELU")
        y2 = ops.aggregate(g, x, "src", alpha if not isinstance(alpha, tuple) else alpha[0], plan=512)
        print(ds, g.n_rows, g.nnz, {k: round(v * 1e3, 1) for k, v in res.items()}, "us",
              "max|fused - alpha path|", float((y1 - y2).abs().max()), flush=True)


if __name__ == "__main__":
    main()
