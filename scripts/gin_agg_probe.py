"""The GIN products aggregate (F = 100, no weight, accumulating into the (1+eps) x buffer: the
executor's gather_acc form) timed on the ogbn-products-shaped CSR, plus a streaming calibration
launch of the same kernel (identity CSR: every x row read once, in order) for rocprofv3 --pmc
FETCH_SIZE / WRITE_SIZE passes (scripts/gin_pmc.py reads them).  Prints one JSON line."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, ops  # noqa: E402


def main(reps=10):
    dev = torch.device("cuda:0")
    g = G.dataset_graph("products", seed=0, device=dev)
    F = 100
    x = torch.randn(g.n_rows, F, device=dev)
    acc0 = 1.5 * x
    y = acc0.clone()
    # calibration: identity CSR, one edge per row -> x streamed once (N x 400 B, line-aligned total)
    gi = G.Graph(torch.arange(g.n_rows + 1, device=dev, dtype=torch.int64),
                 torch.arange(g.n_rows, device=dev, dtype=torch.int32))
    yc = torch.zeros_like(x)
    for _ in range(2):
        ops.aggregate(gi, x, "src", None, out=yc, accumulate=True, plan=512)
    torch.cuda.synchronize()
    ts = []
    for r in range(reps + 1):
        y.copy_(acc0)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        ops.aggregate(g, x, "src", None, out=y, accumulate=True, plan=512)
        b.record()
        torch.cuda.synchronize()
        if r:
            ts.append(a.elapsed_time(b))
    ms = float(np.median(ts))
    gathered = g.nnz * F * 4
    lines = g.nnz * 512  # a 400-B row at a 16-B multiple offset always spans 4 lines of 128 B
    out = {"N": g.n_rows, "E": g.nnz, "F": F, "ms": ms, "edges_per_s": g.nnz / (ms / 1e3),
           "alg_GBps": (gathered + g.nnz * 4 + g.n_rows * (8 + 2 * F * 4)) / (ms / 1e3) / 1e9,
           "line_GBps": (lines + g.nnz * 4 + g.n_rows * (8 + 2 * F * 4)) / (ms / 1e3) / 1e9,
           "calib_bytes": g.n_rows * F * 4 * 2 + g.n_rows * (8 + 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
