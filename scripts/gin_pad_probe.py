"""GIN products aggregate (bf16 rows, F = 100, [E, 1] weights, accumulating) on the table as stored
(200-B rows, 8-B aligned) against the same rows in a 256-B padded table (x[:, :100] of an
[N, 128] bf16 table: every row 128-B aligned, two lines).  Median of HIP-event times; outputs equal."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, ops  # noqa: E402


def timed(fn, reps=10):
    ts = []
    for r in range(reps + 1):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        if r:
            ts.append(a.elapsed_time(b))
    return sorted(ts)[reps // 2]


def main():
    dev = torch.device("cuda:0")
    g = G.dataset_graph("products", seed=0, device=dev)
    F = 100
    x = torch.randn(g.n_rows, F, device=dev).to(torch.bfloat16)
    xp = torch.zeros(g.n_rows, 128, device=dev, dtype=torch.bfloat16)
    xp[:, :F] = x
    w = torch.ones(g.nnz, 1, device=dev)
    acc0 = torch.randn(g.n_rows, F, device=dev)
    y1, y2 = acc0.clone(), acc0.clone()
    out = {}
    for name, xx, y in (("stored_200B", x, y1), ("padded_256B", xp[:, :F], y2)):
        def fn():
            y.copy_(acc0)
            ops.aggregate(g, xx, "src", w, out=y, accumulate=True, plan=512)
        out[name] = timed(fn)
    for name, xx, y in (("stored_200B", x, y1), ("padded_256B", xp[:, :F], y2)):
        y.copy_(acc0)
        ops.aggregate(g, xx, "src", w, out=y, accumulate=True, plan=512)
    torch.cuda.synchronize()
    out["bitwise_equal"] = bool(torch.equal(y1, y2))
    out["copy_ms_note"] = "ms include the [N, 100] fp32 accumulator copy (same in both arms)"
    rep = torch.empty_like(xp)
    out["repack_ms"] = timed(lambda: rep[:, :F].copy_(x))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
