"""Time gta_aggregate_expr on the Flickr-shaped graph (DGN's shape 3, PNA's shape 2) against the
unfused ops and a plain SpMM of one table, with HIP events (median of reps).  A/B of the
expression kernel's forms (knob expr_lean); prints one JSON line per case."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, ops  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda:0")
    g = G.dataset_graph("flickr", seed=0, device=dev)
    F = int(sys.argv[1]) if len(sys.argv) > 1 else 128
    gen = torch.Generator(device=dev).manual_seed(0)
    P, Q = (torch.randn(g.n_rows, F, device=dev, generator=gen) for _ in range(2))
    EW = torch.randn(g.nnz, F, device=dev, generator=gen)
    plan = 512
    dgn = [(P, "src"), (P, "dst"), (Q, "src"), (Q, "dst")]
    pna = [(P, "src"), (Q, "dst"), (EW, "edge")]
    out = {}
    for lean in (1, 0):
        ops.set_debug("expr_lean", lean)
        out[f"dgn_expr_lean{lean}"] = timed(lambda: ops.aggregate_expr(g, 3, dgn, ("ADD",) * 3, None, plan=plan))
        out[f"pna_expr_lean{lean}"] = timed(lambda: ops.aggregate_expr(g, 2, pna, ("ADD", "ADD"), (None, "RELU"), True,
                                                                      plan=plan))
    ops.set_debug("expr_lean", 1)

    def dgn_unfused():
        a = ops.apply_edge(g, "ADD", None, P, "src", P, "dst")
        b = ops.apply_edge(g, "ADD", None, Q, "src", Q, "dst")
        return ops.aggregate(g, ops.apply_edge(g, "ADD", None, a, "edge", b, "edge"), "edge", plan=plan)
    out["dgn_unfused"] = timed(dgn_unfused)
    out["spmm_one_table"] = timed(lambda: ops.aggregate(g, P, "src", plan=plan))
    out["aggregate_edge_tensor"] = timed(lambda: ops.aggregate(g, EW, "edge", plan=plan))
    y1 = ops.aggregate_expr(g, 3, dgn, ("ADD",) * 3, None, plan=plan)
    out["dgn_bitwise_vs_unfused"] = bool(torch.equal(y1, dgn_unfused()))
    print(json.dumps({"F": F, "N": g.n_rows, "E": g.nnz, "us": out}))


if __name__ == "__main__":
    main()
