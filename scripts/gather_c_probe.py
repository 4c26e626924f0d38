"""The ISA gather with DIRECTION src at Reddit scale: y[j] = sum over the edges whose source is j
of x[dst(e)] (a gather C of a scatter R, the transposed aggregate), F = 128 fp32, over the CSC
"dst" view (gta_csc_build): the row-chunked kernel (512-edge plan) against the column-blocked one
(B = auto, ~6 MB slices of x), as the executor picks them (_spmm).  HIP events, interleaved
rounds; the two outputs compared at the per-element bound's scale (different fold orders).

Usage: python scripts/gather_c_probe.py [--rounds R] [--reps K]"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, ops  # noqa: E402


def main():
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 5
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 10
    dev = torch.device("cuda", 0)
    g = G.dataset_graph("reddit", device=dev)
    t0 = time.perf_counter()
    c = ops.csc(g)
    torch.cuda.synchronize()
    csc_s = time.perf_counter() - t0
    view = c.view("dst")
    x = torch.randn(g.n_rows, 128, device=dev)
    B = ops.BlockedPlan.auto_blocks(view, 128)
    forms = {"row_chunked": lambda: ops.aggregate(view, x, "src", None, plan=512),
             f"blocked_B{B}": lambda: ops.aggregate_blocked(view, x, None, blocks=B)}
    stream = torch.cuda.current_stream(dev)
    times = {k: [] for k in forms}
    outs = {}
    for r in range(rounds):
        for k, fn in forms.items():
            outs[k] = fn().clone()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for a, b in ev:
                a.record(stream)
                fn()
                b.record(stream)
            torch.cuda.synchronize()
            times[k].append(float(np.median([a.elapsed_time(b) for a, b in ev])))
        print(json.dumps({"round": r, "ms": {k: round(v[-1], 4) for k, v in times.items()}}), flush=True)
    a, b = list(outs.values())
    print(json.dumps({"N": g.n_rows, "E": g.nnz, "csc_build_s_first_call": round(csc_s, 3),
                      "ms": {k: round(float(np.median(v)), 4) for k, v in times.items()},
                      "G_edges_per_s": {k: round(g.nnz / float(np.median(v)) / 1e6, 2) for k, v in times.items()},
                      "max_abs_diff_between_forms": float((a - b).abs().max()),
                      "max_abs_out": float(a.abs().max())}), flush=True)


if __name__ == "__main__":
    main()
