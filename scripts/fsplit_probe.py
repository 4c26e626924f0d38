"""Probe: the metric aggregate as two launches over feature halves (x[:, :64] / x[:, 64:], alpha heads
0-3 / 4-7), so each launch's X slice footprint is half (3 MB at B = 20) -- does the better L2 hit rate
pay for reading the indices twice?  Prints median ms per variant; checks the halves equal the
one-launch result to fp32 rounding."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g, x, alpha = bench.make_inputs(bench.N_REDDIT, bench.E_REDDIT, dev)
    a_lo, a_hi = alpha[:, :4].contiguous(), alpha[:, 4:].contiguous()
    y = torch.empty(g.n_rows, 128, device=dev)
    y2 = torch.empty(g.n_rows, 128, device=dev)
    variants = {}
    for B in (20, 32, 40):
        plan = g.blocked_plan(B)
        variants[f"B{B} one launch F=128"] = lambda plan=plan, B=B: ops.aggregate_blocked(g, x, alpha, out=y, plan=plan, blocks=B)
        variants[f"B{B} halves, strided alpha"] = lambda plan=plan, B=B: (
            ops.aggregate_blocked(g, x[:, :64], alpha[:, :4], out=y2[:, :64], plan=plan, blocks=B),
            ops.aggregate_blocked(g, x[:, 64:], alpha[:, 4:], out=y2[:, 64:], plan=plan, blocks=B))
        variants[f"B{B} halves, split alpha"] = lambda plan=plan, B=B: (
            ops.aggregate_blocked(g, x[:, :64], a_lo, out=y2[:, :64], plan=plan, blocks=B),
            ops.aggregate_blocked(g, x[:, 64:], a_hi, out=y2[:, 64:], plan=plan, blocks=B))
    times = {k: [] for k in variants}
    for r in range(5):
        for k, fn in variants.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(3):
                fn()
            e1.record()
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / 3)
    for k in variants:
        print(f"{k:32s} median {np.median(times[k]):7.3f} ms", flush=True)
    d = float((y - y2).abs().max())
    print("max |one launch - halves| =", d, flush=True)


if __name__ == "__main__":
    main()
