"""What GraphSAGE Reddit's one weight per edge costs in the column-blocked aggregate: the same
launch pair (k_agg_h32 + k_seg_reduce, B = 20) over the Reddit-shaped graph's 128-wide table
unweighted, with the [E, 1] weight (the lean w1 form: 32 weights per load beside the indices,
broadcast), and with 8 head weights [E, 8] (the metric's form).  HIP events, interleaved rounds.

Usage: python scripts/sage_w1_probe.py [--rounds R] [--reps K]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, ops  # noqa: E402


def pmc_child():
    """Under rocprofv3 --pmc (scripts/pmc_sq.py PMC_TARGET=wcost): each form's launch pair 4 times."""
    dev = torch.device("cuda", 0)
    g = G.dataset_graph("reddit", device=dev)
    x = torch.randn(g.n_rows, 128, device=dev)
    for w in (None, torch.rand(g.nnz, 1, device=dev) + 0.5, torch.rand(g.nnz, 8, device=dev) + 0.5):
        for _ in range(4):
            ops.aggregate_blocked(g, x, w, blocks=20)
        torch.cuda.synchronize()
    return 0


def main():
    if "--pmc-child" in sys.argv:
        return pmc_child()
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 5
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 10
    dev = torch.device("cuda", 0)
    g = G.dataset_graph("reddit", device=dev)
    x = torch.randn(g.n_rows, 128, device=dev)
    w1 = torch.rand(g.nnz, 1, device=dev) + 0.5
    w8 = torch.rand(g.nnz, 8, device=dev) + 0.5
    forms = {"unweighted": None, "w1": w1, "heads8": w8}
    stream = torch.cuda.current_stream(dev)
    times = {k: [] for k in forms}
    for r in range(rounds):
        for k, w in forms.items():
            ops.aggregate_blocked(g, x, w, blocks=20)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for a, b in ev:
                a.record(stream)
                ops.aggregate_blocked(g, x, w, blocks=20)
                b.record(stream)
            torch.cuda.synchronize()
            times[k].append(float(np.median([a.elapsed_time(b) for a, b in ev])))
        print(json.dumps({"round": r, "ms": {k: round(v[-1], 4) for k, v in times.items()}}), flush=True)
    print(json.dumps({"ms": {k: round(float(np.median(v)), 4) for k, v in times.items()}}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
