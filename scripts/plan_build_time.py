"""Time the column-blocked plan build (gta_aggregate_blocked_plan_build) on the Reddit-shaped graph."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g = G.synthetic(bench.N_REDDIT, bench.E_REDDIT, seed=0, device=dev)
    for B in (20, 20, 40):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        p = ops.BlockedPlan(g, B)
        torch.cuda.synchronize()
        print(f"B={B}: plan build {1e3 * (time.perf_counter() - t0):.2f} ms, {p.n_items} items", flush=True)


if __name__ == "__main__":
    main()
