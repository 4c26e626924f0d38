"""Per-rank compute of 2-D edge-tile grids (pr row groups x pc column groups), rank (0, 0)'s
tile timed alone on one GPU, one launch per variant (profiles/r01_shard_probe_2d.json)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed, ops  # noqa: E402

dev = torch.device("cuda:0")
g, x, alpha = bench.make_inputs(bench.N_REDDIT, bench.E_REDDIT, dev)


def shard2d(pr, pc, i, j):
    s = distributed.GridShard(g, i * pc + j, pr, pc)
    return s.graph, x[s.c0:s.c1].contiguous(), alpha[s.edge_ids].contiguous()


def t(fn):
    fn(); torch.cuda.synchronize(); ts=[]
    for _ in range(5):
        a,b=torch.cuda.Event(enable_timing=True),torch.cuda.Event(enable_timing=True)
        a.record(); fn(); b.record(); torch.cuda.synchronize(); ts.append(a.elapsed_time(b))
    return float(np.median(ts))
out = {}
for pr, pc in [(1, 2), (2, 1), (2, 2), (4, 1), (1, 8), (2, 4), (4, 2), (8, 1)]:
    gg, xl, wl = shard2d(pr, pc, 0, 0)
    y = torch.empty(gg.n_rows, bench.F, device=dev)
    res = {"rows": gg.n_rows, "edges": gg.nnz, "table_MB": xl.numel() * 4 / 1e6}
    res["plan512"] = t(lambda: ops.aggregate(gg, xl, "src", wl, out=y, plan=512))
    for B in (4, 8, 16):
        res[f"blk{B}"] = t(lambda: ops.aggregate_blocked(gg, xl, wl, out=y, blocks=B))
    out[f"{pr}x{pc}"] = res
    print(f"{pr}x{pc}", json.dumps(res), flush=True)
    del gg, xl, wl, y; torch.cuda.empty_cache()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", "probe2d.json"), "w"), indent=1)
