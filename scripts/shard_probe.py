"""Per-rank compute of the multi-GPU bench, measured on one GPU: rank 0's shard at p = 2, 4, 8
(bench.py's chunk-major reduce-scatter layout), every aggregate form, so the per-shard block
count can be chosen from data.  No collective runs here (that is the driver's 8-GPU job)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed, ops, partition  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    g, x, alpha = bench.make_inputs(bench.N_REDDIT, bench.E_REDDIT, dev)
    out = {}
    for p in (2, 4, 8):
        for rank in (0, p - 1):
            sh = distributed.DistShard(g, rank, p, chunks=8)
            gl = sh.graph
            xl = x[sh.c0:sh.c1].contiguous()
            wl = alpha[sh.edge_ids].contiguous()
            parts = []
            for k in range(sh.chunks):
                r0, r1 = sh.chunk_rows(k)
                parts.append((r0, r1, partition.sub_rows(gl, r0, r1)))
            y = torch.empty(gl.n_rows, bench.F, device=dev)
            variants = {"plan512": ("plan", 512), "rows": ("plan", 0)}
            for B in (2, 4, 8, 16):
                variants[f"blk{B}"] = ("blocked", B)
            res = {}
            for name, (impl, arg) in variants.items():
                def run():
                    for r0, r1, gg in parts:
                        if impl == "blocked":
                            ops.aggregate_blocked(gg, xl, wl, out=y[r0:r1], blocks=arg)
                        else:
                            ops.aggregate(gg, xl, "src", wl, out=y[r0:r1], plan=(gg.plan(arg) if arg else None))
                run()
                torch.cuda.synchronize()
                ts = []
                for _ in range(5):
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    run()
                    b.record()
                    torch.cuda.synchronize()
                    ts.append(a.elapsed_time(b))
                res[name] = float(np.median(ts))
            res["auto_blocks"] = ops.BlockedPlan.auto_blocks(gl, bench.F)
            res["shard_edges"] = gl.nnz
            out[f"p{p}_rank{rank}"] = res
            print(f"p={p} rank={rank}", json.dumps(res), flush=True)
            del parts, y, xl, wl, sh, gl
            torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "shard_probe.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
