"""Row-chunk plan size on GIN products' aggregate (the layer's weighted launch: bf16 rows at the 256-B
pitch, [E, 1] edge operand, bf16 y with the (1 + eps) x term): chunk = the longest item a row is cut
into (128 / 256 / 512 / 1024 edges; split rows are summed by the combine kernel in chunk order).
Interleaved rounds, HIP events over the aggregate + combine launches.

Usage: python scripts/gin_plan_probe.py [--rounds R] [--reps K]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import configs, ops  # noqa: E402


def main():
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 5
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 10
    dev = torch.device("cuda", 0)
    _, g, tensors = configs.build("gin-products", dev)
    x = tensors[0]["x"]
    w = next(v for k, v in tensors[0].items() if k.startswith("ext:") and tuple(v.shape) == (g.nnz, 1))
    s = torch.tensor([[1.1]], device=dev)
    stream = torch.cuda.current_stream(dev)
    chunks = [128, 256, 512, 1024]
    times = {c: [] for c in chunks}
    for r in range(rounds):
        for c in chunks:
            def run():
                return ops.aggregate(g, x, "src", w, plan=c, self_term=(x, s), out_dtype=torch.bfloat16)
            run()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for a, b in ev:
                a.record(stream)
                run()
                b.record(stream)
            torch.cuda.synchronize()
            times[c].append(float(np.median([a.elapsed_time(b) for a, b in ev])))
        print(json.dumps({"round": r, "ms": {str(c): round(times[c][-1], 4) for c in chunks}}), flush=True)
    deg = (g.indptr[1:] - g.indptr[:-1])
    print(json.dumps({"ms": {str(c): round(float(np.median(times[c])), 4) for c in chunks},
                      "max_degree": int(deg.max()), "rows_over_512": int((deg > 512).sum())}), flush=True)


if __name__ == "__main__":
    main()
