"""What the GIN products aggregate pays for per gathered row: the layer's launch form (bf16 rows,
16-B pieces, [E, 1] edge weights, 512-edge plan, fp32 y) on the products graph over bf16 tables of
several (row width F, row pitch) pairs, interleaved rounds, HIP events.  Separates bytes per row
(sectors) from line requests per row: 200 B at a 256-B pitch (the layer's table), 192 B at 192 B
(1.5 lines, 3 sectors), 192 B at 256 B, 128 B at 128 B (1 line), 256 B at 256 B (2 whole lines).

Usage: python scripts/gin_rowbytes_probe.py [--rounds R] [--reps K]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import configs, ops  # noqa: E402


def main():
    rounds = int(sys.argv[sys.argv.index("--rounds") + 1]) if "--rounds" in sys.argv else 4
    reps = int(sys.argv[sys.argv.index("--reps") + 1]) if "--reps" in sys.argv else 10
    dev = torch.device("cuda", 0)
    _, g, tensors = configs.build("gin-products", dev)
    w = next(v for k, v in tensors[0].items() if k.startswith("ext:") and tuple(v.shape) == (g.nnz, 1))
    N = g.n_rows
    del tensors
    shapes = [(100, 128), (96, 96), (96, 128), (64, 64), (128, 128), (100, 100)]
    tabs = {}
    gen = torch.Generator(device="cpu").manual_seed(3)
    for F, P in shapes:
        t = torch.zeros(N, P, dtype=torch.bfloat16, device=dev)
        t[:, :F] = torch.randn(N, F, generator=gen).to(torch.bfloat16).to(dev)
        tabs[(F, P)] = t[:, :F]
    stream = torch.cuda.current_stream(dev)
    times = {k: [] for k in shapes}
    for r in range(rounds):
        for k in shapes:
            x = tabs[k]
            ops.aggregate(g, x, "src", w, plan=512)
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for a, b in ev:
                a.record(stream)
                ops.aggregate(g, x, "src", w, plan=512)
                b.record(stream)
            torch.cuda.synchronize()
            times[k].append(float(np.median([a.elapsed_time(b) for a, b in ev])))
        print(json.dumps({"round": r, "ms": {f"F{F}_pitch{2 * P}B": round(times[(F, P)][-1], 4) for F, P in shapes}}),
              flush=True)
    for F, P in shapes:
        ms = float(np.median(times[(F, P)]))
        row, pitch = 2 * F, 2 * P
        lines = ops._lines_per_row(row, pitch)
        print(json.dumps({"F": F, "row_B": row, "pitch_B": pitch, "lines_per_row": lines, "ms": round(ms, 4),
                          "ns_per_edge": round(ms * 1e6 / g.nnz, 4)}), flush=True)


if __name__ == "__main__":
    main()
