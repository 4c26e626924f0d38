"""A/B of GIN products' aggregate: bf16 200-B rows in 8-B pieces (25 lanes, two
edges per wave instruction) against 16-B pieces (13 lanes, four edges per wave instruction, knob
agg_bf16_vw8), on the layer's launch shape without its [E, 1] edge operand (gta_aggregate_self:
(1 + eps) x formed in the epilogue, 512-edge plan, bf16 y for the fused MLP; scripts/gin_ld_ab.py
times the weighted launch the layer makes), interleaved rounds, HIP events on the launch stream.  Prints one JSON line per form (median ms, G edges/s) and the max |d| between the forms.

Usage: python scripts/gin_vw8_ab.py [--rounds R] [--reps K] [--ur N]"""
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
    s = torch.tensor([[1.1]], device=dev)
    stream = torch.cuda.current_stream(dev)

    def run():
        return ops.aggregate(g, x, "src", None, plan=512, self_term=(x, s), out_dtype=torch.bfloat16)

    forms = {"8B_pieces": 0, "16B_pieces_ur4": 4, "16B_pieces_ur8": 8}
    times = {k: [] for k in forms}
    outs = {}
    for r in range(rounds):
        for name, v in forms.items():
            ops.set_debug("agg_bf16_vw8", v)
            try:
                outs[name] = run().clone()  # warm-up + the output kept for the comparison
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
                for a, b in ev:
                    a.record(stream)
                    run()
                    b.record(stream)
                torch.cuda.synchronize()
                times[name].append(float(np.median([a.elapsed_time(b) for a, b in ev])))
            finally:
                ops.set_debug("agg_bf16_vw8", 4)
    d = max((outs["8B_pieces"].float() - outs[k].float()).abs().max().item() for k in outs)
    for name in forms:
        ms = float(np.median(times[name]))
        print(json.dumps({"form": name, "ms": round(ms, 4), "all": [round(t, 4) for t in times[name]],
                          "G_edges_per_s": round(g.nnz / ms / 1e6, 2), "n": g.n_rows, "e": g.nnz}), flush=True)
    print(json.dumps({"max_abs_diff_between_forms": d}))


if __name__ == "__main__":
    main()
