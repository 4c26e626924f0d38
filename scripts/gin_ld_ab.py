"""Row-pitch A/B of GIN products' aggregate: the bf16 model input x [N, 100] stored with a row pitch
of 100 (200-B rows: 2.5 lines each), 104 (208 B: every row 16-B aligned) or 128 elements (256 B:
every row on its own pair of 128-B lines), with 8-B or 16-B gather pieces (knob agg_bf16_vw8 0 /
4 / 8) and the edge operand's weights loaded per lane and edge (agg_w1 = 0, the round-4 form) or
64 per load beside the indices (agg_w1 = 1).  The layer's exact launch (gta_aggregate_self with the
layer's [E, 1] edge operand, 512-edge plan, bf16 y) -- and the unweighted launch (--unweighted) --
in interleaved rounds, HIP events on the launch stream; outputs compared bitwise across pitches
(same per-lane order, so the pitch cannot change a sum).

Usage: python scripts/gin_ld_ab.py [--rounds R] [--reps K] [--unweighted]"""
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
    N, F = x.shape
    w = None
    if "--unweighted" not in sys.argv:  # the layer's edge operand (GIN op 1's external [E, 1] tensor)
        w = next(v for k, v in tensors[0].items() if k.startswith("ext:") and tuple(v.shape) == (g.nnz, 1))
    xs = {}
    for ld in (100, 104, 128):
        buf = torch.zeros(N, ld, dtype=x.dtype, device=dev)
        buf[:, :F] = x
        xs[ld] = buf[:, :F]
    s = torch.tensor([[1.1]], device=dev)
    stream = torch.cuda.current_stream(dev)
    forms = [(100, 0, 0), (100, 0, 1), (100, 4, 1), (104, 4, 1), (128, 0, 1), (128, 4, 1), (128, 8, 1)]
    names = {f: f"ld{f[0]}_vw{f[1]}_w1{f[2]}" for f in forms}
    times = {f: [] for f in forms}
    outs = {}
    for r in range(rounds):
        for f in forms:
            ld, v, w1 = f
            ops.set_debug("agg_bf16_vw8", v)
            ops.set_debug("agg_w1", w1)
            try:
                xv = xs[ld]

                def run():
                    return ops.aggregate(g, xv, "src", w, plan=512, self_term=(xv, s), out_dtype=torch.bfloat16)
                outs[f] = run().clone()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
                for a, b in ev:
                    a.record(stream)
                    run()
                    b.record(stream)
                torch.cuda.synchronize()
                times[f].append(float(np.median([a.elapsed_time(b) for a, b in ev])))
            finally:
                ops.set_debug("agg_bf16_vw8", 4)
                ops.set_debug("agg_w1", 1)
        print(json.dumps({"round": r, "ms": {names[f]: round(times[f][-1], 4) for f in forms}}), flush=True)
    print(json.dumps({"weighted": w is not None,
                      "bitwise_equal": {"ld100_vs_ld128_vw4": torch.equal(outs[(100, 4, 1)], outs[(128, 4, 1)]),
                                        "ld100_vs_ld104_vw4": torch.equal(outs[(100, 4, 1)], outs[(104, 4, 1)]),
                                        "w1_vs_per_lane_vw0": torch.equal(outs[(100, 0, 0)], outs[(100, 0, 1)])}}))
    for f in forms:
        ms = float(np.median(times[f]))
        print(json.dumps({"form": names[f], "ms": round(ms, 4), "G_edges_per_s": round(g.nnz / ms / 1e6, 2),
                          "n": N, "e": g.nnz}), flush=True)


if __name__ == "__main__":
    main()
