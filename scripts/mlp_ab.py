"""A/B of one libgta knob on GIN products' fused MLP (gta_update_mlp on the layer's exact input: the
aggregate's bf16 sum [2,449,029 x 100] at its 104-element pitch, bf16 W1 [100 x 128], W2 [128 x 128],
RELU / RELU, fp32 out).  Interleaved rounds, HIP events on the launch stream, outputs compared
bitwise across the knob values.

Usage: python scripts/mlp_ab.py --knob NAME --values A,B[,...] [--rounds R] [--reps K]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops  # noqa: E402


def main():
    argv = sys.argv
    knob = argv[argv.index("--knob") + 1]
    values = [int(v) for v in argv[argv.index("--values") + 1].split(",")]
    rounds = int(argv[argv.index("--rounds") + 1]) if "--rounds" in argv else 5
    reps = int(argv[argv.index("--reps") + 1]) if "--reps" in argv else 20
    dev = torch.device("cuda", 0)
    M, K1, N = 2449029, 100, 128
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.empty(M, 104, dtype=torch.bfloat16, device=dev)[:, :K1]
    x.copy_(torch.randn(M, K1, generator=g).to(torch.bfloat16).to(dev))
    w1 = (torch.randn(K1, N, generator=g) / K1 ** 0.5).to(torch.bfloat16).to(dev)
    w2 = (torch.randn(N, N, generator=g) / N ** 0.5).to(torch.bfloat16).to(dev)
    out = torch.empty(M, N, device=dev)
    stream = torch.cuda.current_stream(dev)
    default = ops.get_debug(knob)
    times = {v: [] for v in values}
    outs = {}
    for r in range(rounds):
        for v in values:
            ops.set_debug(knob, v)
            try:
                ops.update_mlp(x, w1, w2, sf1="RELU", sf2="RELU", out=out)
                outs[v] = out.clone()
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
                for a, b in ev:
                    a.record(stream)
                    ops.update_mlp(x, w1, w2, sf1="RELU", sf2="RELU", out=out)
                    b.record(stream)
                torch.cuda.synchronize()
                times[v].append(float(np.median([a.elapsed_time(b) for a, b in ev])))
            finally:
                ops.set_debug(knob, default)
        print(json.dumps({"round": r, "ms": {str(v): round(t[-1], 4) for v, t in times.items()}}), flush=True)
    byt = M * (104 * 2 + N * 4)
    for v in values:
        ms = float(np.median(times[v]))
        print(json.dumps({knob: v, "ms": round(ms, 4), "TBps": round(byt / ms / 1e9, 3)}), flush=True)
    print(json.dumps({"bitwise_equal": all(torch.equal(outs[values[0]], outs[v]) for v in values)}))


if __name__ == "__main__":
    main()
