"""A/B of the fp32 UPDATE forms on the layer shapes, in one process: k_mm_ring (default) against
k_mm_wave (knob mm_wave, row fragments per wave mm_wave_fr = auto / 2 / 3 / 4), interleaved rounds,
HIP-event medians of back-to-back update_mm calls, every variant checked bitwise against the
ring's output.  "default" is what update_mm runs with no knob touched (the auto split and the
auto wave plan).  Prints one JSON line per (shape, variant).

Usage: python scripts/mm_wave_ab.py [--rounds R] [M,K,N ...]
"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops  # noqa: E402

SHAPES = [(232965, 602, 128), (29000, 602, 128), (44625, 500, 128), (899756, 500, 128), (89250, 500, 128),
          (232965, 128, 128), (16384, 1433, 128), (2708, 1433, 128), (232965, 602, 64), (29000, 602, 256)]
VARIANTS = [("ring", {"mm_wave": 0}), ("ring_auto_split", {"mm_wave": 0, "mm_split": -1}), ("default", {"mm_split": -1}),
            ("wave_auto", {"mm_wave": 2}), ("wave_fr2", {"mm_wave": 2, "mm_wave_fr": 2}),
            ("wave_fr3", {"mm_wave": 2, "mm_wave_fr": 3}), ("wave_fr4", {"mm_wave": 2, "mm_wave_fr": 4})]


def timed(fn, reps):
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    args = sys.argv[1:]
    rounds = 3
    if "--rounds" in args:
        i = args.index("--rounds")
        rounds = int(args[i + 1])
        del args[i:i + 2]
    shapes = [tuple(int(v) for v in a.split(",")) for a in args] or SHAPES
    dev = torch.device("cuda", 0)
    for M, K, N in shapes:
        g = torch.Generator(device="cpu").manual_seed(M + K + N)
        x = torch.randn(M, K, generator=g).to(dev)
        w = (torch.randn(K, N, generator=g) / K ** 0.5).to(dev)
        outs = {name: torch.empty(M, N, device=dev) for name, _ in VARIANTS}
        ms = {name: [] for name, _ in VARIANTS}
        for r in range(rounds):
            for name, knobs in VARIANTS:
                knobs = {"mm_split": 0, **knobs}
                old = {k: ops.get_debug(k) for k in knobs}
                try:
                    for k, v in knobs.items():
                        ops.set_debug(k, v)
                    run = lambda: ops.update_mm(x, w, out=outs[name])  # noqa: E731
                    run()
                    ms[name].append(timed(run, 10))
                finally:
                    for k, v in old.items():
                        ops.set_debug(k, v)
        torch.cuda.synchronize()
        for name, _ in VARIANTS:
            t = float(np.median(ms[name]))
            print(json.dumps({"M": M, "K": K, "N": N, "variant": name, "ms": round(t, 4),
                              "TFs": round(2 * M * K * N / t / 1e9, 1),
                              "bitwise_vs_ring": bool(torch.equal(outs[name], outs["ring"])),
                              "all_ms": [round(v, 4) for v in ms[name]]}), flush=True)
        del x, w, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
