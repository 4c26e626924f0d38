"""A/B of the model input's row pitch on whole BASELINE layers: x on line-pitched storage (what
workloads.make_tensors now builds, ops.line_pitch) against the same values contiguous (pitch = F).
Interleaved rounds, one synchronisation per forward, median of reps; the layer outputs of the two
layouts are compared bitwise (the pitch changes addresses, not the per-lane sum order).

Usage: python scripts/pitch_layers_ab.py [config ...] [--rounds R] [--reps K]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import configs  # noqa: E402


def forward(layers, tensors):
    x = None
    for lay, t in zip(layers, tensors):
        if x is not None:
            t["x"] = x
        res, _ = lay.run(t, sync=False)
        x = res.outputs[sorted(res.outputs)[-1]]
    return x


def main():
    argv = sys.argv[1:]
    rounds = int(argv[argv.index("--rounds") + 1]) if "--rounds" in argv else 5
    reps = int(argv[argv.index("--reps") + 1]) if "--reps" in argv else 5
    names = [a for i, a in enumerate(argv) if not a.startswith("--") and (i == 0 or argv[i - 1] not in ("--rounds", "--reps"))]
    dev = torch.device("cuda:0")
    for name in names or ["gin-products", "sage-reddit", "gat8-reddit", "gat8-flickr"]:
        layers, g, tensors = configs.build(name, dev)
        x = tensors[0]["x"]
        flat = x.contiguous()
        t_flat = [dict(t) for t in tensors]
        for k, v in tensors[0].items():
            if v is x:
                t_flat[0][k] = flat
        forms = {"pitched": tensors, "contiguous": t_flat}
        times = {k: [] for k in forms}
        outs = {}
        for r in range(rounds):
            for k, ts in forms.items():
                outs[k] = forward(layers, ts).clone()  # warm-up (graph capture) + the kept output
                tt = []
                for _ in range(reps):
                    torch.cuda.synchronize()
                    t1 = time.perf_counter()
                    forward(layers, ts)
                    torch.cuda.synchronize()
                    tt.append(time.perf_counter() - t1)
                times[k].append(1e3 * sorted(tt)[len(tt) // 2])
        rec = {"config": name, "F": x.shape[1], "dtype": str(x.dtype), "pitch": x.stride(0),
               "ms": {k: round(sorted(v)[len(v) // 2], 4) for k, v in times.items()},
               "all": {k: [round(t, 4) for t in v] for k, v in times.items()},
               "bitwise_equal": bool(torch.equal(outs["pitched"], outs["contiguous"]))}
        print(json.dumps(rec), flush=True)
        del layers, g, tensors, forms, t_flat, x, flat, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
