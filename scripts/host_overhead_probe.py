"""Host cost of one replayed layer call (GCN Cora, 2 layers: launch-bound): per-forward wall time of
(a) the captured graphs' replay() alone, (b) executor.run_stream with the caller's same tensors
dict (the fast cache key), (c) run_stream with a fresh dict per call (what distributed.layer_record
and pipeline callers do), each over many forwards with one synchronisation at the end.

Usage: python scripts/host_overhead_probe.py [config] [--iters N]"""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import configs, executor  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    iters = int(sys.argv[sys.argv.index("--iters") + 1]) if "--iters" in sys.argv else 200
    name = args[0] if args and args[0] != str(iters) else "gcn-cora"
    dev = torch.device("cuda", 0)
    layers, g, tensors = configs.build(name, dev)

    def forward(fresh):
        x = None
        for lay, t in zip(layers, tensors):
            if fresh:
                t = dict(t)
            if x is not None:
                t["x"] = x
            res, _ = executor.run_stream(lay.opgraph, lay.stream, g, t, lay.sem, sync=False)
            x = res.outputs[sorted(res.outputs)[-1]]
        return x

    for _ in range(4):  # capture every layer's graph (second call) and settle the inputs
        forward(False)
    torch.cuda.synchronize()
    out = {"config": name, "iters": iters}
    for label, fn in (("run_stream_same_dict", lambda: forward(False)), ("run_stream_fresh_dict", lambda: forward(True))):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        out[label + "_us"] = round(1e6 * (time.perf_counter() - t0) / iters, 2)
    runs = [e.run for e in executor._AUTO.values() if e.run is not None]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        for r in runs[-len(layers):]:
            r.replay()
    torch.cuda.synchronize()
    out["replay_only_us"] = round(1e6 * (time.perf_counter() - t0) / iters, 2)
    t0 = time.perf_counter()
    for _ in range(iters):
        forward(True)
        torch.cuda.synchronize()
    out["fresh_dict_synced_us"] = round(1e6 * (time.perf_counter() - t0) / iters, 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
