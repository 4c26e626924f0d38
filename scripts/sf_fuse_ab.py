"""A/B of the attention-gather + SF fusion on a whole layer, interleaved in one process:
executor._attention_with_sf on (default) vs off; median ms per forward of each."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import configs, executor  # noqa: E402


def main(name="gat8-reddit", rounds=5, reps=10):
    dev = torch.device("cuda:0")
    layers, g, tensors = configs.build(name, dev)
    orig = executor.Executor._attention_with_sf
    res = {"on": [], "off": []}
    for r in range(rounds):
        for arm in ("on", "off"):
            executor.Executor._attention_with_sf = orig if arm == "on" else (lambda self, op, block: None)
            executor.clear_auto_graphs()
            for lay, t in zip(layers, tensors):
                lay.run(t, sync=True)  # warm-up (and the capture of the arm's graph)
                lay.run(t, sync=True)
            times = []
            for _ in range(reps):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for lay, t in zip(layers, tensors):
                    lay.run(t, sync=False)
                torch.cuda.synchronize()
                times.append(time.perf_counter() - t0)
            res[arm].append(1e3 * sorted(times)[reps // 2])
    executor.Executor._attention_with_sf = orig
    print(name, {k: [round(v, 4) for v in vs] for k, vs in res.items()}, flush=True)


if __name__ == "__main__":
    for n in (sys.argv[1:] or ["gat8-reddit", "gat8-flickr"]):
        main(n)
