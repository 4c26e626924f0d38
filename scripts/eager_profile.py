"""cProfile of repeated eager forwards of a small config (host-side overhead of the executor path)."""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import configs  # noqa: E402


def main(name="gcn-cora", reps=200):
    dev = torch.device("cuda:0")
    layers, g, tensors = configs.build(name, dev)

    def fwd():
        x = None
        for lay, t in zip(layers, tensors):
            if x is not None:
                t["x"] = x
            res, _ = lay.run(t)
            x = res.outputs[sorted(res.outputs)[-1]]
    for _ in range(5):
        fwd()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fwd()
    torch.cuda.synchronize()
    print(f"{name}: {1e3 * (time.perf_counter() - t0) / reps:.3f} ms per eager forward", flush=True)
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(reps):
        fwd()
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["gcn-cora"]))
