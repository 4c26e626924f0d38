"""k_mm_rows on GIN's first UPDATE shape (fp32 x [2.45M, 100] x bf16 W [100, 128]) with x rows at
their natural 400-B pitch vs a 512-B (line-aligned) pitch: isolates the cost of A fragments that
straddle 128-B lines."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops  # noqa: E402


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            fn()
        b.record()
        torch.cuda.synchronize()
        t.append(a.elapsed_time(b) / reps)
    return float(np.median(t))


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    M, K, N = 2449029, 100, 128
    w = (torch.randn(K, N, device=dev) * K ** -0.5).to(torch.bfloat16)
    out = {}
    for pitch in (100, 104, 128):
        base = torch.randn(M, pitch, device=dev)
        x = base[:, :K]
        ms = timed(lambda: ops.update_mm(x, w, sf="RELU"))
        out[f"pitch {pitch * 4} B"] = ms
        print(f"pitch {pitch * 4} B: {ms:.3f} ms", flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(out, open(os.path.join(ROOT, "gpurun_out", "mm_ld_probe.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
