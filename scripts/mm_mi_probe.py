"""Row-streaming GEMM (k_mm_rows) with 2 vs 4 16-row fragments per wave (knob mm_rows_mi) on the
layer shapes; results must be bitwise equal (same k order per output)."""
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
    out = {}
    for M, K, N, dt in [(232965, 602, 128, None), (232965, 602, 256, None), (89250, 500, 128, None),
                        (89250, 64, 128, None), (2449029, 100, 128, torch.bfloat16), (2449029, 128, 128, torch.bfloat16),
                        (232965, 128, 16, None)]:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(K, N, device=dev) * K ** -0.5
        if dt is not None:
            w = w.to(dt)
        rec, ys = {}, {}
        for mi in (2, 4):
            ops.set_debug("mm_rows_mi", mi)
            ys[mi] = ops.update_mm(x, w).clone()
            ms = timed(lambda: ops.update_mm(x, w))
            rec[f"mi{mi}_ms"] = ms
            rec[f"mi{mi}_TF"] = 2 * M * K * N / ms / 1e9
        ops.set_debug("mm_rows_mi", 2)
        rec["bitwise_equal"] = bool(torch.equal(ys[2], ys[4]))
        key = f"M={M} K={K} N={N} {'bf16 W' if dt is not None else 'fp32'}"
        out[key] = rec
        print(key, json.dumps(rec), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "mm_mi_probe.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
