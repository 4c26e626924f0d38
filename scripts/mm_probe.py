"""Row-streaming GEMM (k_mm_rows) on the layer shapes with the dword-store and the 16-B-store epilogue."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    for M, K, N, dt in [(89250, 64, 128, None), (89250, 500, 128, None), (232965, 602, 128, None),
                        (2449029, 100, 128, torch.bfloat16), (2449029, 128, 128, torch.bfloat16), (2708, 1433, 128, None)]:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(K, N, device=dev) * K ** -0.5
        if dt is not None:
            w = w.to(dt)
        res = {}
        for vs in (0, 1):
            ops.set_debug("mm_vstore", vs)
            ops.update_mm(x, w)
            t = []
            for _ in range(5):
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(10):
                    ops.update_mm(x, w)
                b.record()
                torch.cuda.synchronize()
                t.append(a.elapsed_time(b) / 10)
            res[vs] = float(np.median(t))
        ops.set_debug("mm_vstore", 1)
        print(f"M={M} K={K} N={N}: dword stores {res[0]:.3f} ms ({2 * M * K * N / res[0] / 1e9:.0f} TF), "
              f"16-B stores {res[1]:.3f} ms ({2 * M * K * N / res[1] / 1e9:.0f} TF)", flush=True)


if __name__ == "__main__":
    main()
