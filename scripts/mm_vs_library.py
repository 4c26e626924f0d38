"""k_mm_rows (libgta UPDATE) against the vendor library GEMM (torch.mm -> hipBLASLt/rocBLAS, fp32)
on the layer shapes: the reference point for the fp32 MFMA kernel."""
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
    torch.backends.cuda.matmul.allow_tf32 = False
    out = {}
    for M, K, N in [(232965, 602, 128), (232965, 602, 256), (89250, 500, 128), (2708, 1433, 128)]:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(K, N, device=dev) * K ** -0.5
        ours = timed(lambda: ops.update_mm(x, w))
        lib = timed(lambda: torch.mm(x, w))
        d = float((ops.update_mm(x, w) - torch.mm(x, w)).abs().max())
        torch.backends.cuda.preferred_blas_library("cublas")  # rocBLAS on ROCm
        rb = timed(lambda: torch.mm(x, w))
        torch.backends.cuda.preferred_blas_library("cublaslt")  # hipBLASLt (the default)
        rec = {"libgta_ms": ours, "libgta_TF": 2 * M * K * N / ours / 1e9, "torch_mm_ms": lib,
               "torch_mm_TF": 2 * M * K * N / lib / 1e9, "rocblas_ms": rb, "rocblas_TF": 2 * M * K * N / rb / 1e9,
               "max_abs_diff": d}
        out[f"M={M} K={K} N={N}"] = rec
        print(f"M={M} K={K} N={N}", json.dumps(rec), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "mm_vs_library.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
