"""fp32 UPDATE forms on the layer shapes, interleaved in one process: k_mm_ring (LDS-DMA ring),
k_mm_rows (register-staged A, synchronous W chunks) and the tuned hipBLASLt path inside libgta.
Prints ms and TFLOP/s per form (fp32 MFMA peak 157.3 TF/s) and writes gpurun_out/mm_ab.json."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops  # noqa: E402

FORMS = {"ring": {"mm_blaslt": 0, "mm_ring": 1, "mm_ring_form": 0, "mm_ring_a16u": 0},
         "ring_d2": {"mm_blaslt": 0, "mm_ring": 1, "mm_ring_form": 3},
         "ring_a16u": {"mm_blaslt": 0, "mm_ring": 1, "mm_ring_form": 0, "mm_ring_a16u": 1},
         "rows": {"mm_blaslt": 0, "mm_ring": 0},
         "hipblaslt": {"mm_blaslt": 1, "mm_ring": 0, "mm_blaslt_tune": 1, "mm_blaslt_max_m": 1 << 62},
         "hipblaslt_top1": {"mm_blaslt": 1, "mm_ring": 0, "mm_blaslt_tune": 0, "mm_blaslt_max_m": 1 << 62}}
DEFAULTS = {"mm_blaslt": 1, "mm_ring": 1, "mm_blaslt_tune": 0, "mm_ring_form": 0, "mm_ring_prio": 0,
            "mm_ring_a16u": 1, "mm_blaslt_max_m": 65535}


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    shapes = [(232965, 602, 128), (232965, 602, 256), (89250, 500, 128), (2449029, 100, 128),
              (2449029, 128, 128), (232965, 128, 128)]
    if len(sys.argv) > 1:
        shapes = [tuple(int(v) for v in s.split("x")) for s in sys.argv[1:]]
    old_min = ops.MM_ROWS_MIN_M
    ops.MM_ROWS_MIN_M = 0
    out = {}
    try:
        for M, K, N in shapes:
            x = torch.randn(M, K, device=dev)
            w = torch.randn(K, N, device=dev) * K ** -0.5
            y = {}
            t = {f: [] for f in FORMS}
            for r in range(7):
                for f, knobs in FORMS.items():
                    for k, v in DEFAULTS.items():
                        ops.set_debug(k, v)
                    for k, v in knobs.items():
                        ops.set_debug(k, v)
                    if r == 0:
                        y[f] = ops.update_mm(x, w).clone()
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record()
                    for _ in range(5):
                        ops.update_mm(x, w)
                    b.record()
                    torch.cuda.synchronize()
                    t[f].append(a.elapsed_time(b) / 5)
            rec = {}
            for f in FORMS:
                ms = float(np.median(t[f]))
                rec[f] = {"ms": ms, "TF": 2 * M * K * N / ms / 1e9}
            rec["ring_eq_rows_bitwise"] = bool(all(torch.equal(y[f], y["rows"]) for f in FORMS if f.startswith("ring")))
            rec["ring_vs_blaslt_max_abs"] = float((y["ring"] - y["hipblaslt"]).abs().max())
            out[f"M={M} K={K} N={N}"] = rec
            print(f"M={M} K={K} N={N} " + "  ".join(f"{f} {rec[f]['ms']:.3f} ms {rec[f]['TF']:.1f} TF"
                                                    for f in FORMS) + f"  bitwise(ring,rows)={rec['ring_eq_rows_bitwise']}",
                  flush=True)
            del x, w, y
            torch.cuda.empty_cache()
    finally:
        for k, v in DEFAULTS.items():
            ops.set_debug(k, v)
        ops.MM_ROWS_MIN_M = old_min
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "mm_ab.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
