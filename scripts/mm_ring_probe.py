"""k_mm_ring diagnostic: TF/s of the default ring form across K (tail / no tail), M (x resident in the
Infinity Cache or not) and persistent blocks per CU, hipBLASLt's first choice beside it.
Writes gpurun_out/mm_ring_probe.json."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops  # noqa: E402

CASES = [(232965, 602, 128), (232965, 602, 256), (89250, 500, 128), (65536, 602, 128), (16384, 602, 128),
         (232965, 128, 128), (232965, 256, 128), (2449029, 100, 128), (2449029, 128, 128), (899756, 500, 128)]
FORMS = {"ring": {"mm_blaslt": 0}, "ring_tail": {"mm_blaslt": 0, "mm_ring_tail": 1},
         "ring_fr2": {"mm_blaslt": 0, "mm_ring_fr": 2},
         "ring_fr1": {"mm_blaslt": 0, "mm_ring_fr": 1},
         "ring_bpc2": {"mm_blaslt": 0, "mm_ring_blocks_per_cu": 2},
         "ring_bpc1": {"mm_blaslt": 0, "mm_ring_blocks_per_cu": 1}, "blaslt_top1": {"mm_blaslt": 1, "mm_blaslt_max_m": 1 << 62}}


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    ops.MM_ROWS_MIN_M = 0
    out = {}
    for M, K, N in CASES:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(K, N, device=dev) * K ** -0.5
        t = {f: [] for f in FORMS}
        for r in range(5):
            for f, knobs in FORMS.items():
                ops.set_debug("mm_blaslt", 1)
                ops.set_debug("mm_blaslt_max_m", 65535)
                ops.set_debug("mm_ring_blocks_per_cu", 0)
                ops.set_debug("mm_ring_fr", 0)
                ops.set_debug("mm_ring_tail", 0)
                for k, v in knobs.items():
                    ops.set_debug(k, v)
                ops.update_mm(x, w)
                a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                a.record()
                for _ in range(10):
                    ops.update_mm(x, w)
                b.record()
                torch.cuda.synchronize()
                t[f].append(a.elapsed_time(b) / 10)
        rec = {f: {"ms": float(np.median(v)), "TF": 2 * M * K * N / float(np.median(v)) / 1e9} for f, v in t.items()}
        out[f"{M}x{K}x{N}"] = rec
        print(f"M={M} K={K} N={N} " + "  ".join(f"{f} {r['ms']:.3f} ms {r['TF']:.1f} TF" for f, r in rec.items()),
              flush=True)
    ops.set_debug("mm_blaslt", 1)
    ops.set_debug("mm_blaslt_max_m", 65535)
    ops.set_debug("mm_ring_blocks_per_cu", 0)
    ops.set_debug("mm_ring_fr", 0)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "mm_ring_probe.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
