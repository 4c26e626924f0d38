"""GIN MLP timing: the fused gta_update_mlp against the two unfused mixed UPDATEs it replaces, on
the ogbn-products shape ([2,449,029 x 100] . [100 x 128] -> relu -> . [128 x 128] -> relu), HIP-event
medians of back-to-back launches; bytes = x read + out written (fused) or + the [M, 128] fp32
intermediate written and read (unfused).  Prints one JSON line per (M, K1) shape."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops  # noqa: E402


def timed(fn, reps=20):
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for _ in range(3):
        fn()
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev]))


def main():
    dev = torch.device("cuda", 0)
    for M, K1, N1, N2 in ((2449029, 100, 128, 128), (2449029, 128, 128, 128), (232965, 128, 128, 128)):
        g = torch.Generator(device="cpu").manual_seed(M + K1)
        x = torch.randn(M, K1, generator=g).to(dev)
        w1 = (torch.randn(K1, N1, generator=g) / K1 ** 0.5).to(torch.bfloat16).to(dev)
        w2 = (torch.randn(N1, N2, generator=g) / N1 ** 0.5).to(torch.bfloat16).to(dev)
        out = torch.empty(M, N2, device=dev)
        z = torch.empty(M, N1, device=dev)
        fused = timed(lambda: ops.update_mlp(x, w1, w2, sf1="RELU", sf2="RELU", out=out))
        y1 = out.clone()
        unf = timed(lambda: (ops.update_mm(x, w1, sf="RELU", out=z), ops.update_mm(z, w2, sf="RELU", out=out)))
        torch.cuda.synchronize()
        byt = M * (K1 + N2) * 4
        print(json.dumps({"M": M, "K1": K1, "N1": N1, "N2": N2, "fused_ms": round(fused, 4), "unfused_ms": round(unf, 4),
                          "fused_TBps": round(byt / fused / 1e9, 3), "unfused_TBps_incl_z": round((byt + 2 * M * N1 * 4) / unf / 1e9, 3),
                          "bitwise": bool(torch.equal(y1, out))}), flush=True)
        del x, w1, w2, out, z, y1
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
