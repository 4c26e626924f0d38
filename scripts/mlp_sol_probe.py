"""What the GIN products fused MLP's traffic costs when nothing else is done: the same bytes moved by
plain streaming kernels, beside `gta_update_mlp` on the layer's exact input (the aggregate's bf16 sum
[2,449,029 x 100] at its 104-element pitch, bf16 W1 [100 x 128] / W2 [128 x 128], RELU / RELU, fp32
out [2,449,029 x 128]).
  write   out.fill_(0)                       1.25 GB written
  read    x_pitched.view(int32).sum over rows (int64 accumulate, one pass) 0.51 GB read
  copy    out2.copy_(out)                    1.25 GB read + 1.25 GB written
  mlp     gta_update_mlp                     0.51 GB read + 1.25 GB written
HIP events, interleaved rounds, median.

Usage: python scripts/mlp_sol_probe.py [--rounds R] [--reps K]"""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops  # noqa: E402


def main():
    argv = sys.argv
    rounds = int(argv[argv.index("--rounds") + 1]) if "--rounds" in argv else 5
    reps = int(argv[argv.index("--reps") + 1]) if "--reps" in argv else 20
    dev = torch.device("cuda", 0)
    M, K1, N = 2449029, 100, 128
    g = torch.Generator(device="cpu").manual_seed(7)
    xs = torch.empty(M, 104, dtype=torch.bfloat16, device=dev)
    x = xs[:, :K1]
    x.copy_(torch.randn(M, K1, generator=g).to(torch.bfloat16).to(dev))
    w1 = (torch.randn(K1, N, generator=g) / K1 ** 0.5).to(torch.bfloat16).to(dev)
    w2 = (torch.randn(N, N, generator=g) / N ** 0.5).to(torch.bfloat16).to(dev)
    out = torch.empty(M, N, device=dev)
    out2 = torch.empty(M, N, device=dev)
    xi = xs.view(torch.int32)
    red = torch.empty(52, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream(dev)
    forms = {
        "write": (lambda: out2.fill_(0.0), M * N * 4),
        "read": (lambda: torch.sum(xi, dim=0, dtype=torch.int64, out=red), M * 104 * 2),
        "copy": (lambda: out2.copy_(out), 2 * M * N * 4),
        "mlp": (lambda: ops.update_mlp(x, w1, w2, sf1="RELU", sf2="RELU", out=out), M * (104 * 2 + N * 4)),
    }
    times = {k: [] for k in forms}
    for r in range(rounds):
        for k, (fn, _) in forms.items():
            fn()
            ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
            for a, b in ev:
                a.record(stream)
                fn()
                b.record(stream)
            torch.cuda.synchronize()
            times[k].append(float(np.median([a.elapsed_time(b) for a, b in ev])))
        print(json.dumps({"round": r, "ms": {k: round(t[-1], 4) for k, t in times.items()}}), flush=True)
    for k, (_, byt) in forms.items():
        ms = float(np.median(times[k]))
        print(json.dumps({"form": k, "ms": round(ms, 4), "GB": round(byt / 1e9, 3), "TBps": round(byt / ms / 1e9, 3)}),
              flush=True)


if __name__ == "__main__":
    main()
