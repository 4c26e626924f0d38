"""UPDATE GEMM timing on the layer shapes (all hand-written: k_mm_ring / k_mm_rows + split-K).

For each (M, K, N, dtype): median of HIP-graph replays of one update_mm call (the launch gaps a
layer's graph sees), and the kernel-only time from HIP events over back-to-back eager calls.
Prints one JSON line per shape: ms, TF/s, GB/s (x + W read once, out written once).
Usage: python scripts/mm_probe.py [--shapes cora|mid|big|gin|all] [--knob k=v ...]
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops  # noqa: E402

SHAPES = {
    "cora": [(2708, 1433, 128, "f32"), (2708, 128, 64, "f32")],
    "cora_x": [(2708, 1433, 128, "f32"), (2708, 1432, 128, "f32")],
    "short_k": [(16384, 144, 128, "f32"), (16384, 137, 128, "f32"), (2816, 144, 128, "f32"), (2816, 1433, 128, "f32")],
    "k144": [(16384, 144, 128, "f32")],
    "big_one": [(232965, 602, 128, "f32")],
    "mid_one": [(16384, 1433, 128, "f32")],
    "mid": [(16384, 128, 128, "f32"), (29000, 602, 128, "f32"), (44625, 500, 128, "f32"), (29000, 602, 256, "f32"),
            (16384, 1433, 128, "f32"), (5000, 602, 128, "f32")],
    "big": [(232965, 602, 128, "f32"), (232965, 602, 256, "f32"), (89250, 500, 128, "f32"), (232965, 128, 128, "f32"),
            (899756, 500, 128, "f32")],
    "gin": [(2449029, 100, 128, "mixed"), (2449029, 128, 128, "mixed"), (2449029, 100, 128, "f32"),
            (2449029, 128, 128, "bf16")],
}


LDX = 0  # --ldx L: x is the first K columns of an [M, L] table (rows L * 4 B apart)


def one(M, K, N, dt, dev, reps=20):
    g = torch.Generator(device="cpu").manual_seed(M + K + N)
    x = torch.randn(M, max(K, LDX), generator=g).to(dev)[:, :K]
    w = (torch.randn(K, N, generator=g) / K ** 0.5).to(dev)
    if dt == "bf16":
        x, w = x.to(torch.bfloat16), w.to(torch.bfloat16)
    elif dt == "mixed":
        w = w.to(torch.bfloat16)
    out = torch.empty(M, N, device=dev)
    for _ in range(3):
        ops.update_mm(x, w, out=out)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(s)
        ops.update_mm(x, w, out=out)
        b.record(s)
    torch.cuda.synchronize()
    k_ms = sorted(a.elapsed_time(b) for a, b in ev)[reps // 2]
    # HIP-graph replay of the same call (W^T cached before the capture)
    gr = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(s)
    with torch.cuda.stream(side):
        ops.update_mm(x, w, out=out)
    s.wait_stream(side)
    torch.cuda.synchronize()
    per_graph = 10  # ten back-to-back calls per graph: the per-call cost inside a layer's graph
    with torch.cuda.graph(gr):
        for _ in range(per_graph):
            ops.update_mm(x, w, out=out)
    for _ in range(3):
        gr.replay()
    torch.cuda.synchronize()
    ev2 = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(5)]
    for a, b in ev2:
        a.record(s)
        gr.replay()
        b.record(s)
    torch.cuda.synchronize()
    g_ms = sorted(a.elapsed_time(b) for a, b in ev2)[2] / per_graph
    ref = (x.double() @ w.double()) if M <= 50000 else None
    err = None if ref is None else float((out.double() - ref).abs().max())
    flop = 2.0 * M * K * N
    byt = x.numel() * x.element_size() + w.numel() * w.element_size() + out.numel() * 4
    return {"M": M, "K": K, "N": N, "dtype": dt, "splits": ops._mm_splits(M, K, N, {"f32": 0, "bf16": 1, "mixed": 2}[dt]),
            "event_ms": round(k_ms, 4), "graph_call_ms": round(g_ms, 4), "TFps": round(flop / g_ms / 1e9, 1),
            "GBps": round(byt / g_ms / 1e6, 1), "max_abs_err_vs_fp64": err}


def main():
    dev = torch.device("cuda", 0)
    args = sys.argv[1:]
    which = "all"
    if "--ldx" in args:
        global LDX
        LDX = int(args[args.index("--ldx") + 1])
    if "--shapes" in args:
        which = args[args.index("--shapes") + 1]
    for i, a in enumerate(args):
        if "=" in a and not a.startswith("--") and (i == 0 or args[i - 1] not in ("--sweep", "--ldx")):
            k, v = a.split("=")
            ops.set_debug(k, int(v))
    names = list(SHAPES) if which == "all" else which.split(",")
    sweep = [None]
    if "--sweep" in args:  # knob=v1,v2,... : every shape at every value
        k, vals = args[args.index("--sweep") + 1].split("=")
        sweep = [(k, int(v)) for v in vals.split(",")]
    for nm in names:
        for shp in SHAPES[nm]:
            for kv in sweep:
                if kv:
                    ops.set_debug(*kv)
                rec = one(*shp, dev)
                if kv:
                    rec[kv[0]] = kv[1]
                print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
