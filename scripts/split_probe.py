"""Few-row fp32 UPDATE forms timed as HIP-graph replays (no Python launch cost in the number):
hipBLASLt (first choice), and the split-K entry with its slices on k_mm_ring or k_mm_rows for
several slice counts.  Outputs of the split forms are compared with the ring/rows pair bitwise.
Writes gpurun_out/split_probe.json."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import _lib, ops  # noqa: E402
from gta_graph_tensor_acclelrator_for_general_gnn_amd.ops import _L, _ptr, _rows, _stream, check  # noqa: E402


def split_call(x, wt, out, M, K, N, splits, ws, nb):
    check(_L().gta_update_mm_t_split(_ptr(x), _rows(x, "x"), None, M, K, _ptr(wt), _rows(wt, "w^T"), N, _lib.GTA_F32,
                                     0, _ptr(out), _rows(out, "out"), splits, _ptr(ws), nb, _stream(x.device)),
          "update_mm_t_split")


def timed(fn, calls=10, reps=7):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(calls):
            fn()
    g.replay()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3 / calls)
    return float(np.median(ts))


def main():
    dev = torch.device("cuda:0")
    shapes = [(2708, 1433, 128), (2708, 1433, 64), (2708, 128, 64), (3327, 3703, 128)]
    res = {}
    for M, K, N in shapes:
        torch.manual_seed(0)
        x = torch.randn(M, K, device=dev)
        w = torch.randn(K, N, device=dev) * K ** -0.5
        wt = ops._transposed(w)
        out = torch.empty(M, N, device=dev)
        rec = {}
        ops.set_debug("mm_ring", 0)
        def plain():
            check(_L().gta_update_mm_t(_ptr(x), K, None, M, K, _ptr(wt), _rows(wt, "w^T"), N, _lib.GTA_F32, 0,
                                       _ptr(out), N, _stream(dev)), "update_mm_t")
        rec["hipblaslt_us"] = timed(plain)
        ref = out.clone()
        ops.set_debug("mm_blaslt", 0)
        for splits in (4, 8, 16, 32, 48):
            if K // 32 < splits // 2:
                continue
            nb = check(_L().gta_update_mm_t_split_workspace_bytes(M, K, N, splits), "ws")
            ws = torch.empty(nb // 4, device=dev)
            outs = {}
            for form, ring in (("rows", 0), ("ring", 1)):
                ops.set_debug("mm_ring", ring)
                rec[f"{form}_s{splits}_us"] = timed(lambda: split_call(x, wt, out, M, K, N, splits, ws, nb))
                outs[form] = out.clone()
            rec[f"s{splits}_bitwise"] = bool(torch.equal(outs["rows"], outs["ring"]))
            rec[f"s{splits}_max_vs_blaslt"] = float((outs["ring"] - ref).abs().max())
        ops.set_debug("mm_ring", 1)
        ops.set_debug("mm_blaslt", 1)
        res[f"{M}x{K}x{N}"] = rec
        print(f"{M}x{K}x{N} " + " ".join(f"{k}={v:.1f}" if isinstance(v, float) and k.endswith("us") else f"{k}={v}"
                                          for k, v in rec.items() if not k.endswith("vs_blaslt")), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "split_probe.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
