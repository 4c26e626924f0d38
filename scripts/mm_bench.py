"""Time gta_update_mm (UPDATE on MFMA) on the layer shapes, both kernel forms, and cross-check them."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops  # noqa: E402

SHAPES = [  # (name, M, K, N, x dtype, w dtype)
    ("gat-reddit op0", 232965, 602, 128, torch.float32, torch.float32),
    ("gat-reddit op1", 232965, 128, 8, torch.float32, torch.float32),
    ("gin-products mlp1", 2449029, 100, 128, torch.float32, torch.bfloat16),
    ("gin-products mlp2", 2449029, 128, 128, torch.float32, torch.bfloat16),
    ("sage-reddit op3", 232965, 602, 128, torch.float32, torch.float32),
    ("bf16 x", 2449029, 128, 128, torch.bfloat16, torch.bfloat16),
]


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    res = {}
    for name, M, K, N, tx, tw in SHAPES:
        x = torch.randn(M, K, device=dev).to(tx)
        w = (torch.randn(K, N, device=dev) * K ** -0.5).to(tw)
        outs = {}
        for form in (0, 1):
            ops.MM_FORM = "rows" if form else "tile"
            ops.MM_ROWS_MIN_M = 0
            if form:
                for bpc in (2, 8):
                    ops.set_debug("mm_blocks_per_cu", bpc)
                    ms = timed(lambda: ops.update_mm(x, w))
                    res[f"{name}:form1:bpc{bpc}"] = {"ms": ms}
                ops.set_debug("mm_blocks_per_cu", 0)
                for pf in (0, 2):
                    ops.set_debug("mm_prefetch", pf)
                    ms = timed(lambda: ops.update_mm(x, w))
                    res[f"{name}:form1:bpcpf{pf}"] = {"ms": ms}
                ops.set_debug("mm_prefetch", 1)
            ms = timed(lambda: ops.update_mm(x, w))
            outs[form] = ops.update_mm(x, w)
            nbytes = M * K * x.element_size() + M * N * 4 + K * N * w.element_size()
            res[f"{name}:form{form}"] = {"ms": ms, "GBps": nbytes / ms / 1e6,
                                         "TFLOPs": 2 * M * K * N / ms / 1e9}
        d = float((outs[0] - outs[1]).abs().max() / outs[0].abs().max())
        res[f"{name}:form1"]["max_rel_diff_vs_form0"] = d
        print(name, json.dumps(res[f"{name}:form0"]), json.dumps(res[f"{name}:form1"]),
              {k.split(":")[-1]: round(v["ms"], 3) for k, v in res.items() if k.startswith(name + ":form1:bpc")},
              flush=True)
        del x, w, outs
    ops.MM_FORM = "rows"
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "mm_bench.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
