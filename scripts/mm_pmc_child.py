"""PMC child of scripts/pmc_sq.py (PMC_TARGET=mm): the Reddit x.W fp32 UPDATE as GraphSAGE / GAT
Reddit launch it -- x [232,965 x 602] on the model input's line-pitched storage (608), W [602 x 128],
k_mm_wave's plan (three whole rounds of FR-4 units + the remainder as an FR-3 launch) -- 4 times
(the first, cold, is dropped by the summary)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(11)
    x = ops.pitched(torch.randn(232965, 602, generator=g).to(dev))
    w = (torch.randn(602, 128, generator=g) / 602 ** 0.5).to(dev)
    out = torch.empty(232965, 128, device=dev)
    for _ in range(4):
        ops.update_mm(x, w, out=out)
    torch.cuda.synchronize()
    return 0


if __name__ == "__main__":
    sys.exit(main())
