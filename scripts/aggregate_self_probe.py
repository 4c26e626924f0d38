"""gta_aggregate_self (GIN ops 3-4 in one launch) against apply_node MUL then the aggregate then ADD,
bitwise, for widths that take each aggregate kernel form (lean F = 128, generic LPE = 64 with NV 2/4)."""
import os, sys
import numpy as np
import torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops, graph as G
dev = torch.device("cuda:0")
z = np.load(os.path.join(ROOT, "tests", "golden", "cora_graph.npz"))
g = G.from_numpy(z["indptr"], z["indices"], device=dev)
for F in (602, 128, 600, 604, 300):
    torch.manual_seed(0)
    x = torch.randn(g.n_rows, F, device=dev)
    w = torch.ones(g.nnz, 1, device=dev)
    s = torch.tensor([[1.1]], device=dev)
    T = ops.apply_node("MUL", None, x, s, b_broadcast_row=True)
    Gv = ops.aggregate(g, x, "src", w)
    A1 = ops.apply_node("ADD", None, Gv, T)
    A2 = ops.aggregate(g, x, "src", w, self_term=(x, s))
    torch.cuda.synchronize()
    print(F, "T==x*s", torch.equal(T, x * torch.tensor(1.1, device=dev)), "A1==A2", torch.equal(A1, A2),
          "A1==G+T", torch.equal(A1, Gv + T), "A2==G+T", torch.equal(A2, Gv + T), flush=True)
