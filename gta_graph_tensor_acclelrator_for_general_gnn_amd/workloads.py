"""Deterministic synthetic inputs for a GTA op graph (no datasets/checkpoints exist offline).

For an OpGraph this builds every tensor the executor needs, named as the
executor looks them up:
  "x"              model input [N, F_in] ~ N(0, 1), on line-pitched storage (ops.line_pitch: the
                   layout the aggregates gather whole rows from, chosen once here)
  "w:<op>"         MM weights [F_in_op, F_out_op] ~ N(0, 1/F_in)  (applynode/applyedge MM)
  "ext:<op>:<s>"   external (-1) inputs: scalar edge weights [E, 1] (GCN 1/sqrt(d_i d_j)
                   normalisation for GCN/SGC, 1/deg(i) for GraphSAGE-mean, 1 for GIN),
                   GIN op 3's operands (x, 1+eps), DGN's hidden-width node inputs
  "x_edge"         edge features [E, F] for PNA's applyedge MM on the model input
Shapes follow the op YAML sizes (bytes / 4).
"""
import torch

from . import graph as G
from . import ops


def make_tensors(opgraph, graph, network=None, seed=0, device=None, dtype_w=torch.float32, dtype_x=torch.float32):
    """dtype_x: the model input's storage type (bfloat16 for the bf16 GIN configuration: the
    aggregate then gathers 2-byte rows, BASELINE.md's GIN byte model; every kernel widens them
    exactly and sums in fp32)."""
    device = device or graph.device
    gen = torch.Generator(device="cpu")
    gen.manual_seed(seed)

    def randn(*shape, scale=1.0):
        return (torch.randn(*shape, generator=gen) * scale).to(device)

    n, e = graph.n_rows, graph.nnz
    t = {}
    # the model input width: first op reading x
    fin = None
    for op in opgraph.ops:
        for s, src in enumerate(opgraph.inputs[op.idx]):
            if src.kind == "x" and op.type != "applyedge":
                w = op.in_width(s)
                if w and (fin is None):
                    fin = w
    if fin is not None:
        t["x"] = ops.pitched(randn(n, fin).to(dtype_x))
    for op in opgraph.ops:
        if op.comp == "MM":
            k = op.in_width(0)
            t[f"w:{op.idx}"] = randn(k, op.out_width, scale=k ** -0.5).to(dtype_w)
        for s, src in enumerate(opgraph.inputs[op.idx]):
            if src.kind == "x" and op.type == "applyedge":
                t.setdefault("x_edge", randn(e, op.in_width(s)))
            if src.kind == "x" and op.type != "applyedge" and fin is not None and op.in_width(s) != fin:
                t[f"ext:{op.idx}:{s}"] = randn(n, op.in_width(s))
            if src.kind != "ext":
                continue
            width = op.in_width(s) or 1
            key = f"ext:{op.idx}:{s}"
            if op.type == "applyedge":
                if network in ("GCN", "SGC"):
                    t[key] = G.gcn_norm_weights(graph).view(-1, 1).to(device)
                elif network == "GraphSAGE":
                    deg = graph.degrees().clamp_min(1).to(torch.float32)
                    t[key] = (1.0 / deg)[graph.row_of_edge().long()].view(-1, 1).to(device)
                elif network == "GIN":
                    t[key] = torch.ones(e, 1, device=device)
                else:
                    t[key] = (torch.rand(e, width, generator=gen) + 0.5).to(device)
            else:
                if width == 1:  # GIN (1 + eps)
                    t[key] = torch.full((1, 1), 1.1, device=device)
                elif "x" in t and t["x"].shape[1] == width:
                    t[key] = t["x"]
                else:
                    t[key] = randn(n, width)
    return t
