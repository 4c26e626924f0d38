"""The BASELINE.json configurations as runnable workloads (synthetic graphs of the named shapes).

  gcn-cora     2-layer GCN on Cora (hidden 128): layer 1 (1433->128) then layer 2 (128->64)
  gat8-flickr  GAT layer 1 on Flickr (89,250 nodes / 899,756 edges), 8 heads, F=500
  sage-reddit  GraphSAGE-mean layer 1 on Reddit (232,965 / 114,615,892), F=602
  gin-products GIN layer 1 on an ogbn-products-shaped CSR (2,449,029 / 123,718,280), F=100,
               node features stored in bf16 (200-B rows: BASELINE.md's "4 + 200 B (bf16)" per
               edge), both MLP GEMMs in bf16 on MFMA, every sum in fp32
  gat8-reddit  GAT layer 1 on Reddit, 8 heads, F=602: not a BASELINE config; the full layer
               around the metric's aggregate (edge-softmax, GEMMs, aggregate, ELU)
  sgc/dgn/pna-flickr, gat8-flickr-trans
               the other genGraphOP networks (and GAT's reordered form) at Flickr scale: not
               BASELINE configs; they show every network's stream runs at size
(config 0 -- V2/GAT_Cora.yaml through the V2 lowering -- is legacy.py: create_list restated
byte-exactly (tests/test_legacy_v2.py) and its stream executed on libgta (test_gpu_executor.py).)
"""
import torch

from . import graph as G, pipeline, workloads

CONFIGS = {
    "gcn-cora": dict(network="GCN", dataset="cora", feature=1433, layers=(1, 2)),
    "gat8-flickr": dict(network="GAT", dataset="flickr", feature=500, layers=(1,), heads=8),
    "gat8-reddit": dict(network="GAT", dataset="reddit", feature=602, layers=(1,), heads=8),
    "sage-reddit": dict(network="GraphSAGE", dataset="reddit", feature=602, layers=(1,)),
    "gin-products": dict(network="GIN", dataset="products", feature=100, layers=(1,), bf16=True),
    "gat8-flickr-trans": dict(network="GAT", dataset="flickr", feature=500, layers=(1,), heads=8, reorder=True),
    "sgc-flickr": dict(network="SGC", dataset="flickr", feature=500, layers=(1,)),
    "dgn-flickr": dict(network="DGN", dataset="flickr", feature=500, layers=(1,)),
    "pna-flickr": dict(network="PNA", dataset="flickr", feature=500, layers=(1,)),
}


def build(name, device, seed=0, graph=None):
    """-> (list of pipeline.Layer, graph, tensors of the first layer)."""
    c = CONFIGS[name]
    g = graph if graph is not None else G.dataset_graph(c["dataset"], seed=seed, device=device)
    layers = []
    meta = None
    for i, L in enumerate(c["layers"]):
        feat = c["feature"] if L == 1 else [0, c["feature"], 128, 64, 16][L]
        lay = pipeline.Layer(c["network"], L, g, feat, reorder=c.get("reorder", False), heads=c.get("heads", 16),
                             metadata=meta)
        meta = meta or lay.metadata
        layers.append(lay)
    dtype_w = torch.bfloat16 if c.get("bf16") else torch.float32
    tensors = [workloads.make_tensors(lay.opgraph, g, c["network"], seed=seed + k, dtype_w=dtype_w,
                                      dtype_x=dtype_w if k == 0 else torch.float32)
               for k, lay in enumerate(layers)]
    return layers, g, tensors


def run(name, device, seed=0):
    """Run every layer of the config, feeding each layer's sink output into the next as x."""
    layers, g, tensors = build(name, device, seed)
    results = []
    x = None
    for lay, t in zip(layers, tensors):
        if x is not None:
            t["x"] = x
        res, ex = lay.run(t)
        results.append((lay, res, ex))
        sinks = sorted(res.outputs)
        x = res.outputs[sinks[-1]]
    return results, g
