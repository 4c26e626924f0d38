"""Time full BASELINE-config layers through the executor (secondary numbers, not the headline)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import configs, executor  # noqa: E402


def main(names=None, reps=5, trace=False, graphed=False):
    dev = torch.device("cuda:0")
    out = {}
    for name in (names or list(configs.CONFIGS)):
        t0 = time.perf_counter()
        layers, g, tensors = configs.build(name, dev)
        build_s = time.perf_counter() - t0
        times = []
        nrep = reps if g.nnz > 10 ** 6 else 10 * reps  # small graphs: launch-bound, more samples
        for r in range(nrep + 1):
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            x = None
            for lay, t in zip(layers, tensors):
                if x is not None:
                    t["x"] = x
                res, _ = lay.run(t, sync=False)  # one synchronisation per forward, at its end
                x = res.outputs[sorted(res.outputs)[-1]]
            torch.cuda.synchronize()
            if r:
                times.append(time.perf_counter() - t1)
        ms = 1e3 * sorted(times)[len(times) // 2]
        graphed_ms = None
        if graphed:  # the same forward replayed as HIP graphs (one per layer)
            runs, prev = [], None
            for lay, t in zip(layers, tensors):
                if prev is not None:
                    t["x"] = prev  # layer k reads layer k-1's (static) graph output
                runs.append(executor.GraphedRun(lay.opgraph, lay.stream, g, t, lay.sem))
                prev = runs[-1].outputs[sorted(runs[-1].outputs)[-1]]
            gt = []
            for r in range(reps + 1):
                torch.cuda.synchronize()
                t1 = time.perf_counter()
                for gr in runs:
                    gr.replay()
                torch.cuda.synchronize()
                if r:
                    gt.append(time.perf_counter() - t1)
            graphed_ms = 1e3 * sorted(gt)[len(gt) // 2]
            del runs
        if trace:  # one more forward with per-op HIP-event tracing (Chrome JSON)
            x = None
            events = []
            for lay, t in zip(layers, tensors):
                if x is not None:
                    t["x"] = x
                res, ex = executor.run_stream(lay.opgraph, lay.stream, g, t, lay.sem, trace=True)
                events += ex.trace_events
                x = res.outputs[sorted(res.outputs)[-1]]
            executor.save_chrome_trace(events, os.path.join(ROOT, "gpurun_out", f"trace_{name}.json"))
        out[name] = {"N": g.n_rows, "E": g.nnz, "layers": [l.layer for l in layers],
                     "op_array": [l.op_array for l in layers], "tile_size_list": [l.tile_size_list for l in layers],
                     "ms_per_forward": ms, "ms_per_forward_hipgraph": graphed_ms, "edges_per_s": g.nnz * len(layers) / (ms / 1e3), "build_s": build_s}
        print(name, json.dumps(out[name]), flush=True)
        del layers, g, tensors
        torch.cuda.empty_cache()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "layer_bench.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops
    argv = [a for a in sys.argv[1:] if a not in ("--trace", "--hipgraph", "--no-mlp", "--graph-all", "--no-bf16-sum",
                                                 "--no-edge-flat", "--no-edge-expr")]
    if "--no-edge-expr" in sys.argv[1:]:  # the applyedge trees of DGN / PNA unfused (A/B of gta_aggregate_expr, ABI 14)
        executor.EDGE_EXPR = False
    if "--no-edge-flat" in sys.argv[1:]:  # apply_edge on the row-sweep forms (A/B of gta_apply_edge_flat, ABI 13)
        ops.APPLY_EDGE_FLAT = False
    if "--no-bf16-sum" in sys.argv[1:]:  # GIN's sum handed to the fused MLP in fp32 (A/B of ABI 10)
        executor.MLP_BF16_SUM = False
    if "--graph-all" in sys.argv[1:]:  # automatic HIP-graph replay at every graph size (A/B of the threshold)
        executor.AUTO_GRAPH_MAX_EDGES = 1 << 40
    if "--no-mlp" in sys.argv[1:]:  # the GIN MLP as two UPDATE launches (A/B of the fused chain)
        executor.FUSE_MLP = False
    if "--mm-rows-min" in argv:  # ops.MM_ROWS_MIN_M: smallest M for the row-streaming UPDATE entry
        i = argv.index("--mm-rows-min")
        ops.MM_ROWS_MIN_M = int(argv[i + 1])
        del argv[i:i + 2]
    main(argv or None, trace="--trace" in sys.argv[1:], graphed="--hipgraph" in sys.argv[1:])
