"""Full BASELINE-config layers on N GPUs (one process per GPU, distributed.py).

  python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P scripts/dist_layers.py [config ...] [--reps R] [--layout rows|cols]

Each rank builds the same compiled layer (front end -> search -> stream, on the
global graph), keeps its shard, and executes the stream.  --layout rows (default):
destination-row shards, one all-gather per source table; cols: source-column
shards, reduce-scatter per gather and all-gather per dst-side scatter.  Rank 0 prints one JSON line per config: ms per forward
(max over ranks), edges/s, exchanged bytes, and the max normalised difference
of the re-assembled output vs a 1-device execution of the same stream.
GTA_DIST_BACKEND=gloo GTA_SINGLE_DEVICE=1 rehearses several ranks on one GPU.
"""
import json
import os
import sys
import time

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import configs, distributed, executor  # noqa: E402


def main():
    args = sys.argv[1:]
    reps = 5
    if "--reps" in args:
        i = args.index("--reps")
        reps = int(args[i + 1])
        del args[i:i + 2]
    layout = "rows"
    if "--layout" in args:
        i = args.index("--layout")
        layout = args[i + 1]
        del args[i:i + 2]
    probe = 0  # --probe W: one process times rank 0's shard of a W-way cut (compute only, no exchange)
    if "--probe" in args:
        i = args.index("--probe")
        probe = int(args[i + 1])
        del args[i:i + 2]
    replicate = "--no-replicate" not in args  # rows: keep model inputs whole (no exchange of x)
    args = [a for a in args if a != "--no-replicate"]
    names = args or ["sage-reddit", "gin-products"]
    rank, world = int(os.environ.get("RANK", 0)), int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    dev = torch.device("cuda:0" if os.environ.get("GTA_SINGLE_DEVICE") else f"cuda:{local}")
    torch.cuda.set_device(dev)
    backend = os.environ.get("GTA_DIST_BACKEND", "nccl")
    if world > 1:
        dist.init_process_group(backend, rank=rank, world_size=world, device_id=dev if backend == "nccl" else None)
    out = {}
    for name in names:
        layers, g, tensors = configs.build(name, dev)
        if layout == "rows":
            shard = distributed.RowShard(g, rank, probe or world, replicate_inputs=replicate)
        else:
            shard = distributed.DistShard(g, rank, probe or world)
        times, comm_bytes, rep_bytes = [], 0, 0
        for r in range(reps + 1):
            if world > 1:
                dist.barrier()
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            x = None
            for lay, t in zip(layers, tensors):
                t = dict(t)
                if x is not None:
                    t["x"] = x
                res, ex = distributed.run_stream(lay.opgraph, lay.stream, shard, t, lay.sem)
                x = res.outputs[sorted(res.outputs)[-1]]
                if r == 0:
                    comm_bytes += ex.dist.bytes
                    rep_bytes += ex.dist.replicated_bytes
            torch.cuda.synchronize(dev)
            dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev if backend == "nccl"
                              else "cpu")
            if world > 1:
                dist.all_reduce(dt, op=dist.ReduceOp.MAX)
            if r:
                times.append(float(dt))
        full = ex.dist.full_rows(x) if world > 1 else x
        err = None
        if rank == 0 and not probe:  # the same stream on one device, same inputs
            y = None
            for lay, t in zip(layers, tensors):
                t = dict(t)
                if y is not None:
                    t["x"] = y
                r1, _ = executor.run_stream(lay.opgraph, lay.stream, g, t, lay.sem)
                y = r1.outputs[sorted(r1.outputs)[-1]]
            fin = torch.isfinite(y)
            err = float(((full - y).abs()[fin]).max() / (y.abs()[fin].max() + 1e-30))
        ms = 1e3 * sorted(times)[len(times) // 2]
        rec = {"config": name, "n_gpus": world, "N": g.n_rows, "E": g.nnz, "shard_edges": shard.graph.nnz,
               "ms_per_forward": ms, "edges_per_s": g.nnz * len(layers) / (ms / 1e3),
               "exchanged_bytes_per_rank": comm_bytes, "replicated_input_bytes": rep_bytes, "layout": layout, "probe_world": probe or None, "backend": backend if world > 1 else None,
               "max_norm_diff_vs_1dev": err}
        out[name] = rec
        if rank == 0:
            print(json.dumps(rec), flush=True)
        del layers, g, tensors, shard, ex, res, x, full
        torch.cuda.empty_cache()
    if rank == 0:
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        with open(os.path.join(ROOT, "gpurun_out", f"dist_layers_{layout}_{world}{f'_probe{probe}' if probe else ''}.json"), "w") as f:
            json.dump(out, f, indent=1)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
