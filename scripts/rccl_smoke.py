"""RCCL on the box: bench.py's collective calls, as bench.py makes them, in a process group of
the ranks started by torch.distributed.run (one per GPU).  Backend "nccl" (= RCCL), the default
group bound to the rank's device (eager init), the row groups of distributed.row_groups, then per
row chunk an async reduce_scatter_tensor (edges mode) and an async all_gather_into_tensor (rows
mode) of chunk-major padded rows, an all_reduce MAX / SUM of float64 timings.  Each result is
checked against its closed form; prints one JSON line on rank 0."""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed  # noqa: E402


def main():
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist.init_process_group("nccl", device_id=dev)
    pr, pc = distributed.grid_shape(world, "edges")
    groups = distributed.row_groups(pr, pc) if pc > 1 else None
    group = groups[rank // pc] if groups else None
    j = rank % pc
    chunks, mk, F = 2, 1000, 128
    # edges mode: chunk c = [pc * mk] padded rows, one mk-row part per rank of the row group
    y = torch.arange(chunks * pc * mk * F, device=dev, dtype=torch.float32).view(-1, F) * (rank + 1)
    own = torch.empty(chunks * mk, F, device=dev)
    works = []
    for c in range(chunks):
        a, b = c * pc * mk, (c + 1) * pc * mk
        works.append(dist.reduce_scatter_tensor(own[c * mk:(c + 1) * mk], y[a:b], group=group, async_op=True))
    for w in works:
        w.wait()
    scale = sum(q + 1 for q in range(rank - j, rank - j + pc))  # sum of (rank+1) over the row group
    base = torch.arange(chunks * pc * mk * F, device=dev, dtype=torch.float32).view(-1, F)
    want = torch.cat([base[c * pc * mk + j * mk:c * pc * mk + (j + 1) * mk] for c in range(chunks)]) * scale
    rs_ok = bool(torch.equal(own, want))
    # rows mode: every rank's chunk part gathered into the padded full table
    part = torch.full((chunks * mk, F), float(rank), device=dev)
    full = torch.empty(chunks * world * mk, F, device=dev)
    works = [dist.all_gather_into_tensor(full[c * world * mk:(c + 1) * world * mk], part[c * mk:(c + 1) * mk],
                                         async_op=True) for c in range(chunks)]
    for w in works:
        w.wait()
    ag_ok = all(bool((full[c * world * mk + q * mk:c * world * mk + (q + 1) * mk] == q).all())
                for c in range(chunks) for q in range(world))
    t = torch.tensor([float(rank)], device=dev, dtype=torch.float64)
    t2 = t.clone()
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(t2, op=dist.ReduceOp.SUM)
    ar_ok = float(t) == world - 1 and float(t2) == world * (world - 1) / 2
    torch.cuda.synchronize()
    dist.barrier()
    if rank == 0:
        print(json.dumps({"backend": dist.get_backend(), "world_size_seen": dist.get_world_size(),
                          "grid": f"{pr}x{pc}", "reduce_scatter_ok": rs_ok, "all_gather_ok": ag_ok,
                          "all_reduce_ok": ar_ok}), flush=True)
    dist.destroy_process_group()
    return 0 if (rs_ok and ag_ok and ar_ok) else 1


if __name__ == "__main__":
    sys.exit(main())
