"""Does torch's gloo run the exchange calls bench.py makes (reduce_scatter_tensor on a row-group
subgroup, all_gather_into_tensor, async) on DEVICE tensors?  One-GPU rehearsal helper: run under
torch.distributed.run with GTA_SINGLE_DEVICE ranks on cuda:0.  Prints one line per call and rank."""
import os
import sys
import time

import torch
import torch.distributed as dist


def main():
    dist.init_process_group("gloo")
    r, w = dist.get_rank(), dist.get_world_size()
    dev = torch.device("cuda", 0)
    x = (torch.arange(4 * w, dtype=torch.float32, device=dev).view(2 * w, 2) + r).contiguous()
    out = torch.empty(2, 2, device=dev)
    for name, fn in (
        ("reduce_scatter_tensor", lambda: dist.reduce_scatter_tensor(out, x)),
        ("reduce_scatter_tensor async", lambda: dist.reduce_scatter_tensor(out, x, async_op=True).wait()),
        ("all_gather_into_tensor async", lambda: dist.all_gather_into_tensor(torch.empty(2 * w, 2, device=dev), out,
                                                                            async_op=True).wait()),
    ):
        t0 = time.time()
        try:
            fn()
            torch.cuda.synchronize()
            print(r, name, "ok", round(time.time() - t0, 3), flush=True)
        except Exception as e:  # noqa: BLE001 -- the probe reports what gloo does
            print(r, name, "FAIL", type(e).__name__, str(e)[:150], flush=True)
    if w >= 4:
        groups = [dist.new_group([0, 1]), dist.new_group([2, 3])] + [dist.new_group([k, k + 1]) for k in range(4, w, 2)]
        g = groups[r // 2]
        try:
            dist.reduce_scatter_tensor(out, x[:4].contiguous(), group=g, async_op=True).wait()
            print(r, "subgroup reduce_scatter ok", flush=True)
        except Exception as e:  # noqa: BLE001
            print(r, "subgroup FAIL", str(e)[:150], flush=True)
    dist.barrier()
    dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
