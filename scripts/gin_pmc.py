"""Fabric traffic of the GIN products aggregate: rocprofv3 --pmc FETCH_SIZE and
WRITE_SIZE, separate passes, over the exact launch the layer runs -- gta_aggregate_self over bf16
200-B rows (at the model input's line pitch, round 5), the layer's [E, 1] edge operand, (1 + eps) x
formed in the epilogue, the executor's 512-edge plan, y stored in bf16 for the fused MLP (ABI 10) -- calibrated in the same pass like bench.py's metric traffic: a 1 GiB
float4 copy gives the streaming read factor, and the same aggregate kernel over a permutation graph
(one edge per row: every 200-B row of the 2.45 M-row bf16 table read once, in random order, 4 x
64-B sectors each at 8-B alignment) gives this row gather's factor.  The real launch's FETCH is then
its known streams (indices, row pointers, the in-order self-term rows) plus gathers.

Usage: python scripts/gin_pmc.py [--out DIR]      (parent: runs the two passes, prints one JSON line)
       python scripts/gin_pmc.py --child           (under rocprofv3)
"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

REPS = 3
F = 100
CALIB_ROWS = 1 << 21  # 1 GiB of fp32 [., 128] rows


def child():
    import torch
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import configs, graph as G, ops
    dev = torch.device("cuda", 0)
    _, g, tensors = configs.build("gin-products", dev)
    x = tensors[0]["x"]
    assert x.dtype == torch.bfloat16 and x.shape[1] == F, (x.dtype, x.shape)
    w = next(v for k, v in tensors[0].items() if k.startswith("ext:") and tuple(v.shape) == (g.nnz, 1))
    s = torch.tensor([[1.1]], device=dev)
    n = g.n_rows
    if "--no-calib" in sys.argv:  # the layer's launches only (counter groups of scripts/pmc_sq.py)
        for _ in range(REPS + 1):
            ops.aggregate(g, x, "src", w, plan=512, self_term=(x, s), out_dtype=torch.bfloat16)
        torch.cuda.synchronize()
        return 0
    # streaming calibration: a float4 copy of a 1 GiB table (k_apply_node4: read once, written once)
    xc = torch.ones(CALIB_ROWS, 128, device=dev)
    yc = torch.empty_like(xc)
    for _ in range(2):
        ops.apply_node(None, None, xc, out=yc)
    del xc, yc
    # gather calibration: the aggregate's row gather over a permutation graph (one edge per row,
    # every 200-B row of the table read once, in random order)
    ip = torch.arange(n + 1, device=dev, dtype=torch.int64)
    perm = torch.argsort(G.hash32(torch.arange(n, device=dev, dtype=torch.int64), 7, 9)).to(torch.int32)
    gc = G.Graph(ip, perm)
    for _ in range(2):
        ops.aggregate(gc, x, "src", None, plan=512)
    torch.cuda.synchronize()
    del gc, ip, perm
    for _ in range(REPS):
        ops.aggregate(g, x, "src", w, plan=512, self_term=(x, s), out_dtype=torch.bfloat16)
    torch.cuda.synchronize()
    with open(os.environ["GIN_PMC_META"], "w") as fh:
        json.dump({"n": int(n), "e": int(g.nnz), "pitch_bytes": int(x.stride(0) * x.element_size())}, fh)
    return 0


def counters(d, name):
    """-> [(kind, value)] in dispatch order: 'copy' (k_apply_node4), 'agg' (k_aggregate, not the
    combine kernel)."""
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            kn = row.get("Kernel_Name", "")
            if row.get("Counter_Name") != name:
                continue
            kind = "copy" if "k_apply_node4" in kn else ("agg" if "k_aggregate" in kn and "combine" not in kn else None)
            if kind:
                did = row.get("Dispatch_Id") or row.get("Correlation_Id") or "0"
                rows.append((int(did), kind, float(row["Counter_Value"])))
    return [(k, v) for _, k, v in sorted(rows)]


def main():
    if "--child" in sys.argv:
        return child()
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else os.path.join(ROOT, "gpurun_out", "gin_pmc")
    os.makedirs(out, exist_ok=True)
    exe = shutil.which("rocprofv3")
    meta = os.path.join(out, "meta.json")
    env = dict(os.environ, GIN_PMC_META=meta, TMPDIR="/tmp")
    res = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = os.path.join(out, ctr.lower())
        cmd = [exe, "--pmc", ctr, "--output-format", "csv", "-d", d, "-o", "run", "--", sys.executable,
               os.path.abspath(__file__), "--child"]
        r = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=400)
        if r.returncode != 0:
            print(json.dumps({"error": f"{ctr} pass rc={r.returncode}", "stderr": r.stderr[-400:]}))
            return 1
        res[ctr] = counters(d, ctr)
    m = json.load(open(meta))
    n, e = m["n"], m["e"]
    pitch = m.get("pitch_bytes", 2 * F)
    # the self-term row read in order: whole 64-B sectors of a line-pitched row, 200 B of a packed one
    self_row = -(-2 * F // 64) * 64 if pitch % 64 == 0 else 2 * F
    fetch, write = res["FETCH_SIZE"], res["WRITE_SIZE"]
    copies = [v for k, v in fetch if k == "copy"]
    aggs = [v for k, v in fetch if k == "agg"]
    aggs_w = [v for k, v in write if k == "agg"]
    # read factors, bytes per counted kB: streaming (the 1 GiB copy) and this kernel's 200-B row
    # gather (each row once: 4 x 64-B sectors at 8-B alignment, + 4 B index + 8 B row pointer)
    kr_s = CALIB_ROWS * 512 / (copies[1] * 1024.0)
    cal_streams = n * (4 + 8)
    kr_g = n * 256 / ((aggs[1] - cal_streams / kr_s / 1024.0) * 1024.0)  # 4 sectors per row at either pitch
    real_kb = sorted(aggs[2:2 + REPS])[REPS // 2]
    real_w_kb = sorted(aggs_w[2:2 + REPS])[REPS // 2]
    # the real launch: known streams (indices and edge weights 4 + 4 B per edge, row pointers 8 B and
    # the self-term row per row, read in order) at kr_s, the rest of FETCH is row gathers at kr_g
    streams = e * 8 + n * (8 + self_row)
    gathers = (real_kb * 1024.0 - streams / kr_s) * kr_g
    traffic = streams + gathers + real_w_kb * 1024.0
    rec = {"what": "GIN products aggregate (gta_aggregate_self, bf16 200-B rows, [E, 1] edge weights, plan 512, bf16 y)",
           "n": n, "e": e, "row_pitch_bytes": pitch,
           "fetch_kb": {"copy": copies[1], "gather_calibration": aggs[1], "launch_median": real_kb},
           "write_kb_launch_median": real_w_kb, "read_factor_stream": round(kr_s, 4),
           "read_factor_gather": round(kr_g, 4), "streams_GB": round(streams / 1e9, 3),
           "gathers_GB": round(gathers / 1e9, 3), "writes_GB": round(real_w_kb * 1024.0 / 1e9, 3),
           "traffic_GB": round(traffic / 1e9, 3), "gather_B_per_edge": round(gathers / e, 1),
           "sector_model_gather_B_per_edge": 256,
           "algorithmic_GB": round((e * (4 + 4 + 200) + n * (8 + 200 + 200)) / 1e9, 3)}
    print(json.dumps(rec))
    return 0


if __name__ == "__main__":
    sys.exit(main())
