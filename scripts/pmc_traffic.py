"""Per-launch HBM bytes of the aggregate kernel from two rocprofv3 --pmc passes.

Method (MI355X_MICROARCH.md §HBM, cdna_hip_programming.md §7): FETCH_SIZE and
WRITE_SIZE are collected in SEPARATE passes (TCC slots: FETCH_SIZE costs 3,
WRITE_SIZE 2); both are in KB.  On gfx950 FETCH_SIZE reports exactly half of
the bytes of wide (16 B/lane) coalesced reads, so the read side is doubled;
WRITE_SIZE is exact for 16-B-per-lane stores.  The aggregate's reads are 16 B
per lane (float4 rows) and its stores are float4 rows.
  hbm_bytes_per_launch = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
Writes profiles/pmc_traffic.json.
"""
import csv
import glob
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


# the metric's aggregate kernels: plan path k_aggregate<..., 0, 1> / k_agg_lean, blocked path
# k_agg_h32 (lean half-wave, default), k_agg_seg4 or k_agg_seg2d, then k_seg_reduce
METRIC_KERNELS = {"plan": re.compile(r"k_aggregate<\d+, \d+, \d+, 0, 1>|k_agg_lean<"),
                  "blocked": re.compile(r"k_agg_seg2d<|k_agg_seg4<|k_agg_h32<|k_seg_reduce<")}
METRIC_KERNEL = METRIC_KERNELS["blocked"]


def read_counter(d, counter):
    """Per-launch value: sum over the dispatches of one aggregate launch (seg2d + reduce are one launch
    pair; consecutive matching dispatches are grouped by Dispatch_Id order)."""
    files = glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True)
    rows = []
    for f in files:
        for row in csv.DictReader(open(f)):
            if METRIC_KERNEL.search(row.get("Kernel_Name", "")) and row.get("Counter_Name") == counter:
                rows.append((int(row.get("Dispatch_Id", 0)), row["Kernel_Name"], float(row["Counter_Value"])))
    rows.sort()
    vals, cur = [], 0.0
    for _, name, v in rows:
        cur += v
        if "k_seg_reduce" in name or not ("k_agg_seg2d" in name or "k_agg_seg4" in name or "k_agg_h32" in name):
            vals.append(cur)
            cur = 0.0
    return vals


def main(fetch_dir="gpurun_out/pmc_fetch", write_dir="gpurun_out/pmc_write", n=232965, e=114615892):
    f = read_counter(os.path.join(ROOT, fetch_dir), "FETCH_SIZE")
    w = read_counter(os.path.join(ROOT, write_dir), "WRITE_SIZE")
    if not f or not w:
        print("no counters found", len(f), len(w))
        return 1
    # skip the first (cold) dispatch when there are several
    fs = f[1:] if len(f) > 1 else f
    ws = w[1:] if len(w) > 1 else w
    fetch_kb = sum(fs) / len(fs)
    write_kb = sum(ws) / len(ws)
    hbm = 2 * fetch_kb * 1024 + write_kb * 1024
    out = {"n": n, "e": e, "impl": "blocked", "kernel": "k_agg_h32 + k_seg_reduce", "dispatches": [len(f), len(w)],
           "FETCH_SIZE_KB_avg": fetch_kb, "WRITE_SIZE_KB_avg": write_kb,
           "hbm_bytes_per_launch": hbm,
           "method": "2*FETCH_SIZE*1024 + WRITE_SIZE*1024 (gfx950 FETCH_SIZE half-count correction), "
                     "separate --pmc passes, first dispatch skipped"}
    with open(os.path.join(ROOT, "profiles", "pmc_traffic.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out))
    return 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
