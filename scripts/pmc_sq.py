"""SQ / TA / TD / TCC counters of a hot launch, one rocprofv3 --pmc pass per counter group (each
within the per-block slot limits).  Targets (PMC_TARGET):
  metric (default) -- `bench.py --pmc-child`: the bench's own inputs and launches (k_agg_h32 + k_seg_reduce)
  gin              -- `scripts/gin_pmc.py --child --no-calib`: GIN products' aggregate exactly as the
                      layer launches it (k_aggregate<..., ushort> of gta_aggregate_self, bf16 y)
  wcost            -- `scripts/sage_w1_probe.py --pmc-child`: the Reddit blocked pair unweighted, with [E, 1]
                      and with [E, 8] weights (PMC_SPLIT=1 keeps the k_agg_h32 instances apart)
  mm               -- `scripts/mm_pmc_child.py`: the Reddit x.W fp32 UPDATE ([232,965 x 602] at the
                      model input's 608 pitch . [602 x 128], k_mm_wave), with the MFMA group
Per-kernel means over the launches after the first (cold) one.
Usage: python scripts/pmc_sq.py OUT_DIR [bench args]  -> OUT_DIR/<group>/... CSVs and OUT_DIR/summary.json"""
import csv
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GROUPS = {
    "sq_time": ["SQ_WAVES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
                "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_VALU"],
    "sq_insts": ["SQ_INSTS_VALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                 "SQ_ACTIVE_INST_LDS", "SQ_INSTS_SMEM", "GRBM_GUI_ACTIVE"],
    "l2": ["TCC_HIT_sum", "TCC_MISS_sum", "TCP_TCC_READ_REQ_sum"],
    # the texture path (round 4): TA / TD busy and stall cycles, L1 -> L2 read latency
    # MFMA occupancy and the effective clock (round 5): fp32 UPDATE
    "mfma": ["SQ_VALU_MFMA_BUSY_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY",
             "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "GRBM_GUI_ACTIVE"],
    "tex": ["TA_TA_BUSY_sum", "TA_ADDR_STALLED_BY_TC_CYCLES_sum", "TD_TD_BUSY_sum", "TD_TC_STALL_sum",
            "TCP_TCC_READ_REQ_LATENCY_sum", "TCP_TCC_READ_REQ_sum", "TCP_PENDING_STALL_CYCLES_sum", "GRBM_GUI_ACTIVE"],
}
TARGETS = {
    "metric": (["bench.py", "--pmc-child", "--steps", "4"], ("k_agg_h32", "k_seg_reduce")),
    "gin": (["scripts/gin_pmc.py", "--child", "--no-calib"], ("k_aggregate",)),
    "mm": (["scripts/mm_pmc_child.py"], ("k_mm_wave",)),
    "wcost": (["scripts/sage_w1_probe.py", "--pmc-child"], ("k_agg_h32",)),
}
TARGET = os.environ.get("PMC_TARGET", "metric")
KERNELS = TARGETS[TARGET][1]


def _kernel(name):
    """The KERNELS entry a dispatch belongs to (a combine / reduce helper only when named)."""
    return next((k for k in KERNELS if k in name and ("combine" in k or "combine" not in name)), None)


def summarize(d):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", "")
            k = _kernel(name)
            if k is None:
                continue
            if os.environ.get("PMC_SPLIT"):  # one entry per template instance (e.g. k_mm_wave<8, 4, 1>)
                k = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            did = int(row.get("Dispatch_Id") or row.get("Correlation_Id") or 0)
            per.setdefault((k, row["Counter_Name"]), []).append((did, float(row["Counter_Value"])))
    out = {}
    for (k, c), vals in per.items():
        vals = [v for _, v in sorted(vals)]
        vals = vals[1:] if len(vals) > 1 else vals
        out.setdefault(k, {})[c] = sum(vals) / len(vals)
    return out


EXTRA = []  # bench.py arguments after OUT_DIR (e.g. --blocks 16 --knobs seg_lean=0)


def main(out_dir):
    os.makedirs(out_dir, exist_ok=True)
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"), GIN_PMC_META=os.path.join(out_dir, "meta.json"))
    script = TARGETS[TARGET][0]
    summary = {}
    for gname, counters in GROUPS.items():
        d = os.path.join(out_dir, gname)
        shutil.rmtree(d, ignore_errors=True)
        cmd = ["timeout", "-s", "KILL", "120", shutil.which("rocprofv3") or "rocprofv3", "--kernel-trace", "--pmc",
               *counters, "--output-format", "csv", "-d", d, "-o", "run", "--", sys.executable,
               os.path.join(ROOT, script[0]), *script[1:], *EXTRA]
        p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True)
        print(gname, "rc", p.returncode, p.stderr[-300:] if p.returncode else "", flush=True)
        if p.returncode != 0:
            summary[gname] = {"error": p.returncode}
            if p.returncode in (124, 137, -9):
                break
            continue
        summary[gname] = summarize(d)
    with open(os.path.join(out_dir, "summary.json"), "w") as fh:
        json.dump(summary, fh, indent=1)
    print(json.dumps(summary))
    return 0


if __name__ == "__main__":
    EXTRA.extend(sys.argv[2:])
    if os.environ.get("PMC_GROUPS"):  # e.g. PMC_GROUPS=l2: only those counter groups
        keep = os.environ["PMC_GROUPS"].split(",")
        for g in list(GROUPS):
            if g not in keep:
                del GROUPS[g]
    sys.exit(main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc_sq"))
