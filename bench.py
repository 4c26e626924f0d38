"""Headline benchmark: GAT neighbour AGGREGATE on Reddit-shaped CSR (BASELINE.json metric).

One "step" = one pass of the hot path over the whole graph: the fused COMP_MUL_COMP_ADD block
[3, 11, 12] of GAT layer 1 (scatter C -> applyedge MUL -> gather ADD, reference
code/interpreter.py:575-636, 764-802), i.e.
    Y[i, :] = sum_{e -> i} alpha[e, head(c)] * X1[src(e), :]
with N = 232,965, E = 114,615,892, F = 128 fp32 = 8 heads x 16, alpha [E, 8] fp32 (metric.py).
Inputs are synthetic, counter-hashed (every value a function of (seed, id)) and resident in HBM
before the timed region.

--gpus N (one process per GPU via torch.distributed.run; RCCL = the "nccl" backend):
  --mode edges (default; the north-star form): the edges are cut into a pr x pc grid of the
      reference's row-tile x column tiles (code/preprocessing.py:26-38): row groups of destination
      rows and column groups of source columns, both nnz-balanced from the tile metadata (column
      cuts from the all-reduced per-column nnz).  Each rank aggregates its tile into partial
      vertex aggregates; the pc ranks of a row group sum them with an RCCL reduce-scatter per
      destination-row chunk (three chunks of 55 / 30 / 15 % of the rows by default), issued while the
      next chunk aggregates.  Every rank ends with its complete rows of Y.  Grid 1x2, 2x2, 4x2 at
      N = 2, 4, 8 (--grid PRxPC to override).
  --mode rows: destination-row tiles (complete rows, no reduction) followed by the RCCL
      all-gather of Y that the next layer's scatter C needs, per row chunk, overlapped likewise.
Each rank generates only its row group's edges and its column slice of X (metric.Shard).
Total work is fixed (one Reddit graph): "scaling": "strong"; value = E / max-rank step time.

Printed JSON (rank 0):
  parity        sampled output rows of every rank (incl. the heaviest and lightest) re-derived in fp64
                by the oracle (oracle/isa_ref.aggregate), |err| <= 1e-5 * sum|terms| + 1e-6 each
  roofline      the aggregate launch pair (k_agg_h32 + k_seg_reduce) of every rank's tile: traffic = memory-side
                bytes per step from two rocprofv3 --pmc passes each rank runs on its own tile's kernels in
                child processes, before it initialises the GPU (FETCH_SIZE, WRITE_SIZE; at N > 1 the child
                rebuilds the rank's tile alone from metric.column_counts).  Two read factors, each calibrated
                in the same pass on known bytes (MI355X_MICROARCH.md §HBM): streaming reads on a float4 copy
                (k_apply_node4), gathered 512-B rows on a permutation gather with 16-B lanes; k_agg_h32's
                FETCH is split into its known streams (indices, alpha, item records: streaming factor) and
                the rest (its X gathers: gather factor); k_seg_reduce's partial-row reads take the streaming
                factor; writes take the copy's write factor.  achieved = traffic / HIP-event time of the
                tile's launches alone, frac = achieved / 8 TB/s.  The headline fields are the critical rank's
                (longest compute); per_rank lists every rank's compute_ms, step_ms, exposed_exchange_ms
                (step - compute), traffic, achieved, frac.  alg_* = the SURVEY §8d byte model (548 B/edge:
                every gathered X row), frac_l2 = its rate against the L2-served gather ceiling.
  cpu_baseline  oracle/spmm_ref.c (fp32, OpenMP, every core of sched_getaffinity and the cgroup quota) on a
                bounded row sample of the same workload, rank 0 after the timed region, median of 5 after
                one warm-up.
"""
import argparse
import csv
import fcntl
import glob
import json
import os
import shutil
import signal
import subprocess
import sys
import tempfile
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from gta_graph_tensor_acclelrator_for_general_gnn_amd import distributed, graph as G, metric, ops  # noqa: E402

N_REDDIT, E_REDDIT, F, HEADS = metric.N_REDDIT, metric.E_REDDIT, metric.F, metric.HEADS
PEAK_HBM_GBS = 8000.0     # MI355X_MICROARCH.md chip table (spec)
L2_GATHER_GBS = 18800.0   # MI355X_MICROARCH.md §Indexed rows: rows shared by every workgroup (L2), chip-wide
METRIC_NAME = "edges/sec + achieved HBM GB/s, GAT aggregate on Reddit, 1/2/4/8 MI355X"
CALIB_ROWS = 1 << 21      # known-byte gather for the FETCH_SIZE calibration: 2 M rows x 512 B = 1 GiB table


def log(rank, msg):
    print(f"[bench rank {rank}] {time.strftime('%H:%M:%S')} {msg}", file=sys.stderr, flush=True)


def make_inputs(n=N_REDDIT, e=E_REDDIT, dev=None):
    """(graph, X1, alpha) of the whole metric workload on one device (the probe scripts' entry)."""
    sh = metric.Shard(n, e, 0, 1, 1, 1, dev or torch.device("cuda", 0), keep_rows=False)
    return sh.graph, sh.x, sh.alpha


alg_bytes = metric.alg_bytes
auto_blocks = ops.BlockedPlan.auto_blocks


# ----------------------------------------------------------------------------------------------
# the timed workload
# ----------------------------------------------------------------------------------------------
class Aggregate:
    """One rank's launches: the aggregate of each destination-row chunk of its tile (column-blocked
    plan per chunk), plus the chunk's collective."""

    def __init__(self, shard, mode, pc, world, blocks, impl, groups, backend, rank):
        self.s, self.mode, self.pc, self.world, self.impl = shard, mode, pc, world, impl
        g = shard.grid
        self.parts = []
        for c in range(g.chunks):
            a, b = g.chunk_rows(c) if mode == "edges" else (c * g.mk, (c + 1) * g.mk)
            gg = shard.graph if g.chunks == 1 else G.Graph(shard.graph.indptr[a:b + 1], shard.graph.indices,
                                                           n_cols=shard.graph.n_cols)
            self.parts.append((a, b, gg))
        dev = shard.graph.indptr.device
        self.blocks = blocks or ops.BlockedPlan.auto_blocks(self.parts[0][2], F)
        if impl == "blocked" and (self.blocks < 4 or not ops.BlockedPlan.supports(F, HEADS)):
            self.impl = "plan"
        for a_, b_, gg in self.parts:
            if b_ <= a_:
                continue  # an empty chunk (a row block smaller than the chunk count): nothing to launch
            if self.impl == "blocked" and not gg.blocked_plan(self.blocks).sorted:
                raise SystemExit("blocked aggregate needs sorted rows")
            if self.impl == "plan":
                gg.plan(512)
        n_pad = shard.graph.n_rows
        self.y = torch.zeros(n_pad, F, device=dev)
        self.backend, self.group = backend, (groups[g.i] if groups else None)
        if mode == "edges":
            self.y_own = self.y if pc == 1 else torch.zeros(g.out_rows(), F, device=dev)
        else:  # rows: every rank's chunk parts gathered into the padded full table [C * world * mk, F]
            self.y_own = self.y
            self.y_full = torch.zeros(g.chunks * world * g.mk, F, device=dev) if world > 1 else None
        self.x, self.alpha = shard.x, shard.alpha

    def launch(self, c):
        a, b, gg = self.parts[c]
        if b <= a:
            return
        if self.impl == "blocked":
            ops.aggregate_blocked(gg, self.x, self.alpha, out=self.y[a:b], blocks=self.blocks)
        else:
            ops.aggregate(gg, self.x, "src", self.alpha, out=self.y[a:b], plan=512)

    def step(self):
        g, works = self.s.grid, []
        for c in range(len(self.parts)):
            self.launch(c)
            a, b, _ = self.parts[c]
            if b <= a:
                continue  # every rank of the row group has the same chunk offsets: all skip it
            if self.mode == "edges" and self.pc > 1:
                p0, p1 = g.part(c)
                own = self.y_own[p0:p1]
                # reduce-scatter among the pc ranks of this row group (RCCL on the GPUs; the gloo
                # rehearsals run the same call)
                works.append(dist.reduce_scatter_tensor(own, self.y[a:b], group=self.group, async_op=True))
            elif self.mode == "rows" and self.world > 1:
                w = self.world * g.mk
                out = self.y_full[c * w:(c + 1) * w]
                works.append(dist.all_gather_into_tensor(out, self.y[a:b], async_op=True))
        for wk in works:
            wk.wait()


def layers_leg(names, world, record, say=print):
    """The 'layers' records.  On one GPU a failing layer is reported in its record and the next one
    runs.  With N > 1 ranks a failure propagates: a rank that caught its own error would
    run on into the next layer's collectives while its peers still wait inside the failed layer's
    exchange -- collectives paired across layers, or a hang until the watchdog; raising lets
    torchrun tear every rank down at once."""
    recs = []
    for name in filter(None, (n.strip() for n in names)):
        say(f"layer {name}")
        if world > 1:
            recs.append(record(name))
        else:
            try:
                recs.append(record(name))
            except Exception as exc:  # reported, not fatal: the metric line stands on its own
                recs.append({"config": name, "n_gpus": world, "error": f"{type(exc).__name__}: {exc}"[:300]})
        say(f"layer {name}: {json.dumps(recs[-1])[:200]}")
    return recs


def grid_of(args, world):
    """(mode, pr, pc) of a world-rank run."""
    mode = "single" if world == 1 else args.mode
    if args.grid != "auto":
        pr, pc = (int(v) for v in args.grid.lower().split("x"))
    else:
        pr, pc = distributed.grid_shape(world, "rows" if mode == "rows" else "edges")
    if pr * pc != world:
        raise SystemExit(f"--grid {pr}x{pc} does not match {world} ranks")
    return mode, pr, pc


def build(args, world, rank, dev, backend, note, col_counts=None):
    """This rank's shard and launches.  col_counts: the whole graph's per-column nnz given directly
    (the PMC child rebuilding one rank's tile with no process group); else all-reduced (world > 1)."""
    mode, pr, pc = grid_of(args, world)
    if mode == "rows" and pc != 1:
        raise SystemExit("--mode rows uses a PRx1 grid")
    # edges mode: the last chunk's reduce-scatter is the exchange left exposed after the last launch,
    # so the chunks shrink toward the end: default three chunks of 55 / 30 / 15 % of the rows, the
    # split whose modelled 8-GPU step degrades least as the link rate falls (6.53x at 64 GB/s per
    # direction, 6.35x at 40; two chunks of 70 / 30: 6.70x and 5.95x; every chunk launch costs
    # 0.02-0.06 ms of compute; per-chunk times of the 4 x 2 tile: profiles/r04/tile_chunks_4x2_r0.log,
    # DESIGN §6).  rows mode: two equal chunks.
    chunks = args.row_chunks or (1 if world == 1 else (3 if mode == "edges" and pc > 1 else 2))
    fracs = None
    if mode == "edges" and pc > 1 and chunks > 1:
        cf = getattr(args, "chunk_fracs", "auto")
        if cf == "auto":
            fracs = {2: [0.7, 0.3], 3: [0.55, 0.3, 0.15]}.get(chunks)
        elif cf != "equal":
            fracs = [float(v) for v in cf.split(",")]
    count_reduce = None
    if world > 1 and col_counts is None:
        def count_reduce(t):
            dist.all_reduce(t)
            return t
    if mode == "rows":  # every rank's chunk parts must have one size for the all-gather: pad to the largest group
        shard = metric.Shard(args.n, args.e, rank, pr, 1, chunks, dev, count_reduce=count_reduce, note=note)
        mk_all = max(-(-(b - a) // chunks) for a, b in zip(shard.rcuts[:-1], shard.rcuts[1:]))
        if shard.grid.mk != mk_all:
            shard.grid.mk = mk_all
            ip = shard.graph.indptr
            n_pad = chunks * mk_all
            ip2 = torch.full((n_pad + 1,), int(ip[-1]), dtype=ip.dtype, device=ip.device)
            ip2[:ip.numel()] = ip
            shard.graph = shard.grid.graph = G.Graph(ip2, shard.graph.indices, n_cols=shard.graph.n_cols)
    else:
        shard = metric.Shard(args.n, args.e, rank, pr, pc, chunks, dev, count_reduce=count_reduce, note=note,
                             fracs=fracs, col_counts=col_counts)
    groups = None
    if mode == "edges" and pc > 1:  # the row groups' sub-groups (none for a tile rebuilt alone: backend "none")
        groups = distributed.row_groups(pr, pc) if pr > 1 and backend != "none" else [None] * pr
    agg = Aggregate(shard, mode, pc, world, args.blocks, args.impl, groups, backend, rank)
    return shard, agg, mode, pr, pc, chunks


# ----------------------------------------------------------------------------------------------
# PMC traffic (rocprofv3 --pmc on this very bench, child processes started before the GPU is used)
# ----------------------------------------------------------------------------------------------
def pmc_child(args):
    """Runs under rocprofv3 --pmc: the known-byte calibration launches, then this rank's metric
    launches (its own tile, rebuilt alone: at N > 1 the column cuts come from metric.column_counts,
    the same whole-graph histogram the distributed run all-reduces).  Writes the tile's known
    stream sizes (edges, items) and launch pairs per step to <pmc dir>/meta.json."""
    world, rank = args.pmc_world, args.pmc_rank
    dev = torch.device("cuda", args.pmc_local)
    torch.cuda.set_device(dev)
    n = CALIB_ROWS
    # streaming calibration: a float4 copy of a 1 GiB table (k_apply_node4, 16-B lanes, read once, written once)
    xc = torch.ones(n, F, device=dev)
    yc = torch.empty(n, F, device=dev)
    for _ in range(2):
        ops.apply_node(None, None, xc, out=yc)
    # gather calibration: a permutation gather (1 edge per row, every X row read once, 1 GiB table >
    # Infinity Cache), 32 lanes x float4 per 512-B row as k_agg_h32 reads them
    ip = torch.arange(n + 1, device=dev, dtype=torch.int64)
    perm = torch.argsort(G.hash32(torch.arange(n, device=dev, dtype=torch.int64), 7, 9)).to(torch.int32)
    gc = G.Graph(ip, perm)
    ops.set_debug("agg_lpe", 32)
    try:
        for _ in range(2):
            ops.aggregate(gc, xc, "src", None, out=yc)
    finally:
        ops.set_debug("agg_lpe", 0)
    torch.cuda.synchronize()
    del xc, yc, gc, ip, perm
    col_counts = None
    if world > 1 and grid_of(args, world)[2] > 1:
        col_counts = metric.column_counts(args.n, args.e, dev)
    shard, agg, *_ = build(args, world, rank, dev, "none", lambda m: None, col_counts=col_counts)
    del col_counts
    live = [c for c, (a, b, _) in enumerate(agg.parts) if b > a]
    for _ in range(args.steps):
        for c in live:
            agg.launch(c)
    torch.cuda.synchronize()
    if args.pmc_meta:
        items = sum(agg.parts[c][2].blocked_plan(agg.blocks).n_items for c in live) if agg.impl == "blocked" else 0
        with open(args.pmc_meta, "w") as fh:
            json.dump({"nnz": int(shard.graph.nnz), "n_rows": int(shard.graph.n_rows), "heads": HEADS,
                       "n_items": int(items), "pairs_per_step": len(live), "rank": rank, "world": world}, fh)
    return 0


def _counter_rows(d, counter):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") == counter:
                did = row.get("Dispatch_Id") or row.get("Correlation_Id") or "0"
                rows.append((int(did), row.get("Kernel_Name", ""), float(row["Counter_Value"])))
    rows.sort()
    return rows


def _split(rows, per_step=1):
    """-> (stream calibration dispatches, gather calibration dispatches, [(agg, reduce)] per step)
    from ordered counter rows: a step's launch pairs (one per non-empty row chunk of the tile) summed."""
    copy, gather, pairs, cur = [], [], [], None
    for _, name, v in rows:
        if "k_agg_h32" in name or "k_agg_seg" in name:
            cur = [v, 0.0]
        elif "k_seg_reduce" in name and cur is not None:
            cur[1] = v
            pairs.append(tuple(cur))
            cur = None
        elif "k_apply_node4" in name and not pairs and cur is None:
            copy.append(v)
        elif "k_aggregate" in name and not pairs and cur is None:
            gather.append(v)
    k = max(1, per_step)
    steps = [(sum(a for a, _ in pairs[i:i + k]), sum(b for _, b in pairs[i:i + k]))
             for i in range(0, len(pairs) - k + 1, k)]
    return copy, gather, steps


def _run_group(cmd, env, timeout):
    """Run cmd in its own session; on timeout kill the whole process group (rocprofv3 and its
    child).  -> (returncode or None on timeout, stderr tail)."""
    p = subprocess.Popen(cmd, env=env, cwd=ROOT, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                         start_new_session=True)
    try:
        _, err = p.communicate(timeout=timeout)
        return p.returncode, err[-400:]
    except subprocess.TimeoutExpired:
        try:
            os.killpg(p.pid, signal.SIGKILL)
        except OSError:
            pass
        p.communicate()
        return None, ""


def collect_pmc(args, out_dir, world=1, rank=0, local=0):
    """Two rocprofv3 --pmc passes over `bench.py --pmc-child` on this rank's own tile (FETCH_SIZE,
    WRITE_SIZE; separate passes: TCC slots), run before this process touches the GPU.  The TCC
    counters are device-wide, so children sharing a device (a one-GPU rehearsal of N ranks) take
    turns on a per-device lock file.  Returns the per-step traffic record, or {"error": ...}."""
    exe = shutil.which("rocprofv3")
    if not exe:
        return {"error": "rocprofv3 not found"}
    os.makedirs(out_dir, exist_ok=True)
    env = dict(os.environ, TMPDIR=os.environ.get("TMPDIR", "/tmp"))
    meta_path = os.path.join(out_dir, "meta.json")
    lock = open(os.path.join(tempfile.gettempdir(), f"gta_bench_pmc_dev{local}.lock"), "w")
    fcntl.flock(lock, fcntl.LOCK_EX)
    try:
        res = {}
        for counter in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(out_dir, counter.lower())
            shutil.rmtree(d, ignore_errors=True)
            cmd = [exe, "--kernel-trace", "--pmc", counter, "--output-format", "csv", "-d", d, "-o", "run", "--",
                   sys.executable, os.path.abspath(__file__), "--pmc-child", "--steps", "3", "--pmc-meta", meta_path,
                   "--pmc-world", str(world), "--pmc-rank", str(rank), "--pmc-local", str(local),
                   "--mode", args.mode, "--grid", args.grid, "--row-chunks", str(args.row_chunks),
                   "--chunk-fracs", args.chunk_fracs,
                   "--n", str(args.n), "--e", str(args.e), "--blocks", str(args.blocks), "--impl", args.impl,
                   "--knobs", args.knobs]
            t0 = time.time()
            rc, err = _run_group(cmd, env, 240)
            if rc is None:
                return {"error": f"rocprofv3 --pmc {counter} timed out"}
            if rc != 0:
                return {"error": f"rocprofv3 --pmc {counter} rc={rc}: {err}"}
            try:
                meta = json.load(open(meta_path))
            except (OSError, ValueError):
                return {"error": "pmc child wrote no plan metadata"}
            if meta.get("pairs_per_step", 1) == 0:
                return {"error": "this rank's tile has no edges: no launches to count"}
            copy, gather, steps = _split(_counter_rows(d, counter), meta.get("pairs_per_step", 1))
            if not copy or not gather or not steps:
                return {"error": f"{counter}: no calibration/metric dispatches in {d}"}
            steps = steps[1:] if len(steps) > 1 else steps   # the first step runs on cold caches
            res[counter] = {"copy_kb": copy[-1], "gather_kb": gather[-1],
                            "agg_kb": float(np.mean([a for a, _ in steps])),
                            "reduce_kb": float(np.mean([b for _, b in steps])), "launches": len(steps),
                            "pass_s": round(time.time() - t0, 1)}
    finally:
        fcntl.flock(lock, fcntl.LOCK_UN)
        lock.close()
    return pmc_traffic(res, meta)


def pmc_traffic(res, meta, n=CALIB_ROWS):
    """Per-step bytes (a step = the tile's launch pairs, one per non-empty row chunk; one pair on one
    GPU) from the counter means (res[counter][...] in KB) and the tile's plan metadata:
      read factors   kr_s = copy bytes read / copy FETCH; kr_g = permutation-gather X bytes / (gather
                     FETCH - its index + indptr streams / kr_s); write factor kw = copy bytes / copy WRITE
      k_agg_h32      streams S = 4 E (indices) + 4 H E (alpha) + 16 items (item records), read once;
                     gathers = (FETCH - S / kr_s) * kr_g; + WRITE * kw (partial rows)
      k_seg_reduce   FETCH * kr_s (partial rows, item lists) + WRITE * kw (y)
    Why kr_s is ~2: FETCH_SIZE = TCC_EA0_RDREQ x 64 B, and a wide streaming read leaves L2 as 128-B
    requests tallied at 64 B (MI355X_MICROARCH.md §HBM); the copy measures it on this box, in this pass.
    The bytes are memory-side (L2 <-> fabric): Infinity-Cache hits are counted, so they bound the
    HBM bytes from above.  Recomputable from the committed CSVs (profiles/r0*/pmc_*)."""
    fe, wr = res["FETCH_SIZE"], res["WRITE_SIZE"]
    kb = 1024.0
    copy_bytes = n * 4 * F
    kr_s = copy_bytes / (fe["copy_kb"] * kb)
    kw = copy_bytes / (wr["copy_kb"] * kb)
    g_stream = n * 4 + (n + 1) * 8                   # permutation gather: col idx + indptr
    kr_g = copy_bytes / (fe["gather_kb"] * kb - g_stream / kr_s)
    E, H, items = meta["nnz"], meta["heads"], meta["n_items"]
    streams = 4.0 * E + 4.0 * H * E + 16.0 * items
    gathers = (fe["agg_kb"] * kb - streams / kr_s) * kr_g
    agg = streams + gathers + wr["agg_kb"] * kb * kw
    red = fe["reduce_kb"] * kb * kr_s + wr["reduce_kb"] * kb * kw
    return {"bytes_per_launch": agg + red, "agg_bytes": agg, "reduce_bytes": red,
            "agg_split": {"streams": streams, "gathers": gathers, "writes": wr["agg_kb"] * kb * kw},
            "read_factor_stream": kr_s, "read_factor_gather": kr_g, "write_factor": kw, "meta": meta,
            "passes": res,
            "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) on this bench's own launches; "
                      "read factors calibrated in the same pass: streaming (kr_s, float4 copy of a 1 GiB table) "
                      "and gathered 512-B rows (kr_g, permutation gather with 16-B lanes, its index streams "
                      "taken out at kr_s); k_agg_h32 = known streams (indices, alpha, item records) + "
                      "(FETCH - streams/kr_s)*kr_g + WRITE*kw; k_seg_reduce = FETCH*kr_s + WRITE*kw; "
                      "counts L2<->fabric bytes (Infinity-Cache hits included); first step skipped",
            "traffic_side": "memory side of L2 (TCC_EA0 requests): HBM + Infinity-Cache hits, an upper bound "
                            "on HBM bytes; kr_s ~ 2 because FETCH_SIZE tallies a 128-B streaming request "
                            "at 64 B (MI355X_MICROARCH.md §HBM), measured in the same pass"}


# ----------------------------------------------------------------------------------------------
# oracle leg: parity of sampled rows (fp64) and the CPU baseline (TEST ORACLE, outside the timed region)
# ----------------------------------------------------------------------------------------------
def oracle_parity(shard, y_own, owned, k=256):
    from oracle import isa_ref
    s = shard.sample_rows(y_own, owned, k=k)
    if s is None:
        return 0.0, 0.0, 0
    ref = isa_ref.aggregate(s["indptr"], s["indices"], s["x"], "src", s["alpha"])
    bound = 1e-5 * isa_ref.aggregate_abs(s["indptr"], s["indices"], s["x"], "src", s["alpha"]) + 1e-6
    err = np.abs(s["y"].astype(np.float64) - ref)
    return float((err / bound).max()), float(err.max()), len(s["rows"])


def gin_bf16_accuracy(dev, n_random=64):
    """gin-products' bf16 storage choice (x, W5, W7 in bf16) against fp64 of the UNROUNDED fp32
    inputs at sampled rows (oracle/sampled.gin_unrounded_errors, SURVEY.md §8c rtol 2e-2; the
    full-size test is tests/test_gpu_configs.py::test_gin_products_bf16_vs_fp64_of_unrounded_inputs).
    One eager forward, after the timed layers."""
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import configs, workloads
    from oracle.sampled import SampledChecker, gin_unrounded_errors
    results, g = configs.run("gin-products", dev)
    lay, _, ex = results[0]
    t32 = workloads.make_tensors(lay.opgraph, g, "GIN", seed=0)
    ip, ix = g.numpy()
    chk = SampledChecker(ex, ip, ix)
    sp = np.concatenate(list(chk.special_rows().values()))
    rows = np.unique(np.concatenate([sp, np.random.default_rng(3).choice(g.n_rows, n_random, replace=False)]))
    errs = gin_unrounded_errors(chk, t32, rows)
    return {"check": f"bf16 layer vs fp64 of the unrounded fp32 x / W5 / W7 on {len(rows)} rows "
                     "(special rows + random), per op: max|d| / max|ref|", "rtol": 2e-2,
            "max_rel_err": {f"op{k}": round(v[0], 6) for k, v in errs.items()},
            "max_err_over_terms": {f"op{k}": round(v[1], 6) for k, v in errs.items()},
            "within_rtol": all(v[0] <= 2e-2 and v[1] <= 2e-2 for v in errs.values())}


def cpu_quota():
    """CPUs of the cgroup v2 quota (cpu.max), or None."""
    try:
        q = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q[0] == "max" else int(q[0]) / int(q[1])
    except (OSError, ValueError, IndexError):
        return None


def cpu_baseline(shard, target_s=12.0, repeats=5):
    """Oracle C aggregate (OpenMP) on the first rows of this rank's row group of the same workload
    (median of `repeats` timed runs after one warm-up run), ~target_s of CPU work per
    thread count: every core of sched_getaffinity(0), and -- when a cgroup quota caps the job below
    that -- as many threads as the quota allows.  value / cores = the faster run; both are listed.
    At N > 1 the rank holds only its column slice of X: the sample's X rows are regenerated (every X
    row is a pure function of (seed, id))."""
    from oracle import cbase
    cbase.load()
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    quota = cpu_quota()
    counts = [affinity]
    if quota and int(np.ceil(quota)) < affinity:
        counts.append(int(np.ceil(quota)))
    ip = shard.rows_ip.cpu().numpy()
    ix = shard.rows_src.to(torch.int32).cpu().numpy()
    if shard.x.shape[0] >= shard.n:
        xh = shard.x.cpu().numpy()
    else:
        xh = metric.x_rows(torch.arange(shard.n), shard.x.device, shard.seed).cpu().numpy()
    ah = shard.rows_alpha
    n = len(ip) - 1
    a_cache = {}

    def run(rows, threads):
        e1 = int(ip[rows])
        if e1 not in a_cache:
            a_cache.clear()
            a_cache[e1] = ah[:e1].cpu().numpy()
        t0 = time.perf_counter()
        cbase.aggregate(ip[: rows + 1], ix[:e1], xh, a_cache[e1], 0, rows, threads=threads)
        return time.perf_counter() - t0, e1

    runs = []
    for threads in counts:
        rows = min(n, 2000)
        dt, ecount = run(rows, threads)  # rate probe
        rate = ecount / max(dt, 1e-6)
        want_edges = min(int(rate * target_s / (repeats + 1)), int(ip[-1]))
        rows = int(min(n, max(1, np.searchsorted(ip, want_edges))))
        run(rows, threads)               # warm-up
        times = [run(rows, threads)[0] for _ in range(repeats)]
        ecount = int(ip[rows])
        runs.append({"threads": threads, "value": ecount / float(np.median(times)), "rows": rows, "edges": ecount,
                     "times_s": [round(t, 4) for t in times]})
    best = max(runs, key=lambda r: r["value"])
    r0 = shard.rcuts[shard.grid.i]
    return {"value": best["value"], "unit": "edges/s", "cores": best["threads"], "kind": "port",
            "sample": f"destination rows [{r0},{r0 + best['rows']}) = {best['edges']} edges of the same graph/X/alpha, "
                      f"median of {repeats} after 1 warm-up, oracle/spmm_ref.c fp32 OpenMP; sched_getaffinity = "
                      f"{affinity} cores, cgroup quota = {quota} CPUs; runs: "
                      + ", ".join(f"{r['threads']} threads {r['value'] / 1e6:.1f} M edges/s" for r in runs),
            "affinity_cores": affinity, "runs": runs}


def rank_roofline(per_rank, peak=PEAK_HBM_GBS):
    """Roofline fields from every rank's measurements (a list of dicts: rank, tile_edges, tile_rows,
    compute_ms = HIP-event time of the tile's launches alone, step_ms = the rank's own step time
    before the closing barrier, traffic = PMC bytes per step or None).  The headline fields are the
    critical rank's -- the one with the longest compute, which bounds the step; exposed_exchange_ms
    = step_ms - compute_ms per rank (collectives not hidden under compute, plus launch gaps)."""
    rows = []
    for s in per_rank:
        t = s.get("traffic")
        t = None if t is None or not np.isfinite(t) else float(t)
        ach = None if t is None else t / (s["compute_ms"] / 1e3) / 1e9
        rows.append({"rank": int(s["rank"]), "tile_edges": int(s["tile_edges"]), "tile_rows": int(s["tile_rows"]),
                     "compute_ms": s["compute_ms"], "step_ms": s["step_ms"],
                     "exposed_exchange_ms": max(0.0, s["step_ms"] - s["compute_ms"]),
                     "traffic": t, "achieved": ach, "frac": None if ach is None else ach / peak})
    crit = max(rows, key=lambda r: r["compute_ms"])
    fr = [r["frac"] for r in rows if r["frac"] is not None]
    tot = [r["traffic"] for r in rows]
    job = sum(tot) / (crit["compute_ms"] / 1e3) / 1e9 if all(v is not None for v in tot) else None
    return {"achieved": crit["achieved"], "frac": crit["frac"], "traffic": crit["traffic"],
            "kernel_ms": crit["compute_ms"], "rank_basis": crit["rank"],
            "frac_min": min(fr) if fr else None, "frac_max": max(fr) if fr else None,
            "job_achieved_GBps": job, "job_peak_GBps": peak * len(rows),
            "per_rank": rows}


# ----------------------------------------------------------------------------------------------
def main():
    if os.environ.get("GTA_STALL_DUMP"):  # diagnostics: every rank prints its Python stack every S seconds
        import faulthandler
        faulthandler.dump_traceback_later(float(os.environ["GTA_STALL_DUMP"]), repeat=True, file=sys.stderr)
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--mode", choices=["edges", "rows"], default="edges",
                    help="N>1: edges = 2-D edge tiles + RCCL reduce-scatter of partial aggregates (north star); "
                         "rows = destination-row tiles + RCCL all-gather of Y")
    ap.add_argument("--grid", default="auto", help="PRxPC rank grid (auto: 1x2, 2x2, 4x2; rows: Nx1)")
    ap.add_argument("--row-chunks", type=int, default=0, help="row chunks per tile for comm overlap (0 = auto)")
    ap.add_argument("--chunk-fracs", default="auto",
                    help="edges mode: relative row-chunk sizes, e.g. 0.7,0.3 ('equal'; 'auto' = 0.55,0.3,0.15 for "
                         "three, the default count, and 0.7,0.3 for two)")
    ap.add_argument("--impl", choices=["blocked", "plan"], default="blocked")
    ap.add_argument("--blocks", type=int, default=0, help="column blocks (0 = auto, ~6 MB X slices)")
    ap.add_argument("--n", "--graph-nodes", dest="n", type=int, default=N_REDDIT)
    ap.add_argument("--e", "--graph-edges", dest="e", type=int, default=E_REDDIT)
    ap.add_argument("--parity-rows", type=int, default=256, help="sampled rows per rank for the fp64 oracle")
    ap.add_argument("--layers", default="auto",
                    help="BASELINE-config layers timed after the metric at the same N (destination-row shards; "
                         "'none' to skip; 'auto': every BASELINE config on one GPU -- GCN Cora, GAT-8 Flickr, "
                         "GraphSAGE Reddit, GIN products -- and the two multi-GPU ones at N > 1): the 'layers' field")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-s", type=float, default=12.0,
                    help="CPU work per thread count of the cpu_baseline leg (seconds, approx.)")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 --pmc traffic passes")
    ap.add_argument("--pmc-dir", default="", help="keep the --pmc CSVs here (default: a temp dir)")
    ap.add_argument("--knobs", default="", help="libgta tuning knobs for every launch, e.g. seg_lean=0,mm_ring=0 "
                                               "(also passed to the PMC children)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--pmc-meta", default="", help=argparse.SUPPRESS)
    ap.add_argument("--pmc-world", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--pmc-rank", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--pmc-local", type=int, default=0, help=argparse.SUPPRESS)
    args = ap.parse_args()
    for kv in filter(None, args.knobs.split(",")):
        k, v = kv.split("=")
        ops.set_debug(k.strip(), int(v))
    if args.pmc_child:
        return pmc_child(args)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    backend = os.environ.get("GTA_DIST_BACKEND", "nccl")   # gloo: CPU / one-GPU rehearsals
    if os.environ.get("GTA_SINGLE_DEVICE"):
        local = 0

    # PMC passes first: child processes on this rank's own tile, before this process initialises the GPU
    pmc = None
    if not args.no_pmc:
        log(rank, "rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) on this rank's kernels")
        if args.pmc_dir:
            keep = args.pmc_dir if world == 1 else os.path.join(args.pmc_dir, f"rank{rank}")
        else:
            keep = tempfile.mkdtemp(prefix=f"gta_pmc_r{rank}_")
        pmc = collect_pmc(args, keep, world, rank, local)
        if not args.pmc_dir:
            shutil.rmtree(keep, ignore_errors=True)
        log(rank, f"pmc: {json.dumps({k: v for k, v in pmc.items() if k != 'passes'})[:300]}")

    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        # the ranks of this node share its CPUs: host-side torch ops (graph generation, the gloo
        # rehearsals' staging) with every rank at the full OMP count oversubscribe them -- an 8-rank
        # one-GPU rehearsal at 16 threads each on a 16-CPU quota stalled for minutes in shard building
        cpus = cpu_quota() or len(os.sched_getaffinity(0))
        torch.set_num_threads(max(1, int(cpus) // int(os.environ.get("LOCAL_WORLD_SIZE", world))))
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        log(rank, f"process group up: backend {dist.get_backend()}, world {dist.get_world_size()}")

    t_build = time.time()
    shard, agg, mode, pr, pc, chunks = build(args, world, rank, dev, backend, lambda m: log(rank, m))
    torch.cuda.synchronize()
    log(rank, f"inputs + plans ready in {time.time() - t_build:.1f} s: mode {mode}, grid {pr}x{pc}, "
              f"{chunks} row chunks, impl {agg.impl}, B={agg.blocks}")

    for _ in range(args.warmup):
        agg.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    log(rank, "warmup done, timing")

    # kernel-only timing (HIP events on the launch stream) for the roofline
    stream = torch.cuda.current_stream(dev)
    n_evt = min(max(args.steps, 1), 10)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n_evt)]
    for a, b in evs:
        a.record(stream)
        for c in range(len(agg.parts)):
            agg.launch(c)
        b.record(stream)
    torch.cuda.synchronize()
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    # the same launches split by phase (knob seg_phase: 1 = the gather items only, 2 = the ordered
    # reduce only, reading the slabs the items just wrote): per-kernel times for the roofline
    phase_ms = None
    if agg.impl == "blocked":
        pev = {1: [], 2: []}
        try:
            for _ in range(n_evt):
                for ph in (1, 2):
                    ops.set_debug("seg_phase", ph)
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(stream)
                    for c in range(len(agg.parts)):
                        agg.launch(c)
                    b.record(stream)
                    pev[ph].append((a, b))
        finally:
            ops.set_debug("seg_phase", 0)
        torch.cuda.synchronize()
        phase_ms = {ph: float(np.mean([a.elapsed_time(b) for a, b in v])) for ph, v in pev.items()}

    # timed region: K steps, barrier + sync on both sides, max over ranks
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        agg.step()
    torch.cuda.synchronize()
    own_ms = (time.perf_counter() - t0) * 1e3 / args.steps   # this rank's own step, before the closing barrier
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = dt * 1e3 / args.steps
    value = args.e / (ms_per_step / 1e3)
    log(rank, f"timed: {ms_per_step:.3f} ms/step (own {own_ms:.3f}, kernels alone {kern_ms:.3f})")

    # parity: this rank's own output rows (complete sums after the exchange) vs the fp64 oracle
    agg.step()
    torch.cuda.synchronize()
    g = shard.grid
    if mode == "rows" and world > 1:   # check rows taken from the gathered full table (what the next layer reads)
        w_ = world * g.mk
        part = torch.cat([agg.y_full[c * w_ + rank * g.mk:c * w_ + (rank + 1) * g.mk] for c in range(g.chunks)])
        owned = torch.arange(g.chunks * g.mk) + g.r0
        owned = torch.where(owned < g.r1, owned, torch.full_like(owned, -1))
        ratio, max_err, n_rows = oracle_parity(shard, part, owned, args.parity_rows)
    else:
        ratio, max_err, n_rows = oracle_parity(shard, agg.y_own, g.owned_rows(rank), args.parity_rows)
    if world > 1:
        t = torch.tensor([ratio, max_err, float(n_rows)], device=dev, dtype=torch.float64)
        t2 = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(t2, op=dist.ReduceOp.SUM)
        ratio, max_err, n_rows = float(t[0]), float(t[1]), int(t2[2])
    parity = {"check": f"fp64 oracle (oracle/isa_ref.aggregate) on {n_rows} sampled output rows "
                       f"({args.parity_rows} per rank incl. heaviest/lightest; after the exchange)",
              "bound": "|err| <= 1e-5 * sum|terms| + 1e-6 per element", "max_err_over_bound": ratio,
              "max_abs_err": max_err, "ok": bool(ratio <= 1.0)}
    log(rank, f"parity: {parity}")

    # roofline of the dominant kernel pair: every rank's tile launches (compute alone), its own step
    # time and its PMC bytes, gathered on every rank; the critical (longest-compute) rank's in front
    traffic = pmc["bytes_per_launch"] if pmc is not None and "error" not in pmc else float("nan")
    mine = [rank, shard.graph.nnz, g.r1 - g.r0 if world > 1 else shard.graph.n_rows, kern_ms, own_ms, traffic,
            phase_ms[1] if phase_ms else float("nan"), phase_ms[2] if phase_ms else float("nan")]
    stats = torch.zeros(world, len(mine), dtype=torch.float64, device=dev)
    stats[rank] = torch.tensor(mine, dtype=torch.float64)
    if world > 1:
        dist.all_reduce(stats)
    stats = stats.cpu().tolist()
    per_rank = [{"rank": r[0], "tile_edges": r[1], "tile_rows": r[2], "compute_ms": r[3], "step_ms": r[4],
                 "traffic": r[5], "agg_ms": r[6], "reduce_ms": r[7]} for r in stats]
    rr = rank_roofline(per_rank)
    for row, s_ in zip(rr["per_rank"], per_rank):
        row.update({"k_agg_h32_ms": s_["agg_ms"], "k_seg_reduce_ms": s_["reduce_ms"]})
    crit = rr["per_rank"][rr["rank_basis"]]
    log(rank, "per rank: " + "; ".join(f"r{r['rank']} compute {r['compute_ms']:.3f} step {r['step_ms']:.3f} "
                                       f"exposed {r['exposed_exchange_ms']:.3f} ms frac {r['frac']}"
                                       for r in rr["per_rank"]))
    ab = metric.alg_bytes(crit["tile_rows"], crit["tile_edges"])
    alg_gbps = ab / (crit["compute_ms"] / 1e3) / 1e9
    roof = {"bound": "hbm", "achieved": rr["achieved"], "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": rr["frac"],
            # what `traffic` / `frac` count -- no counter on this pool splits HBM from
            # Infinity-Cache hits, so frac is an upper bound on the HBM fraction
            "bytes_side": "fabric side of L2 (L2 misses: HBM reads + Infinity-Cache hits + writes); "
                          "frac = those bytes / time / HBM peak, an upper bound on the HBM fraction",
            "traffic": rr["traffic"], "kernel_ms": rr["kernel_ms"],
            "kernels": "k_agg_h32 + k_seg_reduce" if agg.impl == "blocked" else "k_aggregate + combine",
            "rank_basis": rr["rank_basis"], "frac_min": rr["frac_min"], "frac_max": rr["frac_max"],
            "job_achieved_GBps": rr["job_achieved_GBps"], "job_peak_GBps": rr["job_peak_GBps"],
            "alg_bytes_per_launch": ab, "alg_GBps": alg_gbps, "frac_l2": alg_gbps / L2_GATHER_GBS,
            "l2_gather_peak_GBps": L2_GATHER_GBS,
            "compulsory_bytes": metric.compulsory_bytes(args.n, args.n, args.e) if world == 1 else None,
            "per_rank": rr["per_rank"]}
    if pmc is not None:
        if "error" in pmc:
            roof["pmc_error"] = pmc["error"]
        else:
            roof["traffic_split"] = {"agg": pmc["agg_bytes"], "reduce": pmc["reduce_bytes"],
                                     "agg_split": pmc["agg_split"],
                                     "read_factor_stream": pmc["read_factor_stream"],
                                     "read_factor_gather": pmc["read_factor_gather"],
                                     "write_factor": pmc["write_factor"], "rank": rank}
            roof["pmc_counters_kb"] = pmc["passes"]
            roof["pmc_meta"] = pmc["meta"]
            roof["traffic_method"] = pmc["method"]
            roof["traffic_side"] = pmc["traffic_side"]
            if phase_ms is not None:  # each kernel alone: its PMC bytes over its own HIP-event time (rank 0)
                roof["per_kernel"] = {
                    name: {"ms": phase_ms[ph], "traffic": byt, "achieved": byt / (phase_ms[ph] / 1e3) / 1e9,
                           "frac": byt / (phase_ms[ph] / 1e3) / 1e9 / PEAK_HBM_GBS}
                    for name, ph, byt in (("k_agg_h32", 1, pmc["agg_bytes"]), ("k_seg_reduce", 2, pmc["reduce_bytes"]))}

    if mode == "single":
        par = "one GPU, whole graph"
    elif mode == "edges":
        par = (f"edge partition: {pr}x{pc} grid of row-group x source-column tiles (tile-metadata nnz cuts), "
               f"RCCL reduce-scatter of partial vertex aggregates in each row group, {chunks} overlapped row chunks")
    else:
        par = f"destination-row tiles x{pr} + RCCL all-gather of Y, {chunks} overlapped row chunks"
    result = {
        "metric": METRIC_NAME, "value": value, "unit": "edges/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": ms_per_step, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32",
        "data": "synthetic, counter-hashed: lognormal-degree CSR (mean deg 492), uniform sources, X~N(0,1), "
                "alpha=per-head softmax over in-edges of N(0,1) logits",
        "config": {"workload": "GAT layer-1 aggregate block [3,11,12] (scatter C -> applyedge MUL -> gather ADD)",
                   "graph": "reddit-shaped", "N": args.n, "E": args.e, "F": F, "heads": HEADS,
                   "parallelism": par, "mode": mode, "grid": f"{pr}x{pc}", "row_chunks": chunks,
                   "chunk_rows": shard.grid.mks if mode == "edges" else None,
                   "impl": agg.impl, "blocks": agg.blocks if agg.impl == "blocked" else None,
                   "world_size_seen": dist.get_world_size() if world > 1 else 1,
                   "backend": (dist.get_backend() if world > 1 else None)},
        "achieved_GBps": roof["achieved"],
        "parity": parity,
        "roofline": roof,
    }
    # whole BASELINE-config layers at the same N (configs #4 / #5: GraphSAGE Reddit, GIN products), every
    # rank, after the metric (secondary numbers: the metric above is the headline)
    if args.layers and args.layers != "none":
        del agg
        torch.cuda.empty_cache()
        names = args.layers.split(",")
        if args.layers == "auto":  # BASELINE.json configs #1-#4; #1 / #2 are one-GPU configs
            names = (["gcn-cora", "gat8-flickr"] if world == 1 else []) + ["sage-reddit", "gin-products"]
        result["layers"] = layers_leg(names, world,
                                      lambda name: distributed.layer_record(name, dev, rank, world, reps=3,
                                                                            backend=backend),
                                      lambda msg: log(rank, msg))
        for rec in result["layers"]:  # the bf16 choice's accuracy beside its time
            if rec.get("config") == "gin-products" and world == 1 and "error" not in rec:
                try:
                    rec["bf16_vs_fp64_unrounded"] = gin_bf16_accuracy(dev)
                except Exception as exc:  # reported, not fatal
                    rec["bf16_vs_fp64_unrounded"] = {"error": f"{type(exc).__name__}: {exc}"[:300]}
                log(rank, f"gin-products bf16 accuracy: {rec['bf16_vs_fp64_unrounded']}")
                torch.cuda.empty_cache()
    if rank == 0 and not args.no_cpu_baseline:  # after the timed region; other ranks wait at the barrier
        log(rank, "cpu baseline")
        result["cpu_baseline"] = cpu_baseline(shard, target_s=args.cpu_baseline_s)
    elif rank == 0:
        result["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
