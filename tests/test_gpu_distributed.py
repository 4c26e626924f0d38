"""Whole layers on two ranks sharing one MI355X (gloo over HIP tensors), through
scripts/dist_layers.py: destination-row shards (all-gathered source tables, fusions on) and
source-column shards (reduce-scattered gathers).  Rank 0 re-assembles the sink rows and compares
them with a 1-device execution of the same stream on the same inputs."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.gpu
@pytest.mark.parametrize("layout", ["rows", "cols"])
def test_two_rank_layers_match_one_device(layout):
    env = dict(os.environ, GTA_DIST_BACKEND="gloo", GTA_SINGLE_DEVICE="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "scripts", "dist_layers.py"), "gcn-cora", "gat8-flickr", "--reps", "1",
           "--layout", layout]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert [x["config"] for x in recs] == ["gcn-cora", "gat8-flickr"], r.stdout[-2000:]
    for x in recs:
        assert x["n_gpus"] == 2 and x["layout"] == layout
        assert x["max_norm_diff_vs_1dev"] is not None and x["max_norm_diff_vs_1dev"] <= 1e-6, x
        assert x["exchanged_bytes_per_rank"] > 0, x


@pytest.mark.gpu
def test_two_rank_sage_reddit_full_size():
    """GraphSAGE layer 1 on the full Reddit shape (232,965 / 114.6 M edges) on two row shards
    (gloo, both ranks on one GPU): the re-assembled output equals the 1-device stream to fp32
    rounding."""
    env = dict(os.environ, GTA_DIST_BACKEND="gloo", GTA_SINGLE_DEVICE="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "scripts", "dist_layers.py"), "sage-reddit", "--reps", "1", "--layout", "rows"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    recs = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")]
    assert len(recs) == 1 and recs[0]["config"] == "sage-reddit", r.stdout[-2000:]
    x = recs[0]
    # max |d| / max |ref|: the shard runs its own plans (the blocked aggregate's column blocks and item
    # cuts follow the shard's shape, so each row's partial sums are added in another order) -- fp32
    # rounding, far inside the aggregate bar 1e-5 * sum|terms|
    assert x["n_gpus"] == 2 and x["max_norm_diff_vs_1dev"] is not None and x["max_norm_diff_vs_1dev"] <= 1e-5, x


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["edges", "rows"])
def test_two_rank_bench_full_size(mode):
    """bench.py --gpus 2 at the full metric size, both ranks on one GPU over gloo (RCCL cannot
    put two ranks on one device): each rank generates only its shard, the exchange runs, and every
    rank's sampled output rows match the fp64 oracle (the bench's own parity field).  The N > 1 line
    carries what the N = 1 line does: each rank's own PMC bytes (its child rebuilt the
    tile alone) with the critical rank's frac in front, the per-rank compute / exposed-exchange
    split, and the CPU baseline from rank 0."""
    env = dict(os.environ, GTA_DIST_BACKEND="gloo", GTA_SINGLE_DEVICE="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup", "1", "--mode", mode,
           "--parity-rows", "128", "--cpu-baseline-s", "3", "--layers", "gcn-cora"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0, r.stderr[-3000:]
    rec = [json.loads(line) for line in r.stdout.splitlines() if line.startswith("{")][-1]
    assert rec["n_gpus"] == 2 and rec["config"]["mode"] == mode and rec["config"]["world_size_seen"] == 2
    assert rec["config"]["N"] == 232965 and rec["config"]["E"] == 114615892
    assert rec["parity"]["ok"] and rec["parity"]["max_err_over_bound"] <= 1.0, rec["parity"]
    roof = rec["roofline"]
    assert "pmc_error" not in roof, roof.get("pmc_error")
    assert roof["frac"] is not None and 0.05 < roof["frac"] < 1.0, roof
    assert len(roof["per_rank"]) == 2 and sum(p["tile_edges"] for p in roof["per_rank"]) == (
        114615892 if mode == "edges" else sum(p["tile_edges"] for p in roof["per_rank"]))
    for p in roof["per_rank"]:
        assert p["frac"] is not None and p["traffic"] > 0 and p["compute_ms"] > 0
        assert p["exposed_exchange_ms"] >= 0 and p["step_ms"] > 0
    cb = rec["cpu_baseline"]
    assert cb is not None and cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] == "port", cb
    # the whole-layer records at the same N (row shards; GCN Cora keeps the rehearsal short)
    (lay,) = rec["layers"]
    assert "error" not in lay, lay
    assert lay["config"] == "gcn-cora" and lay["n_gpus"] == 2 and lay["ms_per_forward"] > 0
    assert lay["max_norm_diff_vs_1dev"] is not None and lay["max_norm_diff_vs_1dev"] <= 1e-5, lay


@pytest.mark.gpu
def test_rccl_collectives_as_bench_makes_them():
    """RCCL itself (backend "nccl") on the box's GPU: bench.py's reduce-scatter / all-gather /
    all-reduce calls with its chunk-major layouts, in a torch.distributed.run process group of one
    rank per GPU (one GPU here: world 1, the group and the async work handles still go through RCCL)."""
    import torch
    n = torch.cuda.device_count()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(min(n, 2)),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "scripts", "rccl_smoke.py")]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["backend"] == "nccl" and res["reduce_scatter_ok"] and res["all_gather_ok"] and res["all_reduce_ok"]
