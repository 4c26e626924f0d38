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
