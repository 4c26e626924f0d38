"""The start.py-shaped command line (cli.py; code/start.py:13-62).

CPU: flag parsing, the no-device error, and the whole compile -> stream -> run -> model flow on the
Cora shape with the oracle-backed stand-in kernels (tests/fake_ops.py) in place of libgta; the
modelled numbers must equal costmodel.simulate on the same stream.  GPU: the same flow on libgta."""
import json
import subprocess
import sys

import pytest
import torch

from gta_graph_tensor_acclelrator_for_general_gnn_amd import cli, costmodel, executor, graph as G, tiles

from . import fake_ops


def test_flags_parse_like_start_py_but_false_means_false():
    a = cli.parser().parse_args(["--dataset", "cora", "--network", "GCN"])
    assert (a.isReorder, a.isSinput, a.isPingpang) == (False, False, False)
    assert a.layers == "1,2,3"
    a = cli.parser().parse_args(["--dataset", "cora", "--network", "GAT", "--isReorder", "True",
                                 "--isSinput", "False", "--isPingpang", "1"])
    assert (a.isReorder, a.isSinput, a.isPingpang) == (True, False, True)
    with pytest.raises(SystemExit):
        cli.parser().parse_args(["--dataset", "cora", "--network", "GCN", "--isReorder", "maybe"])
    with pytest.raises(SystemExit):
        cli.parser().parse_args(["--dataset", "imagenet", "--network", "GCN"])


def test_bad_layer_list():
    a = cli.parser().parse_args(["--dataset", "cora", "--network", "GCN", "--layers", "4"])
    with pytest.raises(ValueError, match="layers 1, 2 and 3"):
        cli.run(a, "cpu", log=lambda *_: None)


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-device error")
def test_no_device_is_an_error():
    r = subprocess.run([sys.executable, "-m", "gta_graph_tensor_acclelrator_for_general_gnn_amd", "--dataset", "cora",
                        "--network", "GCN"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and "no HIP device" in r.stderr


@pytest.mark.parametrize("network,reorder", [("GCN", False), ("GAT", True), ("GIN", False)])
def test_flow_on_cora_shape_with_stand_in_kernels(monkeypatch, network, reorder):
    for mod in (executor, tiles):  # the kernels; workloads' table layout (ops.pitched) is plain torch
        monkeypatch.setattr(mod, "ops", fake_ops)
    lines = []
    a = cli.parser().parse_args(["--dataset", "cora", "--network", network, "--layers", "1,2",
                                 "--isReorder", str(reorder), "--isPingpang", "True", "--reps", "1"])
    out = cli.run(a, "cpu", log=lines.append)
    text = "\n".join(lines)
    for phase in ("Starting compilation...", "Compilation Done", "Inst Generated", "Simulation Done",
                  "Latency:", "总访存量:"):
        assert phase in text
    assert f"Test Name: cora-{network}-{'Reorder' if reorder else 'Original'}" in text
    assert [r["layer"] for r in out["layers"]] == [1, 2]
    assert out["N"] == 2708 and out["feature"] == 1433
    # the modelled numbers are simulate()'s for each layer's own stream (the cycle loop restated)
    g = G.dataset_graph("cora", seed=0)
    tot_c = tot_rw = 0
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import pipeline
    for r in out["layers"]:
        lay = pipeline.Layer(network, r["layer"], g, 1433, reorder=reorder, op_array=r["blocks"],
                             tile_size_list=r["tiles"])
        try:
            c, rw = costmodel.simulate_stream(lay.stream_records, lay.tile_size_list, g.n_rows,
                                              executor._tiles_for(g, sparse=False), False,
                                              executor.SPARSITY.get("cora", 1))[:2]
        except RuntimeError:  # the cycle loop does not end on this stream: the CLI reports traffic only
            c, rw = None, r["model_rw"]
        tot_c = None if c is None or tot_c is None else tot_c + c
        tot_rw += rw
        assert r["model_rw"] == rw
    assert out["model_cycles"] == tot_c and out["model_rw"] == tot_rw
    if tot_c is None:
        assert "no modelled latency" in text
    json.dumps(out, default=str)


@pytest.mark.gpu
def test_cli_runs_on_gpu():
    r = subprocess.run([sys.executable, "-m", "gta_graph_tensor_acclelrator_for_general_gnn_amd", "--dataset", "cora",
                        "--network", "GCN", "--layers", "1,2", "--json"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["test_name"] == "cora-GCN-Original" and out["model_cycles"] > 0 and out["model_rw"] > 0
    assert 0 < out["measured_ms"] < 1e3
