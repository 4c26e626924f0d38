"""compiler.search reproduces the reference compile() candidate lists (tests/golden/manifest.json)."""
import os

import pytest

from gta_graph_tensor_acclelrator_for_general_gnn_amd import compiler, ir

from .conftest import load_manifest

CASES = sorted(load_manifest()["compile"].items())


@pytest.mark.parametrize("key,gold", CASES, ids=[k.replace("/", "_") for k, _ in CASES])
def test_candidates_match_reference(golden_dir, manifest, key, gold):
    sizes = manifest["tiles"]["gen_size_64_2708"]
    maxl = manifest["tiles"]["maxlist"]
    if "error" in gold:  # reference raised (GCN-trans: feature_number shorter than its inputs)
        net = key.split("/")[1]
        layer = key.split("-layer")[1][0]
        ops = ir.read_yaml(os.path.join(golden_dir, "ops", f"{net}-cora-layer{layer}-trans.yaml"))
        with pytest.raises(IndexError):
            compiler.search(ops, 2708, sizes, maxl)
        return
    net, ds, layer, m = key.split("-")
    ops = ir.read_yaml(os.path.join(golden_dir, "ops", f"{key}.yaml"))
    res = compiler.search(ops, 2708, sizes, maxl, pingpang=True)
    assert len(res) == gold["n_candidates"]
    got_top = [[list(map(list, r[0])), r[1], r[2], r[3]] for r in res[:8]]
    assert got_top == gold["top"]
    got_last = [[list(map(list, r[0])), r[1], r[2], r[3]] for r in res[-2:]] if res else []
    assert got_last == gold["last"]
