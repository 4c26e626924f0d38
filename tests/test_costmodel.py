"""costmodel reproduces the reference simulate() (cycles, rw) exactly (tests/golden/manifest.json)."""
import os

import numpy as np
import pytest

from gta_graph_tensor_acclelrator_for_general_gnn_amd import costmodel, lowering, ir
from oracle import isa_ref


@pytest.fixture(scope="module")
def tiles_for(golden_dir):
    z = np.load(os.path.join(golden_dir, "cora_graph.npz"))
    ip, ix = z["indptr"], z["indices"]
    cache = {}

    def f(T):
        if T not in cache:
            cache[T] = isa_ref.tile_nnz(ip, ix, 2708, T).ravel().tolist()
        return cache[T]
    return f


def test_simulate_goldens(golden_dir, manifest, tiles_for):
    assert len(manifest["simulate"]) >= 3
    for case in manifest["simulate"]:
        net, ds, layer, m = case["key"].split("-")
        records = ir.read_yaml(os.path.join(golden_dir, "ops", f"{net}-{ds}-{layer}-{m}.yaml"))
        blocks = lowering.lower(records, 2708, case["op_array"], case["tile_size_list"])
        cycles, rw = costmodel.simulate_stream(blocks, case["tile_size_list"], 2708, tiles_for)
        assert (cycles, rw) == (case["cycles"], case["rw"]), case["key"]
        e_tiles = int(sum(tiles_for(case["tile_size_list"][0][0])))
        assert costmodel.model_rw(blocks, 2708, e_tiles) == case["rw"]
