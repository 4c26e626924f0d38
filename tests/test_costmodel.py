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


# ---- f4: the per-instruction model (rw_record / timeline), pinned to the reference's own records ----
import json  # noqa: E402
import time  # noqa: E402

from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, tiles  # noqa: E402

from .conftest import GOLDEN  # noqa: E402

RECORDS = json.load(open(os.path.join(GOLDEN, "simulate_records.json")))


@pytest.mark.parametrize("case", RECORDS, ids=[c["key"] for c in RECORDS])
def test_per_instruction_records_match_reference(golden_dir, tiles_for, case):
    """Every instruction's rw_record bytes / record count / edge-tile nnz, its timeline entries and
    busy cycles, its first start and last end, and the reference's per-type aggregates
    (aggregate_rw_record, aggregate_timeline) -- equal to what simulate() recorded
    (tests/golden/make_golden_r5.py captured them)."""
    net, ds, layer, m = case["key"].split("-")
    records = ir.read_yaml(os.path.join(golden_dir, "ops", f"{net}-{ds}-{layer}-{m}.yaml"))
    blocks = lowering.lower(records, 2708, case["op_array"], case["tile_size_list"])
    insts = costmodel.per_instruction(blocks, case["tile_size_list"], 2708, tiles_for)
    cycles, rw, spans = costmodel.simulate_stream(blocks, case["tile_size_list"], 2708, tiles_for, record=True)
    assert (cycles, rw) == (case["cycles"], case["rw"])
    assert sum(r["rw_bytes"] for r in insts) == case["rw"]
    gold = {(d["TYPE"], d["ID"]): d for d in case["insts"]}
    live = [r for r in insts if r["starts"] > 0]
    assert len(live) == len(gold)
    for r in live:
        g = gold[(r["TYPE"], r["ID"])]
        got = (r["block"], r["record_bytes"], r["records"], r["nnz"], r["starts"], r["busy"],
               spans[(r["block"], r["index"])][0], spans[(r["block"], r["index"])][2])
        want = (g["block"], g["bytes"], g["records"], g["nnz"], g["starts"], g["busy"], g["first"], g["last_end"])
        assert got == want, (r["TYPE"], r["ID"])
    val, cnt = costmodel.rw_info(insts)
    assert (val, cnt) == (case["rw_info"][0], case["rw_info"][1])
    tc, tt = costmodel.timeline_info(insts, spans)
    assert (tc, tt) == (case["timeline_info"][0], case["timeline_info"][1])


def test_sparse_tile_counts_equal_calculate_sparsity(golden_dir):
    """tiles.sparse_counts (O(E): the nonzero tiles of a key sort) holds exactly the dense
    calculate_sparsity list, on the pinned Cora graph and on one with duplicates and self loops."""
    z = np.load(os.path.join(golden_dir, "cora_graph.npz"))
    rng = np.random.default_rng(0)
    ip2 = np.concatenate([[0], np.cumsum(rng.integers(0, 9, 500))]).astype(np.int64)
    ix2 = np.sort(rng.integers(0, 500, int(ip2[-1])).reshape(-1), kind="stable").astype(np.int32)
    ix2 = np.concatenate([np.sort(ix2[ip2[r]:ip2[r + 1]]) for r in range(500)]).astype(np.int32)
    ix2[ip2[7]:ip2[8]] = 7  # a row of self loops
    for ip, ix in ((z["indptr"], z["indices"]), (ip2, ix2)):
        n = len(ip) - 1
        g = G.from_numpy(ip, ix)
        for T in (64, 128, 2752):
            dense = isa_ref.tile_nnz(ip, ix, n, T).ravel()
            tc = tiles.sparse_counts(g, T)
            assert tc.length == dense.size and tc.first == dense[0]
            assert np.array_equal(np.sort(tc.values), np.sort(dense[dense > 0]))
            assert np.array_equal(tc.dense(), dense)


def test_per_instruction_model_at_reddit_scale(golden_dir):
    """The metric stream's per-instruction model (Tile_Times 106,232,040 per edge instruction) in
    seconds, from a Reddit-sized tile-count list (synthetic counts: the model only reads the list),
    dense or sparse alike; its bytes sum to the closed-form rw."""
    stream = ir.read_yaml(os.path.join(golden_dir, "streams", "GAT-reddit-layer1-original-h512.yaml"))
    tiles_ = [[512, 1]] * len(stream)
    n = 232965
    length = -(-n // 512) * n
    rng = np.random.default_rng(0)
    dense = rng.poisson(114615892 / length, length).astype(np.int64)
    sparse = costmodel.TileCounts(length, dense[dense > 0], dense[0])
    out = {}
    for name, data in (("dense", dense), ("sparse", sparse)):
        t0 = time.perf_counter()
        insts = costmodel.per_instruction(stream, tiles_, n, lambda T: data)
        dt = time.perf_counter() - t0
        assert dt < 10.0, (name, dt)
        out[name] = insts
        assert sum(r["rw_bytes"] for r in insts) == costmodel.model_rw(stream, n, int(dense.sum()))
    assert out["dense"] == out["sparse"]
    comp = [r for r in out["dense"] if r["TYPE"] == "COMP_MUL_COMP_ADD"]
    assert comp and comp[0]["starts"] == 106232040
    assert comp[0]["busy"] == int(((dense + 7) // 8).sum()) * 32  # ceil(nnz/8) * ceil(512/16) per tile


def test_starved_gather_c_stream_raises_instead_of_spinning(golden_dir, tiles_for):
    """simulate() never finishes 19 of the 22 gather-C golden streams: a fused or small-tile ORDER-C
    gather starves a dependency credit and the cycle loop runs forever (make_golden_r5.py records
    the one GCNT candidate that completes).  The restatement sees the state where nothing runs and
    nothing can start, and raises."""
    records = ir.read_yaml(os.path.join(golden_dir, "ops", "GCNT-cora-layer1-original.yaml"))
    blocks = lowering.lower(records, 2708, [[0, 1, 2, 3]], [[128, 1]])
    with pytest.raises(RuntimeError, match="deadlock"):
        costmodel.simulate_stream(blocks, [[128, 1]], 2708, tiles_for)
    # the per-instruction closed form needs no cycle loop and still answers
    insts = costmodel.per_instruction(blocks, [[128, 1]], 2708, tiles_for)
    assert sum(r["rw_bytes"] for r in insts) == costmodel.model_rw(blocks, 2708, int(sum(tiles_for(128))))


def test_edge_sums_cache_cannot_alias_a_freed_array():
    """_edge_sums keys on id(data); an entry left by an array whose id a new array now
    carries must not be returned for the new one (the entry holds its array and is checked)."""
    import numpy as np
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import costmodel
    cache = {}
    a = np.array([1, 2, 3, 9], np.int64)
    b = np.array([5, 5, 5, 5], np.int64)
    ra = costmodel._edge_sums(cache, a, 4, 16)
    cache[(id(b), 4)] = cache.pop((id(a), 4))  # what a recycled id would look like
    rb = costmodel._edge_sums(cache, b, 4, 16)
    assert ra[0] == 15 and rb[0] == 20
