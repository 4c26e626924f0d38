"""Pin the oracle to the reference's own outputs (tests/golden, made by make_golden.py)."""
import os

import numpy as np
import pytest

from oracle import isa_ref


@pytest.fixture(scope="module")
def cora(golden_dir):
    z = np.load(os.path.join(golden_dir, "cora_graph.npz"))
    return z["indptr"], z["indices"]


def test_cora_graph_shape(cora):
    ip, ix = cora
    assert len(ip) == 2709 and len(ix) == 10556 and ip[-1] == 10556
    assert np.all(np.diff(ip) >= 0)


@pytest.mark.parametrize("T", [64, 128, 256, 512, 1024, 2048, 2752])
def test_tile_nnz_matches_calculate_sparsity(cora, golden_dir, T):
    """isa_ref.tile_nnz == reference code/preprocessing.py calculate_sparsity(T, 1) bit-exactly."""
    ip, ix = cora
    gold = np.load(os.path.join(golden_dir, "cora_tiles.npz"))[f"T{T}"]
    got = isa_ref.tile_nnz(ip, ix, 2708, T)
    assert got.shape == gold.shape
    assert np.array_equal(got, gold)


def test_gen_size_and_maxlist(cora, manifest):
    ip, ix = cora
    sizes = isa_ref.gen_size(64, 2708)
    assert sizes == manifest["tiles"]["gen_size_64_2708"]
    maxlist = [isa_ref.max_tile(isa_ref.tile_nnz(ip, ix, 2708, T)) for T in sizes]
    assert maxlist == manifest["tiles"]["maxlist"]


def test_tile_nnz_self_loops_and_duplicates():
    # row 0: self loop + duplicate (0,1) pair; dense count_nonzero counts (0,1) once and drops (0,0)
    ip = np.array([0, 3, 4])
    ix = np.array([0, 1, 1, 0])
    got = isa_ref.tile_nnz(ip, ix, 2, 1)
    assert got.tolist() == [[0, 1], [1, 0]]


def test_aggregate_matches_edgewise_composition():
    rng = np.random.default_rng(0)
    n, e, F, H = 50, 400, 12, 4
    ip = np.concatenate([[0], np.sort(rng.integers(0, e, n - 1)), [e]])
    ix = rng.integers(0, n, e)
    x = rng.standard_normal((n, F))
    w = rng.random((e, H))
    xe = isa_ref.scatter(ip, ix, x, "C")
    prod = isa_ref.apply_edge(ip, ix, "MUL", None, xe, "edge", w, "edge")
    ref = isa_ref.gather_add(ip, prod)
    assert np.allclose(isa_ref.aggregate(ip, ix, x, "src", w), ref, rtol=1e-12, atol=1e-12)


def test_c_oracle_matches_numpy_oracle():
    from oracle import cbase
    rng = np.random.default_rng(3)
    n, e, F, H = 300, 5000, 128, 8
    ip = np.concatenate([[0], np.sort(rng.integers(0, e, n - 1)), [e]]).astype(np.int64)
    ix = rng.integers(0, n, e).astype(np.int32)
    x = rng.standard_normal((n, F)).astype(np.float32)
    w = rng.random((e, H)).astype(np.float32)
    got = cbase.aggregate(ip, ix, x, w, threads=2)
    ref = isa_ref.aggregate(ip, ix, x, "src", w)
    bound = 1e-5 * isa_ref.aggregate_abs(ip, ix, x, "src", w) + 1e-6
    assert np.all(np.abs(got - ref) <= bound)
    got1 = cbase.aggregate(ip, ix, x, None, threads=1)
    assert np.allclose(got1, isa_ref.aggregate(ip, ix, x, "src", None), rtol=1e-5, atol=1e-5)
