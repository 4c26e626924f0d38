"""The Reddit/Flickr tile-metadata preprocessing ("FinalVersion For Paper/preprocessing_forReditFlickr.py":
first 25 % of the 16x1 tile rows, re-blocked by summation for each of its 17 block sizes), pinned
to the reference's own outputs (tests/golden/make_golden_preproc.py ran its pipeline on a seeded
16x1 count matrix and kept the arrays it saved).  CPU: the numpy restatement; GPU: the same
matrices straight from the CSR with gta_tile_nnz.  Bit-exact."""
import os

import numpy as np
import pytest

from gta_graph_tensor_acclelrator_for_general_gnn_amd import tiles

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "preproc_reddit_flickr.npz")


@pytest.fixture(scope="module")
def gold():
    return np.load(GOLD)


def test_block_list_matches_the_reference_run(gold):
    assert sorted(int(k.split("_")[1]) for k in gold.files if k.startswith("reblock_")) == \
        sorted(tiles.REDDIT_FLICKR_BLOCKS)


@pytest.mark.parametrize("block", tiles.REDDIT_FLICKR_BLOCKS)
def test_reblock_restatement_bit_exact(gold, block):
    ref = gold[f"reblock_{block}"]
    got = tiles.reblock(gold["tiles16"], block)
    assert got.dtype == ref.dtype and got.shape == ref.shape
    np.testing.assert_array_equal(got, ref)


def test_reblock_edge_cases():
    m = np.arange(12, dtype=np.float64).reshape(6, 2)
    assert tiles.reblock(m, 4).tolist() == [[0.0, 1.0]]            # int(6 * 0.25) = 1 row kept
    assert tiles.reblock(m[:3], 4).shape == (0, 2)                  # int(3 * 0.25) = 0 rows kept
    np.testing.assert_array_equal(tiles.reblock(m, 2, fraction=1.0), [[2, 4], [10, 12], [18, 20]])


@pytest.mark.gpu
@pytest.mark.parametrize("block", [64, 128, 256, 1600, 8192])
def test_reddit_flickr_tiles_from_csr_on_gpu(gold, dev, block):
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G
    g = G.from_numpy(gold["indptr"], gold["indices"], device=dev)
    got = tiles.reddit_flickr_tiles(g, block).cpu().numpy()
    np.testing.assert_array_equal(got, gold[f"reblock_{block}"])
