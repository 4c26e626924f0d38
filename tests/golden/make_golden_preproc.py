"""Golden fixture for the Reddit/Flickr tile-metadata preprocessing by RUNNING the reference.

Test infrastructure only (never shipped, never run on the GPU box).  The reference script
"FinalVersion For Paper/preprocessing_forReditFlickr.py" runs its own pipeline at import time
(`process_and_save(file_path, block_sizes)`, :38-41): np.load of a 16x1 tile-count matrix, the
first 25 % of its rows (slice_matrix :10-13), re-blocked by summation for every block size of its
list (reblock_matrix :15-24), each result np.save'd.  Here numpy.load / numpy.save are patched
for the duration of that import: load hands it a seeded 16x1 count matrix of a synthetic
Flickr-like graph (as the scipy CSR matrix it expects under 'matrix'), save records every output.
Only those arrays are committed (tests/golden/preproc_reddit_flickr.npz), never reference text.

Usage (in the dev container only):  python tests/golden/make_golden_preproc.py
"""
import importlib.util
import os
import sys

import numpy as np

REF = "/root/reference/FinalVersion For Paper/preprocessing_forReditFlickr.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "preproc_reddit_flickr.npz")


def tile16_counts(n=9000, e=90000, seed=0):
    """Seeded CSR (rows sorted, duplicates kept) -> its 16x1 tile counts, as calculate_sparsity
    counts them (self loops removed, a repeated (dst, src) once)."""
    rng = np.random.default_rng(seed)
    deg = rng.poisson(e / n, n)
    indptr = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    indices = np.concatenate([np.sort(rng.integers(0, n, d)) for d in deg]).astype(np.int32)
    dense = np.zeros((n, n), dtype=np.int8)
    rows = np.repeat(np.arange(n), deg)
    dense[rows, indices] = 1
    np.fill_diagonal(dense, 0)
    nt = -(-n // 16)
    pad = np.zeros((nt * 16, n), dtype=np.int32)
    pad[:n] = dense
    return indptr, indices, pad.reshape(nt, 16, n).sum(axis=1).astype(np.float64)


def main():
    import scipy.sparse
    indptr, indices, m16 = tile16_counts()
    saved = {}
    real_load, real_save = np.load, np.save
    np.load = lambda path, *a, **k: {"matrix": scipy.sparse.csr_matrix(m16)}
    np.save = lambda path, arr, *a, **k: saved.__setitem__(os.path.basename(path), np.array(arr))
    try:
        spec = importlib.util.spec_from_file_location("ref_preproc_rf", REF)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)  # runs process_and_save on the patched load/save
    finally:
        np.load, np.save = real_load, real_save
    sys.modules.pop("ref_preproc_rf", None)
    out = {"indptr": indptr, "indices": indices, "tiles16": m16}
    for name, arr in saved.items():  # 'path/to/your/<B>x1_file.npy'
        block = int(name.split("x1")[0])
        out[f"reblock_{block}"] = arr
    np.savez_compressed(OUT, **out)
    print("wrote", OUT, sorted(k for k in out if k.startswith("reblock_")))


if __name__ == "__main__":
    main()
