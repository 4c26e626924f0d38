"""bench.py's PMC byte accounting (pmc_traffic), on counter values alone (no GPU, no rocprofv3).

The read side of FETCH_SIZE is calibrated twice in the same pass: streaming reads on a float4 copy
(MI355X_MICROARCH.md §HBM: FETCH_SIZE reports half of a wide streaming read) and 512-B gathered
rows on a permutation gather.  k_agg_h32's FETCH is split into its known streams and its gathers,
each scaled by its own factor; k_seg_reduce's reads take the streaming factor.  The round-2 check
this pins: the reduce's counted bytes can no longer fall below its compulsory partial-row reads.
"""
import bench


def _passes(copy_f, gather_f, agg_f, red_f, copy_w, agg_w, red_w):
    return {"FETCH_SIZE": {"copy_kb": copy_f, "gather_kb": gather_f, "agg_kb": agg_f, "reduce_kb": red_f},
            "WRITE_SIZE": {"copy_kb": copy_w, "gather_kb": copy_w, "agg_kb": agg_w, "reduce_kb": red_w}}


def test_factors_from_the_calibration_launches():
    n = bench.CALIB_ROWS
    copy_bytes = n * 4 * bench.F
    stream_idx = n * 4 + (n + 1) * 8
    # a streaming read counted at exactly 1/2, a gather at 1/1.75 (its index streams at 1/2)
    copy_kb = copy_bytes / 2 / 1024
    gather_kb = (copy_bytes / 1.75 + stream_idx / 2) / 1024
    meta = {"nnz": 1000, "heads": 8, "n_items": 10, "n_rows": 100}
    r = bench.pmc_traffic(_passes(copy_kb, gather_kb, 1e6, 1e5, copy_bytes / 1024, 2e5, 1e4), meta)
    assert abs(r["read_factor_stream"] - 2.0) < 1e-9
    assert abs(r["read_factor_gather"] - 1.75) < 1e-9
    assert abs(r["write_factor"] - 1.0) < 1e-9


def test_agg_split_and_reduce_bytes():
    n = bench.CALIB_ROWS
    copy_bytes = n * 4 * bench.F
    stream_idx = n * 4 + (n + 1) * 8
    E, H, items = 114615892, 8, 4624949
    streams = 4.0 * E + 4.0 * H * E + 16.0 * items
    gathers, partial = 19.5e9, items * 512.0
    res = _passes(copy_bytes / 2 / 1024, (copy_bytes / 1.75 + stream_idx / 2) / 1024,
                  (streams / 2 + gathers / 1.75) / 1024, (partial / 2) / 1024,
                  copy_bytes / 1024, partial / 1024, 232965 * 512 / 1024)
    r = bench.pmc_traffic(res, {"nnz": E, "heads": H, "n_items": items, "n_rows": 232965})
    assert abs(r["agg_split"]["streams"] - streams) < 1
    assert abs(r["agg_split"]["gathers"] - gathers) / gathers < 1e-9
    # the reduce reads every partial row once and writes y: never below that compulsory traffic
    assert r["reduce_bytes"] >= partial + 232965 * 512 - 1
    assert abs(r["bytes_per_launch"] - (r["agg_bytes"] + r["reduce_bytes"])) < 1
