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


def test_split_sums_a_steps_launch_pairs():
    """A tile cut into row chunks launches one (k_agg_h32, k_seg_reduce) pair per non-empty chunk
    per step: _split sums them per step, after the calibration dispatches."""
    rows = [(0, "k_apply_node4", 5.0), (1, "k_apply_node4", 6.0), (2, "k_aggregate<32>", 7.0),
            (3, "k_aggregate<32>", 8.0)]
    did = 4
    for step in range(3):
        for c, (a, b) in enumerate(((100.0, 10.0), (30.0, 3.0))):
            rows += [(did, "k_agg_h32", a + step), (did + 1, "k_seg_reduce", b)]
            did += 2
    copy, gather, steps = bench._split(rows, per_step=2)
    assert copy == [5.0, 6.0] and gather == [7.0, 8.0]
    assert steps == [(130.0, 13.0), (132.0, 13.0), (134.0, 13.0)]
    assert len(bench._split(rows, per_step=1)[2]) == 6


def test_rank_roofline_fields():
    """The N > 1 line's roofline: the critical (longest-compute) rank's traffic / achieved / frac in
    front, every rank's compute / own step / exposed exchange split, job-wide bytes over the
    critical time; a rank without PMC bytes leaves its own fields and the job total None."""
    per = [{"rank": 0, "tile_edges": 100, "tile_rows": 10, "compute_ms": 0.50, "step_ms": 0.60, "traffic": 3.0e9},
           {"rank": 1, "tile_edges": 120, "tile_rows": 10, "compute_ms": 0.55, "step_ms": 0.58, "traffic": 3.3e9}]
    r = bench.rank_roofline(per)
    assert r["rank_basis"] == 1 and abs(r["kernel_ms"] - 0.55) < 1e-12
    assert abs(r["achieved"] - 3.3e9 / 0.55e-3 / 1e9) < 1e-6 and abs(r["frac"] - r["achieved"] / 8000.0) < 1e-12
    assert abs(r["job_achieved_GBps"] - 6.3e9 / 0.55e-3 / 1e9) < 1e-6 and r["job_peak_GBps"] == 16000.0
    assert [round(x["exposed_exchange_ms"], 6) for x in r["per_rank"]] == [0.1, 0.03]
    assert set(r["per_rank"][0]) == {"rank", "tile_edges", "tile_rows", "compute_ms", "step_ms",
                                     "exposed_exchange_ms", "traffic", "achieved", "frac"}
    assert r["frac_min"] <= r["frac"] <= r["frac_max"]
    per[0]["traffic"] = float("nan")
    r = bench.rank_roofline(per)
    assert r["per_rank"][0]["frac"] is None and r["job_achieved_GBps"] is None and r["frac"] is not None


def test_layers_leg_fails_together_at_n_gt_1():
    """on one GPU a failing layer becomes an error record and the next layer runs; with N > 1
    ranks the failure propagates (torchrun then tears every rank down) instead of the rank running on
    into collectives its peers are not in."""
    import pytest

    def record(name):
        if name == "bad":
            raise MemoryError("out of memory in run_stream")
        return {"config": name, "ms_per_forward": 1.0}
    recs = bench.layers_leg(["ok1", "bad", "ok2"], 1, record, say=lambda m: None)
    assert [r["config"] for r in recs] == ["ok1", "bad", "ok2"] and "MemoryError" in recs[1]["error"]
    with pytest.raises(MemoryError):
        bench.layers_leg(["ok1", "bad", "ok2"], 2, record, say=lambda m: None)
