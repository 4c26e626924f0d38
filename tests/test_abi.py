"""The C-ABI library loads and exports every symbol include/gta.h declares (no GPU calls)."""
import ctypes
import os
import re

import pytest

from gta_graph_tensor_acclelrator_for_general_gnn_amd import _build, _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    src = open(os.path.join(ROOT, "include", "gta.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gta_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    if _build.needs_build():
        _build.build(verbose=False)
    return _lib.load()


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ("gta_abi_version", "gta_last_error", "gta_scatter", "gta_gather_add", "gta_aggregate",
              "gta_apply_edge", "gta_apply_node", "gta_update_mm", "gta_tile_nnz", "gta_aggregate_plan_build",
              "gta_csc_build", "gta_csc_workspace_bytes"):
        assert s in syms


def test_every_declared_symbol_is_exported(lib):
    raw = ctypes.CDLL(_lib.LIB_PATH)
    for s in declared_symbols():
        assert hasattr(raw, s), f"libgta.so does not export {s}"
        assert s in _lib.SIGNATURES, f"_lib.SIGNATURES lacks {s}"


def test_abi_version_and_error_path(lib):
    assert lib.gta_abi_version() == _lib.ABI_VERSION
    # argument validation fails before any device work, so this is safe without a GPU
    rc = lib.gta_aggregate(None, None, 10, 10, 1, None, 0, 0, 0, None, 0, 0, None, None, 0, 0, None, 0, None, None)
    assert rc < 0
    assert b"aggregate" in lib.gta_last_error()
    assert lib.gta_aggregate_plan_bytes(100, 1000, 64) > 0
    assert lib.gta_aggregate_plan_bytes(100, 1000, 0) < 0
    # ABI 11: gather C without the CSC view, a CSC build without workspace, a bad direction
    assert lib.gta_gather_add(1, None, 10, 10, None, None, 10, None, 0, 4, None, 0, 0, None) < 0
    assert b"CSC" in lib.gta_last_error()
    assert lib.gta_gather_add(7, None, 10, 10, None, None, 10, None, 0, 4, None, 0, 0, None) < 0
    assert lib.gta_csc_workspace_bytes(100, 1000) > 0 and lib.gta_csc_workspace_bytes(-1, 0) < 0
    assert lib.gta_csc_build(None, None, 10, 10, 100, None, None, None, None, 0, None) < 0


def test_product_path_refuses_cpu_tensors():
    import torch
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, ops
    g = G.synthetic(20, 60, seed=0)
    with pytest.raises(_lib.GTAError):
        ops.aggregate(g, torch.zeros(20, 4), "src")


def test_tuning_knobs_are_per_thread(lib):
    """ADVICE/VERDICT r1: the tuning knobs are the calling thread's (no process-wide mutable state):
    a knob set on one thread is not seen by another thread's calls."""
    import threading

    from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops
    base = ops.get_debug("seg_lean")
    seen = {}

    def other():
        ops.set_debug("seg_lean", 1 - base)
        seen["other"] = ops.get_debug("seg_lean")
        seen["state"] = ops.knob_state()

    t = threading.Thread(target=other)
    t.start()
    t.join()
    assert seen["other"] == 1 - base
    assert ops.get_debug("seg_lean") == base
    # the HIP-graph cache key follows the calling thread's knobs: the other thread's
    # change is not this thread's state, and a knob set back to its old value drops out
    assert seen["state"] == (("seg_lean", 1 - base),)
    state0 = ops.knob_state()
    ops.set_debug("seg_lean", 1 - base)
    assert ops.knob_state() == tuple(sorted(state0 + (("seg_lean", 1 - base),)))
    ops.set_debug("seg_lean", base)
    assert ops.knob_state() == state0
    with pytest.raises(_lib.GTAError):
        ops.set_debug("no_such_knob", 1)
    with pytest.raises(_lib.GTAError):
        ops.get_debug("no_such_knob")


def test_tuning_handles(lib):
    """ABI 4 knob sets (gta_tuning_*): a handle starts at the defaults, holds its own values apart
    from the thread's knobs, rejects unknown keys, and attaches to / detaches from a stream key
    (the pointer is only a key here: no device work)."""
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops
    thread_val = ops.get_debug("seg_lean")
    t = ops.Tuning(seg_lean=1 - thread_val, mm_split=1 << 40)
    assert t.get("seg_lean") == 1 - thread_val and t.get("mm_split") == 1 << 40  # 64-bit knob values
    assert ops.Tuning().get("mm_split") == -1  # a fresh handle holds the defaults
    assert ops.get_debug("seg_lean") == thread_val        # the thread's knobs are untouched
    with pytest.raises(_lib.GTAError):
        t.set("no_such_knob", 1)
    with pytest.raises(_lib.GTAError):
        t.get("no_such_knob")
    fake_stream = 0x1234560
    t.attach(fake_stream)
    del t                                                # the stream holds a copy: safe to destroy
    ops.Tuning.detach(fake_stream)
    ops.Tuning.detach(fake_stream)                       # detaching twice is harmless


def test_tuning_detaches_its_streams_when_collected(lib):
    """a garbage-collected Tuning detaches the streams still carrying its values,
    but not a stream that another Tuning attached to since (stream pointers are only keys here)."""
    import gc
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops
    s1, s2 = 0x7700010, 0x7700020
    a = ops.Tuning(seg_lean=0)
    a.attach(s1)
    a.attach(s2)
    b = ops.Tuning(seg_lean=1)
    b.attach(s2)                                         # s2 now carries b's values
    del a
    gc.collect()
    assert not ops.Tuning.attached(s1) and ops.Tuning.attached(s2)
    ops.Tuning.detach(s2)
    del b


def test_split_count_reads_the_streams_knob_set(lib):
    """gta_update_mm_t_splits takes the stream, so a knob set attached to it
    (mm_split) decides the split count the same way it decides the GEMM's own launch."""
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops
    M, K, N = 2708, 1433, 128
    default = lib.gta_update_mm_t_splits(M, K, N, 0, None)
    assert default > 1
    fake_stream = 0x5500100
    t = ops.Tuning(mm_split=3)
    t.attach(fake_stream)
    try:
        assert lib.gta_update_mm_t_splits(M, K, N, 0, fake_stream) == 3
        assert lib.gta_update_mm_t_splits(M, K, N, 0, None) == default  # other streams keep the default
    finally:
        ops.Tuning.detach(fake_stream)
    assert lib.gta_update_mm_t_splits(M, K, N, 0, fake_stream) == default
