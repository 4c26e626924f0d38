"""gta_aggregate_expr (ABI 14): a gather of an applyedge expression tree in one launch.

The bar is bitwise equality with the unfused form -- the same apply_edge ops writing their [E, F]
edge tensors, then gta_aggregate(x_mode EDGE) of the last one with the same plan -- since the
fused kernel evaluates each step with the same arithmetic, rounds each intermediate to fp32 as the
stored tensor would, and sums in that aggregate's order.  The unfused ops themselves are checked
against the fp64 oracle by test_gpu_ops.py / test_gpu_executor.py.
"""
import os

import numpy as np
import pytest
import torch

from gta_graph_tensor_acclelrator_for_general_gnn_amd import executor, ir, ops, workloads
from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G
from gta_graph_tensor_acclelrator_for_general_gnn_amd.semantics import Semantics
from oracle import isa_ref

from .test_gpu_ops import _graph

pytestmark = pytest.mark.gpu


def _operand(rng, g, mode, F, dev, positive=False):
    n = {"src": g.n_cols, "dst": g.n_rows, "edge": g.nnz, "row": 1}[mode]
    a = rng.standard_normal((n, F)).astype(np.float32)
    if positive:  # a divisor: away from zero
        a = np.abs(a) + 0.5
    return torch.from_numpy(a).to(dev)


def _edge(g, t, mode):
    """The operand as the unfused form sees it: (tensor, apply_edge mode, broadcast-row flag)."""
    if mode == "row":
        return t, "edge", True
    return t, mode, False


def _step(g, bin_, sf, a, b):
    """One unfused apply_edge step over (tensor, mode, broadcast) operands; a left broadcast row is
    expanded, as the executor does for a non-commuting op."""
    ta, ma, ra = a
    if ra:
        ta, ma = ta.expand(g.nnz, ta.shape[1]).contiguous(), "edge"
    if b is None:
        return ops.apply_edge(g, None, sf, ta, ma), "edge", False
    tb, mb, rb = b
    return ops.apply_edge(g, bin_, sf, ta, ma, tb, mb, b_broadcast_row=rb), "edge", False


def _unfused(g, shape, operands, bins, sfs, swap, plan):
    L = [_edge(g, t, m) for t, m in operands]
    u = _step(g, bins[0], sfs[0], L[0], L[1] if len(L) > 1 else None)
    if shape == 1:
        t = u
    elif shape == 2:
        t = _step(g, bins[1], sfs[1], L[2], u) if swap else _step(g, bins[1], sfs[1], u, L[2])
    else:
        v = _step(g, bins[1], sfs[1], L[2], L[3])
        t = _step(g, bins[2], sfs[2], u, v)
    return ops.aggregate(g, t[0], "edge", plan=plan)


def _bits(t):
    return t.contiguous().view(torch.int32)


CASES = [  # (shape, modes, bins, sfs, swap)
    (1, ("src", "dst"), ("SUB",), ("TANH",), False),
    (1, ("edge",), (None,), ("SIGMOID",), False),
    (1, ("row", "src"), ("DIV",), ("NONE",), False),
    (2, ("src", "dst", "edge"), ("ADD", "ADD"), ("NONE", "RELU"), False),      # PNA ops 5-7
    (2, ("dst", "src", "edge"), ("MUL", "SUB"), ("EXP", "NONE"), True),
    (2, ("src", "row", "dst"), ("DIV", "DIV"), ("ELU", "LEAKY_RELU"), False),
    (3, ("src", "dst", "src", "dst"), ("ADD", "ADD", "ADD"), ("NONE", "NONE", "NONE"), False),  # DGN 2-7
    (3, ("edge", "src", "row", "dst"), ("MUL", "SUB", "MUL"), ("RELU", "TANH", "SIGMOID"), False),
]


@pytest.mark.parametrize("F", [128, 64, 256, 100, 602, 36])
@pytest.mark.parametrize("case", range(len(CASES)))
@pytest.mark.parametrize("plan", [None, 64])
def test_aggregate_expr_bitwise_equals_unfused(dev, F, case, plan):
    """Both forms (k_agg_expr at F = 128 / 256, k_aggregate's XM_EX* form) against the unfused ops."""
    for lean in (1, 0):
        ops.set_debug("expr_lean", lean)
        try:
            _expr_case(dev, F, case, plan)
        finally:
            ops.set_debug("expr_lean", 1)


def _expr_case(dev, F, case, plan):
    shape, modes, bins, sfs, swap = CASES[case]
    g, ip, ix = _graph(300, 5000, seed=F + case, heavy_row=700, empty_rows=3, dev=dev)
    rng = np.random.default_rng(F * 7 + case)
    # a divisor operand (right of a DIV) is kept away from zero: no inf / NaN whose payloads could
    # differ (an intermediate divisor: test_aggregate_expr_intermediate_divisor)
    div_right = set()
    if bins[0] == "DIV":
        div_right.add(1)
    if shape == 2 and bins[1] == "DIV" and not swap:
        div_right.add(2)
    if shape == 3 and bins[1] == "DIV":
        div_right.add(3)
    ops_ = [(_operand(rng, g, m, F, dev, positive=l in div_right), m) for l, m in enumerate(modes)]
    y = ops.aggregate_expr(g, shape, ops_, bins, sfs, swap, plan=plan)
    assert y is not None
    ref = _unfused(g, shape, ops_, bins, sfs, swap, plan)
    assert torch.equal(_bits(y), _bits(ref)), (CASES[case], F, plan)


@pytest.mark.parametrize("F", [128, 256])
def test_aggregate_expr_intermediate_divisor(dev, F):
    """DIV by an intermediate (shape 2 swapped: L2 / sf(L0 + L1); shape 3: u / v), kept positive by EXP."""
    g, _, _ = _graph(500, 9000, seed=F, heavy_row=1500, dev=dev)
    rng = np.random.default_rng(F)
    for shape, modes, bins, sfs, swap in ((2, ("src", "dst", "edge"), ("ADD", "DIV"), ("EXP", "NONE"), True),
                                          (3, ("src", "dst", "edge", "src"), ("SUB", "ADD", "DIV"),
                                           ("NONE", "EXP", "TANH"), False)):
        ops_ = [(_operand(rng, g, m, F, dev), m) for m in modes]
        for plan in (None, 512):
            y = ops.aggregate_expr(g, shape, ops_, bins, sfs, swap, plan=plan)
            ref = _unfused(g, shape, ops_, bins, sfs, swap, plan)
            assert torch.equal(_bits(y), _bits(ref)), (shape, plan)


def test_aggregate_expr_matches_fp64_oracle(dev):
    """The DGN form against the fp64 oracle directly (|d| <= 1e-5 sum|terms| + 1e-6)."""
    g, ip, ix = _graph(400, 6000, seed=3, heavy_row=900, empty_rows=2, dev=dev)
    rng = np.random.default_rng(3)
    F = 128
    ops_ = [(_operand(rng, g, m, F, dev), m) for m in ("src", "dst", "src", "dst")]
    y = ops.aggregate_expr(g, 3, ops_, ("ADD", "ADD", "ADD"), None, plan=512)
    a, b, c, d = (t.cpu().numpy().astype(np.float64) for t, _ in ops_)
    rows = np.repeat(np.arange(g.n_rows), np.diff(ip))
    t = (a[ix] + b[rows]) + (c[ix] + d[rows])
    terms = np.abs(a[ix]) + np.abs(b[rows]) + np.abs(c[ix]) + np.abs(d[rows])
    ref = np.zeros((g.n_rows, F))
    sc = np.zeros((g.n_rows, F))
    np.add.at(ref, rows, t)
    np.add.at(sc, rows, terms)
    err = np.abs(y.cpu().numpy() - ref)
    assert (err <= 1e-5 * sc + 1e-6).all(), err.max()
    # and the ISA oracle's gather of the oracle's apply_edge ops
    u = isa_ref.apply_edge(ip, ix, "ADD", None, a.astype(np.float32), "src", b.astype(np.float32), "dst")
    assert np.allclose(u, a[ix] + b[rows], rtol=1e-6, atol=1e-6)


def test_aggregate_expr_unsupported_alignment_returns_none(dev):
    """An operand whose row stride does not admit the aggregate's vector width: None (run unfused)."""
    g, _, _ = _graph(100, 1000, seed=1, dev=dev)
    base = torch.randn(g.n_rows, 129, device=dev)
    a = base[:, :128]  # ld 129: odd
    b = torch.randn(g.n_rows, 128, device=dev)
    assert ops.aggregate_expr(g, 1, [(a, "src"), (b, "dst")], ("ADD",), None) is None
    with pytest.raises(ValueError):
        ops.aggregate_expr(g, 2, [(b, "src"), (b, "dst")], ("ADD", "ADD"), None)  # shape 2 takes 3


def test_aggregate_expr_empty_graph(dev):
    ip = np.zeros(6, dtype=np.int64)
    g = G.from_numpy(ip, np.zeros(0, dtype=np.int32), device=dev)
    a = torch.randn(5, 128, device=dev)
    y = ops.aggregate_expr(g, 3, [(a, "src"), (a, "dst"), (a, "src"), (a, "dst")], ("ADD", "SUB", "MUL"), None)
    assert torch.equal(y, torch.zeros_like(y))


def _streams(golden_dir, manifest, network):
    return [s for s in manifest["streams"] if "file" in s and s["network"] == network]


@pytest.mark.parametrize("network", ["DGN", "PNA"])
@pytest.mark.parametrize("plan_chunk", [0, 64])
def test_edge_expr_fusion_bitwise_on_gpu(golden_dir, manifest, dev, network, plan_chunk):
    """Every DGN / PNA golden stream (both op orders, every layer) with the fused expression gather
    gives every op's value bitwise equal to the unfused run, and the fusion is taken."""
    z = np.load(os.path.join(golden_dir, "cora_graph.npz"))
    gd = G.from_numpy(z["indptr"], z["indices"], device=dev)
    recs = _streams(golden_dir, manifest, network)
    assert recs
    for rec in recs:
        sem = Semantics.for_network(network, rec["reorder"])
        og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
        st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
        tensors = workloads.make_tensors(og, gd, network, seed=5)
        vals, launches = {}, {}
        for on in (True, False):
            ex = executor.Executor(og, st, gd, tensors, sem, plan_chunk=plan_chunk)
            ex.edge_expr = on
            assert ex.expr, rec["file"]
            outs = ex.run()
            launches[on] = ex.launches
            sinks = {k: v.clone() for k, v in outs.items()}
            vals[on] = (sinks, [ex.tensor_of(i) for i in range(len(og))])
        for k in vals[True][0]:
            assert torch.equal(_bits(vals[True][0][k]), _bits(vals[False][0][k])), f"{rec['file']} sink {k}"
        for i, (a, b) in enumerate(zip(vals[True][1], vals[False][1])):
            assert torch.equal(_bits(a), _bits(b)), f"{rec['file']} op {i}"
        assert launches[True] < launches[False], rec["file"]
