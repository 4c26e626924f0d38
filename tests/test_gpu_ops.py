"""GPU parity of every libgta kernel against the fp64 oracle (oracle/isa_ref.py).

Tolerances (written here):
  scatter / tile_nnz              bit-exact
  aggregate / gather / edge ops   |d| <= 1e-5 * sum|terms| + 1e-6   (fp32 accumulation)
  fp32 MFMA UPDATE                |d| <= 1e-5 * sum|x||w| + 1e-6
  bf16 MFMA UPDATE                vs fp64 of the bf16-rounded inputs, |d| <= 1e-5 * sum|x||w| + 1e-6
"""
import os

import numpy as np
import pytest
import torch

from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, ops
from oracle import isa_ref

pytestmark = pytest.mark.gpu


def _graph(n, e, seed=0, kind="lognormal", heavy_row=None, empty_rows=0, dev=None):
    g = G.synthetic(n, e, seed=seed, kind=kind)
    ip, ix = g.numpy()
    if heavy_row is not None or empty_rows:
        rng = np.random.default_rng(seed)
        deg = np.diff(ip).copy()
        if empty_rows:
            deg[rng.choice(n, empty_rows, replace=False)] = 0
        if heavy_row is not None:
            deg[n // 2] = heavy_row
        ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
        ix = rng.integers(0, n, int(ip[-1])).astype(np.int32)
    gd = G.from_numpy(ip, ix, device=dev)
    return gd, ip, ix


_DT = {"f32": 0, "bf16": 1, "mixed": 2}  # include/gta.h GTA_F32 / GTA_BF16 / GTA_F32_BF16


def _check(got, ref, scale, what):
    got = got.detach().cpu().numpy().astype(np.float64)
    err = np.abs(got - ref)
    bound = 1e-5 * scale + 1e-6
    bad = err > bound
    assert not bad.any(), f"{what}: {bad.sum()} elements out of tolerance, max err {err.max():.3e}"


CASES = [  # (n, e, F, heads)
    (300, 4000, 128, 8),     # metric shape (8 heads x 16)
    (300, 4000, 128, 16),    # genGraphOP GAT layer-1 alpha width 16
    (300, 4000, 128, 1),     # scalar edge weight (GCN)
    (300, 4000, 128, 128),   # full-width edge tensor
    (257, 3000, 602, 1),     # Reddit feature width, SAGE original order
    (200, 2500, 1433, 1),    # Cora feature width (odd)
    (300, 4000, 16, 16),     # GAT edge-softmax width
    (300, 4000, 64, 4),
    (300, 4000, 3, 1),
    (300, 4000, 100, 4),     # products width
]


@pytest.mark.parametrize("n,e,F,heads", CASES)
@pytest.mark.parametrize("plan", [None, 64])
def test_aggregate_src_weighted(dev, n, e, F, heads, plan):
    g, ip, ix = _graph(n, e, seed=F + heads, heavy_row=700, empty_rows=5, dev=dev)
    rng = np.random.default_rng(1)
    x = rng.standard_normal((n, F)).astype(np.float32)
    w = rng.random((g.nnz, heads)).astype(np.float32)
    y = ops.aggregate(g, torch.from_numpy(x).to(dev), "src", torch.from_numpy(w).to(dev), plan=plan)
    ref = isa_ref.aggregate(ip, ix, x, "src", w)
    _check(y, ref, isa_ref.aggregate_abs(ip, ix, x, "src", w), f"aggregate F={F} H={heads} plan={plan}")


@pytest.mark.parametrize("F", [1, 16, 128, 602])
@pytest.mark.parametrize("plan", [None, 128])
def test_aggregate_unweighted_rowscale_accumulate(dev, F, plan):
    n, e = 400, 6000
    g, ip, ix = _graph(n, e, seed=11, heavy_row=1000, empty_rows=3, dev=dev)
    rng = np.random.default_rng(2)
    x = rng.standard_normal((n, F)).astype(np.float32)
    y0 = rng.standard_normal((n, F)).astype(np.float32)
    scale = (1.0 / np.maximum(np.diff(ip), 1)).astype(np.float32)
    yd = torch.from_numpy(y0).to(dev)
    ops.aggregate(g, torch.from_numpy(x).to(dev), "src", None, row_scale=torch.from_numpy(scale).to(dev), out=yd,
                  accumulate=True, plan=plan)
    ref = y0 + isa_ref.aggregate(ip, ix, x, "src", None, scale)
    _check(yd, ref, isa_ref.aggregate_abs(ip, ix, x, "src", None, scale) + np.abs(y0), "aggregate acc")


@pytest.mark.parametrize("F", [16, 128, 5])
def test_gather_add_and_edge_mode(dev, F):
    n, e = 300, 5000
    g, ip, ix = _graph(n, e, seed=3, empty_rows=4, dev=dev)
    rng = np.random.default_rng(4)
    xe = rng.standard_normal((g.nnz, F)).astype(np.float32)
    y = ops.gather_add(g, torch.from_numpy(xe).to(dev))
    ref = isa_ref.gather_add(ip, xe)
    _check(y, ref, isa_ref.gather_add(ip, np.abs(xe)), "gather_add")
    w = rng.random((g.nnz, F)).astype(np.float32)
    y2 = ops.aggregate(g, torch.from_numpy(xe).to(dev), "edge", torch.from_numpy(w).to(dev), plan=64)
    _check(y2, isa_ref.aggregate(ip, ix, xe, "edge", w), isa_ref.aggregate_abs(ip, ix, xe, "edge", w), "edge-mode")


def test_aggregate_dst_mode(dev):
    n, e, F = 200, 3000, 32
    g, ip, ix = _graph(n, e, seed=7, dev=dev)
    rng = np.random.default_rng(5)
    x = rng.standard_normal((n, F)).astype(np.float32)
    w = rng.random((g.nnz, 4)).astype(np.float32)
    y = ops.aggregate(g, torch.from_numpy(x).to(dev), "dst", torch.from_numpy(w).to(dev))
    _check(y, isa_ref.aggregate(ip, ix, x, "dst", w), isa_ref.aggregate_abs(ip, ix, x, "dst", w), "dst-mode")


def test_aggregate_deterministic(dev):
    g, ip, ix = _graph(2000, 60000, seed=9, heavy_row=5000, dev=dev)
    x = torch.randn(2000, 128, device=dev)
    w = torch.rand(g.nnz, 8, device=dev)
    a = ops.aggregate(g, x, "src", w, plan=256)
    b = ops.aggregate(g, x, "src", w, plan=256)
    assert torch.equal(a, b)


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("F", [1, 3, 16, 128, 602])
@pytest.mark.parametrize("direction", ["R", "C"])
def test_scatter_bit_exact(dev, dtype, F, direction):
    n, e = 300, 4000
    g, ip, ix = _graph(n, e, seed=F, empty_rows=3, dev=dev)
    x = torch.randn(n, F, device=dev).to(dtype)
    out = ops.scatter(g, x, direction)
    ref = isa_ref.scatter(ip, ix, x.float().cpu().numpy(), direction)
    assert torch.equal(out.float().cpu(), torch.from_numpy(ref).float())


@pytest.mark.parametrize("bin_kind,sf,a_mode,b_mode,Fa,Fb", [
    ("ADD", "EXP_LEAKY_RELU", "dst", "src", 16, 16),   # GAT ops 4-7 fused: exp(lrelu(eL[dst] + eR[src]))
    ("DIV", None, "edge", "dst", 16, 16),              # GAT op 9 with op 10 (scatter R of the sums)
    ("MUL", None, "src", "edge", 128, 16),             # GAT op 11 (alpha head broadcast)
    ("MUL", None, "src", "edge", 602, 1),              # GCN/SAGE/GIN op 1 with a scalar edge weight
    ("ADD", "RELU", "edge", "edge", 7, 7),
    (None, "ELU", "edge", None, 12, None),
])
def test_apply_edge(dev, bin_kind, sf, a_mode, b_mode, Fa, Fb):
    n, e = 250, 3000
    g, ip, ix = _graph(n, e, seed=Fa, empty_rows=3, dev=dev)
    rng = np.random.default_rng(6)
    rows = {"edge": g.nnz, "src": n, "dst": n}
    a = rng.standard_normal((rows[a_mode], Fa)).astype(np.float32)
    b = None if Fb is None else (rng.random((rows[b_mode], Fb)) + 0.5).astype(np.float32)
    out = ops.apply_edge(g, bin_kind, sf, torch.from_numpy(a).to(dev), a_mode,
                         None if b is None else torch.from_numpy(b).to(dev), b_mode or "edge")
    ref = isa_ref.apply_edge(ip, ix, bin_kind, sf, a, a_mode, b, b_mode or "edge")
    got = out.cpu().numpy().astype(np.float64)
    assert np.allclose(got, ref, rtol=2e-6, atol=1e-6)


@pytest.mark.parametrize("bin_kind,sf,Fa,Fb,bcast", [
    ("ADD", None, 128, 128, False), ("MUL", None, 602, 1, True), ("DIV", "ELU", 128, 16, False),
    (None, "RELU", 64, None, False), ("ADD", "SIGMOID", 10, 10, False), (None, "TANH", 3, None, False),
])
def test_apply_node(dev, bin_kind, sf, Fa, Fb, bcast):
    rng = np.random.default_rng(7)
    n = 777
    a = rng.standard_normal((n, Fa)).astype(np.float32)
    b = None if Fb is None else (rng.random((1 if bcast else n, Fb)) + 0.5).astype(np.float32)
    out = ops.apply_node(bin_kind, sf, torch.from_numpy(a).to(dev), None if b is None else torch.from_numpy(b).to(dev),
                         b_broadcast_row=bcast)
    ref = isa_ref.apply_node(bin_kind, sf, a, b, b_broadcast_row=bcast)
    assert np.allclose(out.cpu().numpy(), ref, rtol=2e-6, atol=1e-6)


@pytest.mark.parametrize("bin_kind,sf,Fa,Fb,bcast", [
    ("MUL", None, 100, 1, True), ("ADD", None, 100, 100, False), ("MUL", "ELU", 128, 1, False),
    (None, "RELU", 128, None, False), ("DIV", "EXP", 4, 4, False), ("SUB", "SIGMOID", 16, 1, True),
    ("ADD", None, 128, 16, False),  # head broadcast: generic kernel
])
def test_apply_node_vector_form_bitwise(dev, bin_kind, sf, Fa, Fb, bcast):
    """k_apply_node4 (float4 rows; b none, same shape or one value per node / for all) == the
    generic per-element kernel bitwise, and == the oracle."""
    rng = np.random.default_rng(Fa + (Fb or 0))
    n = 5003
    a = torch.from_numpy(rng.standard_normal((n, Fa)).astype(np.float32)).to(dev)
    b = None if Fb is None else torch.from_numpy((rng.random((1 if bcast else n, Fb)) + 0.5).astype(np.float32)).to(dev)
    outs = []
    try:
        for vec in (1, 0):
            ops.set_debug("apply_node_vec", vec)
            outs.append(ops.apply_node(bin_kind, sf, a, b, b_broadcast_row=bcast))
    finally:
        ops.set_debug("apply_node_vec", 1)
    assert torch.equal(outs[0], outs[1])
    ref = isa_ref.apply_node(bin_kind, sf, a.cpu().numpy(), None if b is None else b.cpu().numpy(),
                             b_broadcast_row=bcast)
    assert np.allclose(outs[0].cpu().numpy(), ref, rtol=2e-6, atol=1e-6)


@pytest.mark.parametrize("M,K,N", [(2708, 1433, 128), (1000, 602, 128), (777, 128, 16), (64, 64, 64),
                                   (5, 3, 7), (3000, 100, 128), (513, 130, 65)])
@pytest.mark.parametrize("gathered", [False, True])
def test_update_mm_f32(dev, M, K, N, gathered):
    rng = np.random.default_rng(M + K)
    x = rng.standard_normal((M + 10, K)).astype(np.float32)
    w = rng.standard_normal((K, N)).astype(np.float32)
    idx = rng.integers(0, M + 10, M).astype(np.int32) if gathered else None
    out = ops.update_mm(torch.from_numpy(x).to(dev), torch.from_numpy(w).to(dev),
                        None if idx is None else torch.from_numpy(idx).to(dev), m=None if gathered else M)
    ref = isa_ref.mm(x, w, idx) if gathered else isa_ref.mm(x[:M], w)
    scale = (np.abs(x[idx] if gathered else x[:M]).astype(np.float64) @ np.abs(w).astype(np.float64))
    _check(out, ref, scale, "update_mm f32")


@pytest.mark.parametrize("M,K,N", [(2449, 100, 128), (1000, 128, 128), (333, 37, 50), (64, 256, 64)])
def test_update_mm_bf16(dev, M, K, N):
    rng = np.random.default_rng(K)
    x = torch.from_numpy(rng.standard_normal((M, K)).astype(np.float32)).to(torch.bfloat16)
    w = torch.from_numpy(rng.standard_normal((K, N)).astype(np.float32)).to(torch.bfloat16)
    out = ops.update_mm(x.to(dev), w.to(dev), sf="RELU")
    xf, wf = x.float().numpy(), w.float().numpy()
    ref = isa_ref.mm(xf, wf, sf_kind="RELU")
    scale = np.abs(xf).astype(np.float64) @ np.abs(wf).astype(np.float64)
    _check(out, ref, scale, "update_mm bf16")


def test_tile_nnz_gpu_matches_reference_golden(dev, golden_dir):
    z = np.load(os.path.join(golden_dir, "cora_graph.npz"))
    tiles = np.load(os.path.join(golden_dir, "cora_tiles.npz"))
    g = G.from_numpy(z["indptr"], z["indices"], device=dev)
    for T in (64, 512, 2752):
        got = ops.tile_nnz(g, T).cpu().numpy()
        assert np.array_equal(got, tiles[f"T{T}"])


def test_plan_items_and_splits(dev):
    g, ip, ix = _graph(100, 2000, seed=1, heavy_row=1000, dev=dev)
    p = ops.AggregatePlan(g, 256)
    deg = np.diff(ip)
    chunks = np.where(deg <= 256, 1, -(-deg // 256))
    assert p.n_items() == int(chunks.sum())
    assert p.n_split() == int((deg > 256).sum())


@pytest.mark.parametrize("M,K,N", [(2449, 100, 128), (1000, 602, 128), (333, 37, 50)])
def test_update_mm_f32_x_bf16_w(dev, M, K, N):
    """GTA_F32_BF16: fp32 x is rounded to bf16 (RNE) while staged; reference = fp64 of the rounded inputs."""
    rng = np.random.default_rng(K + 7)
    x = torch.from_numpy(rng.standard_normal((M, K)).astype(np.float32))
    w = torch.from_numpy(rng.standard_normal((K, N)).astype(np.float32)).to(torch.bfloat16)
    out = ops.update_mm(x.to(dev), w.to(dev), sf="RELU")
    xr = x.to(torch.bfloat16).float().numpy()
    wf = w.float().numpy()
    ref = isa_ref.mm(xr, wf, sf_kind="RELU")
    _check(out, ref, np.abs(xr).astype(np.float64) @ np.abs(wf).astype(np.float64), "update_mm f32xbf16")


@pytest.mark.parametrize("F,heads", [(128, 8), (128, 16), (128, 4), (64, 4), (256, 16), (128, 0), (64, 0)])
@pytest.mark.parametrize("blocks", [1, 7, 32, 63])
def test_aggregate_blocked_matches_oracle(dev, F, heads, blocks):
    """Column-blocked K6 (work items over B source-column slices + ordered reduce) == fp64 oracle;
    rows must be column-sorted."""
    n, e = 700, 20000
    g0 = G.synthetic(n, e, seed=blocks + F, device="cpu")          # sorted columns
    ip, ix = g0.numpy()
    deg = np.diff(ip).copy()
    deg[5] = 3000                                                   # heavy row, more edges than a block slice
    deg[[7, 8, 9]] = 0                                              # empty rows
    ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    rng = np.random.default_rng(blocks)
    ix = np.concatenate([np.sort(rng.integers(0, n, d)) for d in deg]).astype(np.int32)
    g = G.from_numpy(ip, ix, device=dev)
    x = rng.standard_normal((n, F)).astype(np.float32)
    w = rng.random((len(ix), heads)).astype(np.float32) if heads else None
    y = ops.aggregate_blocked(g, torch.from_numpy(x).to(dev), None if w is None else torch.from_numpy(w).to(dev),
                              blocks=blocks)
    ref = isa_ref.aggregate(ip, ix, x, "src", w)
    _check(y, ref, isa_ref.aggregate_abs(ip, ix, x, "src", w), f"blocked F={F} H={heads} B={blocks}")
    y2 = ops.aggregate_blocked(g, torch.from_numpy(x).to(dev), None if w is None else torch.from_numpy(w).to(dev),
                               blocks=blocks)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("row_edges", [0, 40])
@pytest.mark.parametrize("item_edges", [1, 7, 64, 256, 1 << 30])
@pytest.mark.parametrize("blocks", [1, 5, 16])
def test_blocked_plan_items(dev, item_edges, blocks, row_edges):
    """Bounded work items: every non-empty (merged block, row) segment becomes ceil(len / item_edges)
    items (empty segments none); a row of deg edges merges m = pow2 >= row_edges*B/deg blocks; the
    aggregate and the attention form still match the oracle."""
    n, e, F, H = 600, 15000, 128, 8
    g0 = G.synthetic(n, e, seed=11, device="cpu")
    ip, ix = g0.numpy()
    deg = np.diff(ip).copy()
    deg[3], deg[4] = 4000, 700                                      # heavy rows: many parts per segment
    deg[[10, 11]] = 0
    ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    rng = np.random.default_rng(item_edges % 1000 + blocks)
    ix = np.concatenate([np.sort(rng.integers(0, n, d)) for d in deg]).astype(np.int32)
    g = G.from_numpy(ip, ix, device=dev)
    plan = g.blocked_plan(blocks, item_edges, row_edges)
    bsize = -(-n // blocks)
    want = 0
    for r in range(n):
        seg = np.bincount(ix[ip[r]:ip[r + 1]] // bsize, minlength=blocks)
        m = 1
        while row_edges and deg[r] and m < blocks and deg[r] * m < row_edges * blocks:
            m *= 2
        seg = np.array([seg[j:j + m].sum() for j in range(0, blocks, m)])
        want += int(np.sum(-(-seg // item_edges)))
    assert plan.n_items == want
    x = rng.standard_normal((n, F)).astype(np.float32)
    w = rng.random((len(ix), H)).astype(np.float32)
    xd, wd = torch.from_numpy(x).to(dev), torch.from_numpy(w).to(dev)
    y = ops.aggregate_blocked(g, xd, wd, plan=plan, blocks=blocks)
    _check(y, isa_ref.aggregate(ip, ix, x, "src", w), isa_ref.aggregate_abs(ip, ix, x, "src", w),
           f"blocked items={item_edges} B={blocks}")
    assert torch.equal(y, ops.aggregate_blocked(g, xd, wd, plan=plan, blocks=blocks))
    a = rng.standard_normal((n, H)).astype(np.float64)
    b = rng.standard_normal((n, H)).astype(np.float64)
    ya, sa = ops.gat_aggregate_blocked(g, xd, torch.from_numpy(a).float().to(dev), torch.from_numpy(b).float().to(dev),
                                       want_sums=True, plan=plan, blocks=blocks)
    ref, rsum = isa_ref.gat_aggregate(ip, ix, x.astype(np.float64), a, b, "EXP_LEAKY_RELU", True)
    _check(sa, rsum, rsum, f"att sums items={item_edges}")
    v, _ = isa_ref.edge_softmax(ip, ix, a, b, "EXP_LEAKY_RELU", False)
    scale = isa_ref.aggregate(ip, ix, np.abs(x.astype(np.float64)), "src", v)
    scale = scale / np.repeat(np.where(rsum > 0, rsum, 1.0), F // H, axis=1) * 4
    _check(ya, ref, scale, f"att y items={item_edges}")


def test_aggregate_blocked_accumulate_rowscale(dev):
    n, e, F = 500, 9000, 128
    g = G.synthetic(n, e, seed=3, device=dev)
    ip, ix = g.numpy()
    rng = np.random.default_rng(0)
    x = rng.standard_normal((n, F)).astype(np.float32)
    w = rng.random((g.nnz, 8)).astype(np.float32)
    y0 = rng.standard_normal((n, F)).astype(np.float32)
    sc = (rng.random(n) + 0.5).astype(np.float32)
    yd = torch.from_numpy(y0).to(dev)
    ops.aggregate_blocked(g, torch.from_numpy(x).to(dev), torch.from_numpy(w).to(dev),
                          row_scale=torch.from_numpy(sc).to(dev), out=yd, accumulate=True, blocks=16)
    ref = y0 + isa_ref.aggregate(ip, ix, x, "src", w, sc)
    _check(yd, ref, isa_ref.aggregate_abs(ip, ix, x, "src", w, sc) + np.abs(y0), "blocked acc+scale")


def test_aggregate_blocked_rejects_unsorted_rows(dev):
    ip = np.array([0, 3, 5], dtype=np.int64)
    ix = np.array([2, 0, 1, 1, 0], dtype=np.int32)
    g = G.from_numpy(ip, ix, device=dev, n_cols=4)
    x = torch.zeros(4, 128, device=dev)
    with pytest.raises(ValueError):
        ops.aggregate_blocked(g, x, None, blocks=2)


@pytest.mark.parametrize("heads", [1, 2, 4, 8, 16, 32, 64])
@pytest.mark.parametrize("normalize", [True, False])
def test_edge_softmax_matches_oracle(dev, heads, normalize):
    """Fused GAT ops 6-10 vs the oracle's composition of the unfused ISA ops; the graph has
    empty rows, a 700-edge row (full 64-edge chunks + tail) and short rows (tail only)."""
    g, ip, ix = _graph(400, 5000, seed=3, empty_rows=20, heavy_row=700, dev=dev)
    rng = np.random.default_rng(heads)
    a = rng.standard_normal((g.n_rows, heads)).astype(np.float32)
    bt = rng.standard_normal((g.n_rows, heads + 3)).astype(np.float32)
    b = bt[:, :heads]  # leading dimension heads + 3
    out, sums = ops.edge_softmax(g, torch.from_numpy(a).to(dev), torch.from_numpy(bt).to(dev)[:, :heads],
                                 "EXP_LEAKY_RELU",
                                 normalize=normalize, want_sums=True)
    ref, rsum = isa_ref.edge_softmax(ip, ix, a.astype(np.float64), b.astype(np.float64), "EXP_LEAKY_RELU", normalize)
    _check(sums, rsum, rsum, f"edge_softmax sums H={heads}")
    # alpha = v / s: relative error of v (1 ulp) plus that of s (fp32 sum of deg terms)
    deg = np.diff(ip)[isa_ref.row_of_edge(ip)][:, None]
    _check(out, ref, np.abs(ref) * np.maximum(deg, 1), f"edge_softmax out H={heads}")
    if normalize:  # every non-empty row's alpha sums to 1 per head
        s = isa_ref.gather_add(ip, out.cpu().numpy().astype(np.float64))
        nz = np.diff(ip) > 0
        assert np.allclose(s[nz], 1.0, atol=1e-5)


def test_edge_softmax_other_sf_and_errors(dev):
    g, ip, ix = _graph(200, 2000, seed=4, dev=dev)
    a = torch.randn(g.n_rows, 8, device=dev)
    b = torch.randn(g.n_rows, 8, device=dev)
    out, sums = ops.edge_softmax(g, a, b, "SIGMOID", normalize=True)
    assert sums is None
    ref, _ = isa_ref.edge_softmax(ip, ix, a.double().cpu().numpy(), b.double().cpu().numpy(), "SIGMOID", True)
    _check(out, ref, np.abs(ref) * 64, "edge_softmax SIGMOID")
    with pytest.raises(ops._lib.GTAError):
        ops.edge_softmax(g, a[:, :6].contiguous(), b[:, :6].contiguous())
    with pytest.raises(ValueError):
        ops.edge_softmax(g, a, b[:, :4].contiguous())


@pytest.mark.parametrize("knobs", [{"seg_lean": 0}, {"seg_lean_w1": 0}, {"seg_alpha1": 0}])
@pytest.mark.parametrize("F,heads", [(128, 8), (128, 0), (64, 4), (256, 16), (128, 1)])
def test_aggregate_blocked_kernel_forms(dev, knobs, F, heads):
    """The lean half-wave kernels (k_agg_h32, also with one weight per edge, and with 8 heads' weights
    in one 8-B load per step, seg_alpha1) == the generic half-wave form / the two-load form bitwise
    (same per-item edge order, weights and fma chain), and == the fp64 oracle."""
    n, e = 900, 30000
    g = G.synthetic(n, e, seed=F + heads, device=dev)
    ip, ix = g.numpy()
    rng = np.random.default_rng(F)
    x = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(dev)
    w = torch.from_numpy(rng.random((g.nnz, heads)).astype(np.float32)).to(dev) if heads else None
    y0 = ops.aggregate_blocked(g, x, w, blocks=8)
    try:
        for k, v in knobs.items():
            ops.set_debug(k, v)
        y = ops.aggregate_blocked(g, x, w, blocks=8)
    finally:
        for k in knobs:
            ops.set_debug(k, 1)
    xn, wn = x.cpu().numpy(), None if w is None else w.cpu().numpy()
    _check(y, isa_ref.aggregate(ip, ix, xn, "src", wn), isa_ref.aggregate_abs(ip, ix, xn, "src", wn), f"{knobs}")
    assert torch.equal(y, y0)  # same per-item edge order in every half-wave form


@pytest.mark.parametrize("form", ["rows", "tile"])
@pytest.mark.parametrize("M,K,N,dt", [(5000, 602, 128, "f32"), (3001, 100, 300, "f32"), (1000, 129, 8, "f32"),
                                      (4099, 100, 128, "mixed"), (2000, 256, 200, "bf16"), (700, 77, 33, "bf16"),
                                      (130, 5, 1, "f32")])
def test_update_mm_both_forms(dev, form, M, K, N, dt):
    """Row-streaming (W^T, x read once) and 64x64-tile UPDATE kernels vs fp64 of the same (bf16-rounded)
    operands, incl. N > 128 (several column blocks), K tails and an x view with odd leading dimension."""
    rng = np.random.default_rng(M + K + N)
    xs = torch.from_numpy(rng.standard_normal((M, K + 3)).astype(np.float32))[:, 1:K + 1]  # ldx = K+3, offset 1
    w = torch.from_numpy((rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32))
    if dt == "bf16":
        xs, w = xs.to(torch.bfloat16), w.to(torch.bfloat16)
    elif dt == "mixed":
        w = w.to(torch.bfloat16)
    old = ops.MM_FORM, ops.MM_ROWS_MIN_M
    ops.MM_FORM, ops.MM_ROWS_MIN_M = form, 0
    try:
        out = ops.update_mm(xs.to(dev), w.to(dev))
    finally:
        ops.MM_FORM, ops.MM_ROWS_MIN_M = old
    xr = xs.float().numpy().astype(np.float64)
    if dt != "f32":
        xr = torch.from_numpy(xr).to(torch.bfloat16).double().numpy()
    wf = w.float().numpy().astype(np.float64)
    _check(out, xr @ wf, np.abs(xr) @ np.abs(wf), f"update_mm {form} {dt}")


def test_update_mm_weight_cache_never_stale(dev):
    """A new weight at a freed weight's address (same shape/dtype) must not reuse the old W^T."""
    x = torch.randn(40000, 64, device=dev)  # large enough for the row-streaming (W^T) form
    for seed in range(6):
        w = torch.randn(64, 32, device=dev, generator=torch.Generator(device=dev).manual_seed(seed))
        got = ops.update_mm(x, w)
        ref = (x.double() @ w.double()).float()
        assert torch.allclose(got, ref, rtol=1e-4, atol=1e-4), seed
        w.mul_(2.0)  # in-place update bumps the version: the cache must notice
        assert torch.allclose(ops.update_mm(x, w), 2 * ref, rtol=1e-4, atol=1e-4), seed
        del w


@pytest.mark.parametrize("F,heads", [(128, 8), (128, 16), (128, 1), (64, 4), (64, 16), (256, 8), (256, 16)])
@pytest.mark.parametrize("normalize", [True, False])
@pytest.mark.parametrize("blocks", [1, 5, 16])
def test_gat_aggregate_blocked_matches_oracle(dev, F, heads, normalize, blocks):
    """Fused GAT attention aggregate vs the oracle's op-by-op composition (edge softmax, alpha * x,
    gather); empty rows give 0 (normalize) and a 3000-edge row spans every block."""
    n, e = 800, 20000
    rng = np.random.default_rng(F + heads + blocks)
    deg = np.diff(G.synthetic(n, e, seed=3).numpy()[0]).copy()
    deg[11] = 3000
    deg[[3, 4]] = 0
    ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    ix = np.concatenate([np.sort(rng.integers(0, n, d)) for d in deg]).astype(np.int32)
    g = G.from_numpy(ip, ix, device=dev)
    x = rng.standard_normal((n, F)).astype(np.float32)
    a = rng.standard_normal((n, heads)).astype(np.float32)
    b = rng.standard_normal((n, heads)).astype(np.float32)
    y, sums = ops.gat_aggregate_blocked(g, torch.from_numpy(x).to(dev), torch.from_numpy(a).to(dev),
                                        torch.from_numpy(b).to(dev), normalize=normalize, want_sums=True,
                                        blocks=blocks)
    ref, rsum = isa_ref.gat_aggregate(ip, ix, x.astype(np.float64), a.astype(np.float64), b.astype(np.float64),
                                      "EXP_LEAKY_RELU", normalize)
    _check(sums, rsum, rsum, f"gat sums F={F} H={heads}")
    v, _ = isa_ref.edge_softmax(ip, ix, a.astype(np.float64), b.astype(np.float64), "EXP_LEAKY_RELU", False)
    scale = isa_ref.aggregate(ip, ix, np.abs(x.astype(np.float64)), "src", v)  # sum |v x|
    if normalize:
        hs = np.repeat(np.where(rsum > 0, rsum, 1.0), F // heads, axis=1)
        scale = scale / hs * 4  # |y| terms relative to the row sum (numerator + denominator rounding)
    _check(y, ref, scale, f"gat y F={F} H={heads} norm={normalize}")
    if normalize:
        assert torch.all(y[3] == 0) and torch.all(y[4] == 0)


@pytest.mark.parametrize("blocks,item_edges", [(1, 1 << 30), (5, 256), (16, 64), (20, 256)])
@pytest.mark.parametrize("ldb", [8, 24])
def test_gat_aggregate_lean_bitwise(dev, blocks, item_edges, ldb):
    """k_att_h32 (lean fused attention, F = 128, 8 heads) == the generic half-wave attention
    kernel bitwise (y and the per-head sums; same per-lane edge order, fma chain and sum order),
    with strided score tables and rows that are empty, short (masked steps only) and long."""
    n, e, F, H = 3000, 90000, 128, 8
    rng = np.random.default_rng(blocks + ldb)
    deg = np.diff(G.synthetic(n, e, seed=5).numpy()[0]).copy()
    deg[7], deg[8], deg[9] = 5000, 3, 0
    ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    ix = np.concatenate([np.sort(rng.integers(0, n, d)) for d in deg]).astype(np.int32)
    g = G.from_numpy(ip, ix, device=dev)
    x = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(dev)
    a = torch.from_numpy(rng.standard_normal((n, H)).astype(np.float32)).to(dev)
    bw = torch.from_numpy(rng.standard_normal((n, ldb)).astype(np.float32)).to(dev)
    b = bw[:, ldb - H:]
    plan = g.blocked_plan(blocks, item_edges)
    outs = {}
    try:
        for lean in (0, 1):
            ops.set_debug("att_lean", lean)
            outs[lean] = ops.gat_aggregate_blocked(g, x, a, b, want_sums=True, plan=plan)
    finally:
        ops.set_debug("att_lean", 1)
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])
    ref, rsum = isa_ref.gat_aggregate(ip, ix, x.cpu().numpy().astype(np.float64), a.cpu().numpy().astype(np.float64),
                                      b.cpu().numpy().astype(np.float64), "EXP_LEAKY_RELU", True)
    _check(outs[1][1], rsum, rsum, "lean gat sums")


@pytest.mark.parametrize("case", ["no_edges", "no_rows", "one_row", "dup_self"])
def test_edge_case_graphs_vs_oracle(dev, case):
    """Empty and ragged extremes through every entry point: a graph without edges, without rows,
    one row holding every edge, and duplicate edges plus self loops -- results equal the oracle."""
    rng = np.random.default_rng(5)
    if case == "no_edges":
        ip, ix = np.zeros(6, np.int64), np.zeros(0, np.int32)
    elif case == "no_rows":
        ip, ix = np.zeros(1, np.int64), np.zeros(0, np.int32)
    elif case == "one_row":
        n = 300
        ip = np.zeros(n + 1, np.int64)
        ip[n // 2 + 1:] = 9000
        ix = np.sort(rng.integers(0, n, 9000)).astype(np.int32)
    else:
        n = 50
        deg = rng.integers(0, 40, n)
        ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
        ix = np.concatenate([np.sort(np.concatenate([[r] * 3, rng.integers(0, 5, max(0, d - 3))]))[:d]
                             for r, d in enumerate(deg)]).astype(np.int32)
    n, e = len(ip) - 1, len(ix)
    ncols = max(n, 1)
    g = G.Graph(torch.from_numpy(ip).to(dev), torch.from_numpy(ix).to(dev), n_cols=ncols)
    F, H = 128, 8
    x = rng.standard_normal((ncols, F)).astype(np.float32)
    w = rng.random((e, H)).astype(np.float32)
    xd, wd = torch.from_numpy(x).to(dev), torch.from_numpy(w).to(dev)
    ref = isa_ref.aggregate(ip, ix, x, "src", w) if n else np.zeros((0, F))
    scale = isa_ref.aggregate_abs(ip, ix, x, "src", w) if n else np.zeros((0, F))
    for plan in (None, 64):
        _check(ops.aggregate(g, xd, "src", wd, plan=plan), ref, scale, f"{case} aggregate plan={plan}")
    if n:
        _check(ops.aggregate_blocked(g, xd, wd, blocks=4), ref, scale, f"{case} blocked")
        a = rng.standard_normal((n, H)).astype(np.float32)
        b = rng.standard_normal((ncols, H)).astype(np.float32)
        y, _ = ops.gat_aggregate_blocked(g, xd, torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev), blocks=4)
        yr, _ = isa_ref.gat_aggregate(ip, ix, x.astype(np.float64), a.astype(np.float64), b.astype(np.float64))
        assert np.allclose(y.cpu().numpy(), yr, rtol=1e-4, atol=1e-5)
        al, su = ops.edge_softmax(g, torch.from_numpy(a).to(dev), torch.from_numpy(b).to(dev), want_sums=True)
        ar, sr = isa_ref.edge_softmax(ip, ix, a.astype(np.float64), b.astype(np.float64))
        assert np.allclose(al.cpu().numpy(), ar, rtol=1e-4, atol=1e-6) and np.allclose(su.cpu().numpy(), sr, rtol=1e-4)
    xe = torch.from_numpy(rng.standard_normal((e, 16)).astype(np.float32)).to(dev)
    _check(ops.gather_add(g, xe), isa_ref.gather_add(ip, xe.cpu().numpy()) if n else np.zeros((0, 16)),
           isa_ref.gather_add(ip, np.abs(xe.cpu().numpy())) if n else np.zeros((0, 16)), f"{case} gather")
    for d in ("R", "C"):
        got = ops.scatter(g, xd, d)
        assert got.shape == (e, F)
        assert np.array_equal(got.cpu().numpy(), isa_ref.scatter(ip, ix, x, d))
    out = ops.apply_edge(g, "ADD", "RELU", wd, "edge", xd[:, :H].contiguous(), "src")
    assert np.allclose(out.cpu().numpy(), isa_ref.apply_edge(ip, ix, "ADD", "RELU", w, "edge", x[:, :H], "src"))
    assert ops.update_mm(xd[:0], torch.randn(F, 16, device=dev)).shape == (0, 16)
    if n:
        counts = ops.tile_nnz(g, 16).cpu().numpy()
        assert np.array_equal(counts, isa_ref.tile_nnz(ip, ix, ncols, 16))


@pytest.mark.parametrize("Fa,Fb", [(128, 128), (128, 8), (8, 128), (602, 602), (100, 4), (16, 16), (8, 1), (1, 1),
                                   (256, 16), (48, 48), (3, 3)])
@pytest.mark.parametrize("modes", [("src", "dst"), ("edge", "src"), ("dst", "edge"), ("edge", "row")])
def test_apply_edge_forms_agree(dev, Fa, Fb, modes):
    """Row-sweep K3 kernels (vector columns, packed small widths) == the generic per-element kernel,
    bitwise (same arithmetic per element), incl. head broadcast, odd widths and a broadcast b row."""
    g, ip, ix = _graph(300, 6000, seed=Fa + Fb, empty_rows=4, heavy_row=900, dev=dev)
    rng = np.random.default_rng(Fa * 7 + Fb)
    rows = {"src": g.n_rows, "dst": g.n_rows, "edge": g.nnz, "row": 1}
    a = torch.from_numpy(rng.standard_normal((rows[modes[0]], Fa)).astype(np.float32)).to(dev)
    b = torch.from_numpy(rng.standard_normal((rows[modes[1]], Fb)).astype(np.float32)).to(dev)
    bmode = "edge" if modes[1] == "row" else modes[1]
    outs = []
    for form, flat in ((0, False), (1, False), (1, True)):  # generic, row-sweep, edge-parallel (ABI 13)
        ops.set_debug("apply_edge_form", form)
        ops.APPLY_EDGE_FLAT = flat
        try:
            outs.append(ops.apply_edge(g, "MUL", "LEAKY_RELU", a, modes[0], b, bmode,
                                       b_broadcast_row=modes[1] == "row"))
        finally:
            ops.set_debug("apply_edge_form", 1)
            ops.APPLY_EDGE_FLAT = True
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])


@pytest.mark.parametrize("F", [64, 128, 256])
@pytest.mark.parametrize("n,e", [(300, 6000), (2000, 2001), (7, 31), (100, 65)])
@pytest.mark.parametrize("sf", ["NONE", "RELU", "EXP"])
def test_apply_edge_flat_bitwise(dev, F, n, e, sf):
    """gta_apply_edge_flat (32 edges per wave, whatever the rows) == the row-sweep form bitwise and the
    fp64 oracle: every operand mode, a head-broadcast b, b absent, edge counts not a multiple of 32
    or 8, empty rows."""
    g, ip, ix = _graph(n, e, seed=F + n, empty_rows=min(3, n - 1), dev=dev)
    rng = np.random.default_rng(F + e)
    rows = {"src": g.n_rows, "dst": g.n_rows, "edge": g.nnz}
    for am, bm, Fb in (("src", "dst", F), ("dst", "edge", F // 8), ("edge", "src", F), ("src", None, None)):
        a = torch.from_numpy(rng.standard_normal((rows[am], F)).astype(np.float32)).to(dev)
        b = None if bm is None else torch.from_numpy(rng.standard_normal((rows[bm], Fb)).astype(np.float32)).to(dev)
        outs = []
        for flat in (False, True):
            ops.APPLY_EDGE_FLAT = flat
            try:
                outs.append(ops.apply_edge(g, "ADD", sf, a, am, b, bm or "edge"))
            finally:
                ops.APPLY_EDGE_FLAT = True
        assert torch.equal(outs[0], outs[1]), (am, bm)
        ref = isa_ref.apply_edge(ip, ix, "ADD", sf, a.cpu().numpy(), am, None if b is None else b.cpu().numpy(), bm)
        assert np.allclose(outs[1].cpu().numpy(), ref, rtol=1e-5, atol=1e-5), (am, bm)


@pytest.mark.parametrize("pf", [0, 2])
@pytest.mark.parametrize("M,K,N,dt", [(40000, 602, 128, "f32"), (40000, 100, 128, "mixed"), (40000, 128, 64, "bf16"),
                                      (33000, 37, 200, "f32")])
def test_update_mm_prefetch_forms(dev, pf, M, K, N, dt):
    """The row GEMM with and without A-fragment prefetch: same result to the fp32 bound."""
    rng = np.random.default_rng(K + N + pf)
    x = torch.from_numpy(rng.standard_normal((M, K)).astype(np.float32))
    w = torch.from_numpy((rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32))
    if dt == "bf16":
        x, w = x.to(torch.bfloat16), w.to(torch.bfloat16)
    elif dt == "mixed":
        w = w.to(torch.bfloat16)
    ops.set_debug("mm_prefetch", pf)
    ops.set_debug("mm_ring", 0)  # k_mm_rows (the fp32 shapes default to the ring)
    try:
        out = ops.update_mm(x.to(dev), w.to(dev))
    finally:
        ops.set_debug("mm_prefetch", 1)
        ops.set_debug("mm_ring", 1)
    xr = x.float().numpy().astype(np.float64)
    if dt != "f32":
        xr = torch.from_numpy(xr).to(torch.bfloat16).double().numpy()
    wf = w.float().numpy().astype(np.float64)
    _check(out, xr @ wf, np.abs(xr) @ np.abs(wf), f"update_mm pf={pf} {dt}")


@pytest.mark.parametrize("M,K,N,dt,gathered", [(2708, 1433, 128, "f32", False), (2708, 1433, 128, "f32", True),
                                                (1000, 602, 64, "f32", False), (700, 1000, 16, "bf16", False),
                                                (1500, 300, 200, "mixed", True), (333, 290, 128, "f32", False)])
def test_update_mm_split_k(dev, M, K, N, dt, gathered):
    """Split-K UPDATE for few rows (K slices of >= 32 summed in order by k_mm_slices_sum, SF applied
    after the sum) vs fp64; deterministic run to run."""
    rng = np.random.default_rng(M + K + N)
    x = torch.from_numpy(rng.standard_normal((M + 7, K)).astype(np.float32))
    w = torch.from_numpy(rng.standard_normal((K, N)).astype(np.float32))
    if dt == "bf16":
        x, w = x.to(torch.bfloat16), w.to(torch.bfloat16)
    elif dt == "mixed":
        w = w.to(torch.bfloat16)
    idx = torch.from_numpy(rng.integers(0, M + 7, M).astype(np.int32)) if gathered else None
    assert ops._mm_splits(M, K, N, _DT[dt]) > 1
    xd, wd = x.to(dev), w.to(dev)
    idd = None if idx is None else idx.to(dev)
    out = ops.update_mm(xd, wd, idd, sf="RELU", m=None if gathered else M)
    again = ops.update_mm(xd, wd, idd, sf="RELU", m=None if gathered else M)
    assert torch.equal(out, again)
    xr = x.to(torch.bfloat16).float().numpy() if dt != "f32" else x.numpy()
    wf = w.float().numpy()
    xs = xr[idx.numpy()] if gathered else xr[:M]
    ref = isa_ref.mm(xs, wf, sf_kind="RELU")
    _check(out, ref, np.abs(xs).astype(np.float64) @ np.abs(wf).astype(np.float64), f"split-K {dt}")


@pytest.mark.parametrize("M,K,N,ldx_pad", [(2708, 1433, 128, 0), (16384, 128, 128, 0), (29000, 602, 128, 0),
                                           (44625, 500, 128, 0), (29000, 602, 256, 3), (16384, 1433, 128, 1),
                                           (2708, 128, 64, 0), (3000, 602, 128, 2)])
def test_update_mm_mid_rows_hand_written(dev, M, K, N, ldx_pad):
    """Plain fp32 UPDATE at 1,024 <= M < 65,536 rows -- GCN Cora's layers, 16,384 rows, 8-way
    Reddit (29,000) and 2-way Flickr (44,625) row shards -- on the hand-written kernels alone
    (k_mm_ring: the 8-deep split-K form for few row groups, else the 8- / 4- / 3-deep persistent
    ring): within the fp64 bound, deterministic, and bitwise equal to k_mm_rows on the same
    split plan (strided x: ldx = K + pad)."""
    rng = np.random.default_rng(M + K + N)
    x = torch.from_numpy(rng.standard_normal((M, K + ldx_pad)).astype(np.float32))[:, :K]
    w = torch.from_numpy((rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32))
    xd, wd = x.to(dev), w.to(dev)
    out = ops.update_mm(xd, wd)
    ops.set_debug("mm_ring", 0)
    try:
        own = ops.update_mm(xd, wd)
    finally:
        ops.set_debug("mm_ring", 1)
    xr, wf = x.numpy().astype(np.float64), w.numpy().astype(np.float64)
    scale = np.abs(xr) @ np.abs(wf)
    _check(out, xr @ wf, scale, "update_mm k_mm_ring")
    assert torch.equal(out, own)
    assert torch.equal(out, ops.update_mm(xd, wd))  # deterministic


@pytest.mark.parametrize("M,K,N,gathered,sf", [(40000, 602, 128, False, None), (20000, 602, 128, True, "RELU"),
                                               (33000, 37, 200, False, None), (3001, 64, 64, False, "RELU"),
                                               (17000, 1433, 128, False, None), (777, 100, 100, True, None),
                                               (130, 48, 72, False, "ELU"), (89250, 500, 128, False, None),
                                               (20000, 600, 66, False, "RELU"), (20000, 604, 64, True, None)])
def test_update_mm_ring_bitwise(dev, M, K, N, gathered, sf):
    """k_mm_ring (fp32 UPDATE through the LDS-DMA ring, the default for fp32 GEMMs) == k_mm_rows
    bitwise (same per-lane k order and MFMA chain), and both within the fp64 bound: K tails
    (register steps of 16 k), rows past M, columns past N (two column blocks at N = 200), gathered
    rows, SF epilogues, x rows not 16-B aligned (K = 602, 1433: 16-B DMA pieces at 8-B aligned
    addresses), 128- and 64-row groups, ring depths 8 / 4 / 3 (one, two and more blocks per CU).
    Shapes with enough row groups not to take the split-K form."""
    assert ops._mm_splits(M, K, N) == 1
    rng = np.random.default_rng(M + K + N)
    x = torch.from_numpy(rng.standard_normal((M + 5, K)).astype(np.float32))
    w = torch.from_numpy((rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32))
    idx = torch.from_numpy(rng.integers(0, M + 5, M).astype(np.int32)) if gathered else None
    xd, wd = x.to(dev), w.to(dev)
    idd = None if idx is None else idx.to(dev)
    outs = []
    old_min = ops.MM_ROWS_MIN_M
    try:
        ops.MM_ROWS_MIN_M = 0
        # k_mm_rows, then the ring with 128-row groups, 64-row groups, and the automatic choice
        # (K tails in registers (602, 1433) and as a ring stage (600, 604), N past the last 16-column
        # fragment (66, 100, 200), non-vector stores (N = 66))
        for ring, fr in ((0, 0), (1, 2), (1, 1), (1, 0)):
            ops.set_debug("mm_ring", ring)
            ops.set_debug("mm_ring_fr", fr)
            outs.append(ops.update_mm(xd, wd, idd, sf=sf, m=None if gathered else M))
    finally:
        ops.set_debug("mm_ring", 1)
        ops.set_debug("mm_ring_fr", 0)
        ops.MM_ROWS_MIN_M = old_min
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(outs[0], o)
    xs = x.numpy()[idx.numpy()] if gathered else x.numpy()[:M]
    ref = isa_ref.mm(xs, w.numpy(), sf_kind=sf)
    _check(outs[1], ref, np.abs(xs).astype(np.float64) @ np.abs(w.numpy()).astype(np.float64), "k_mm_ring")


@pytest.mark.parametrize("M,K", [(70000, 602), (65536, 100), (120000, 602), (120000, 128)])
def test_update_mm_default_is_the_ring(dev, M, K):
    """From 65,536 rows the DEFAULT plain fp32 UPDATE (no knobs touched) is the persistent 3-deep
    k_mm_ring: bitwise equal to k_mm_rows and within the fp64 bound.  120,000 rows: 938 128-row
    groups over 768 block slots, so K = 128 runs 64-row groups throughout."""
    rng = np.random.default_rng(M + K)
    x = torch.from_numpy(rng.standard_normal((M, K)).astype(np.float32))
    w = torch.from_numpy((rng.standard_normal((K, 128)) / np.sqrt(K)).astype(np.float32))
    xd, wd = x.to(dev), w.to(dev)
    y = ops.update_mm(xd, wd)
    try:
        ops.set_debug("mm_ring", 0)
        y_rows = ops.update_mm(xd, wd)
    finally:
        ops.set_debug("mm_ring", 1)
    torch.cuda.synchronize()
    assert torch.equal(y, y_rows)
    rows = np.arange(0, M, 97)
    ref = isa_ref.mm(x.numpy()[rows], w.numpy())
    _check(y[rows], ref, np.abs(x.numpy()[rows]).astype(np.float64) @ np.abs(w.numpy()).astype(np.float64), "default UPDATE")


@pytest.mark.parametrize("K,off", [(602, 1), (500, 3), (128, 1)])
def test_update_mm_ring_4b_aligned_rows(dev, K, off):
    """x a column window of a wider table (ldx = K + 4 + off, base off * 4 B into the row): every
    row start only 4-B aligned, as the ring's 16-B A DMA pieces allow.  Ring == k_mm_rows bitwise,
    within the fp64 bound."""
    M, N = 40000, 128  # enough row groups for the one-pass ring (no split-K)
    rng = np.random.default_rng(K + off)
    big = torch.from_numpy(rng.standard_normal((M, K + 4 + off)).astype(np.float32))
    w = torch.from_numpy((rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32))
    bd, wd = big.to(dev), w.to(dev)
    xd = bd[:, off:off + K]
    assert xd.stride(0) == K + 4 + off and xd.data_ptr() % 16 != 0 and ops._mm_splits(M, K, N) == 1
    outs = []
    old_min = ops.MM_ROWS_MIN_M
    try:
        ops.MM_ROWS_MIN_M = 0
        for ring in (0, 1):
            ops.set_debug("mm_ring", ring)
            outs.append(ops.update_mm(xd, wd))
    finally:
        ops.set_debug("mm_ring", 1)
        ops.MM_ROWS_MIN_M = old_min
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(outs[0], o)
    xs = big.numpy()[:, off:off + K]
    ref = isa_ref.mm(xs, w.numpy())
    _check(outs[1], ref, np.abs(xs).astype(np.float64) @ np.abs(w.numpy()).astype(np.float64), "ring, 4-B aligned rows")


def test_tuning_attached_to_a_stream(dev):
    """ABI 4: a knob set attached to a stream governs every call on that stream, from any thread,
    and nothing else.  Observable through seg_phase = 1 (the blocked aggregate's item launch alone:
    y is left untouched) against the default (items + ordered reduce: y written)."""
    import threading
    g = G.synthetic(2000, 40000, seed=3, device=dev)
    x = torch.randn(2000, 128, device=dev)
    w = torch.rand(g.nnz, 8, device=dev)
    y_ref = ops.aggregate_blocked(g, x, w, blocks=4)
    sentinel = torch.full_like(y_ref, 7.0)
    s = torch.cuda.Stream(dev)
    t = ops.Tuning(seg_phase=1)
    t.attach(s)
    try:
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            y_att = ops.aggregate_blocked(g, x, w, out=sentinel.clone(), blocks=4)
        out = {}

        def other():
            with torch.cuda.stream(s):
                out["y"] = ops.aggregate_blocked(g, x, w, out=sentinel.clone(), blocks=4)
            s.synchronize()
        th = threading.Thread(target=other)
        th.start()
        th.join()
        y_plain = ops.aggregate_blocked(g, x, w, out=sentinel.clone(), blocks=4)  # current stream: nothing attached
        s.synchronize()
        torch.cuda.synchronize()
        assert torch.equal(y_att, sentinel) and torch.equal(out["y"], sentinel)
        assert torch.equal(y_plain, y_ref)
        assert ops.Tuning.attached(s)
    finally:
        ops.Tuning.detach(s)
    assert not ops.Tuning.attached(s)
    with torch.cuda.stream(s):
        y_det = ops.aggregate_blocked(g, x, w, out=sentinel.clone(), blocks=4)
    s.synchronize()
    assert torch.equal(y_det, y_ref)


@pytest.mark.parametrize("M,K,N,gathered,sf", [(2708, 1433, 128, False, None), (2708, 1433, 128, True, "RELU"),
                                               (2708, 1432, 64, False, None), (1000, 1350, 64, False, None),
                                               (600, 1000, 200, False, "ELU"), (900, 700, 66, False, None)])
def test_update_mm_split_ring_bitwise(dev, M, K, N, gathered, sf):
    """Split-K UPDATE with every (128-row group, K slice) a k_mm_ring block (8-deep ring, grid.y =
    the slices) == the k_mm_rows slices bitwise (same 16-k-multiple slices), both within the fp64
    bound: x rows 4-B (K = 1433, 1350) and 16-B aligned (1432), K tails inside the last slice, two
    column blocks (N = 200), gathered rows, SF after the slice sum (float4 sum kernel); N = 66 (not a
    multiple of 4) stays on k_mm_rows and the scalar sum."""
    assert ops._mm_splits(M, K, N) > 1
    rng = np.random.default_rng(M + K + N)
    x = torch.from_numpy(rng.standard_normal((M + 5, K)).astype(np.float32))
    w = torch.from_numpy((rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32))
    idx = torch.from_numpy(rng.integers(0, M + 5, M).astype(np.int32)) if gathered else None
    xd, wd = x.to(dev), w.to(dev)
    idd = None if idx is None else idx.to(dev)
    outs = []
    try:
        for ring, fr in ((0, 0), (1, 1), (1, 2)):
            ops.set_debug("mm_ring", ring)
            ops.set_debug("mm_ring_fr", fr)
            outs.append(ops.update_mm(xd, wd, idd, sf=sf, m=None if gathered else M))
    finally:
        ops.set_debug("mm_ring", 1)
        ops.set_debug("mm_ring_fr", 0)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[0], outs[2])
    xs = x.numpy()[idx.numpy()] if gathered else x.numpy()[:M]
    ref = isa_ref.mm(xs, w.numpy(), sf_kind=sf)
    _check(outs[1], ref, np.abs(xs).astype(np.float64) @ np.abs(w.numpy()).astype(np.float64), "split k_mm_ring")


@pytest.mark.parametrize("F,heads,n_cols", [(128, 8, (1 << 23) + 77), (64, 4, (1 << 24) + 33)])
def test_aggregate_tables_past_32bit_offsets(dev, F, heads, n_cols):
    """Maximum sizes: gathered tables past the lean kernels' 32-bit addressing (2^23 + 77 rows of
    512 B = 4 GiB + 39 KB of byte offsets; 2^24 + 33 rows, past __umul24's 24-bit source ids).
    The host guards send every entry -- row-chunk plan, one wave per row, column-blocked, fused
    GAT attention -- to its 64-bit form; all match the fp64 oracle, with sources in the table's
    last rows (row 0 gathers the last 40) and a 700-edge row split across items and blocks."""
    rng = np.random.default_rng(F)
    n_rows = 3000
    deg = rng.integers(0, 40, n_rows)
    deg[0], deg[7], deg[9] = 40, 700, 0
    ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    ix = np.concatenate([np.sort(rng.integers(0, n_cols, d)) for d in deg]).astype(np.int32)
    ix[:40] = np.arange(n_cols - 40, n_cols, dtype=np.int32)
    g = G.from_numpy(ip, ix, device=dev, n_cols=n_cols)
    torch.manual_seed(F)
    xd = torch.randn(n_cols, F, device=dev)  # 4.3 GB
    uniq, local = np.unique(ix, return_inverse=True)  # the oracle sees only the gathered rows
    xs = xd[torch.from_numpy(uniq.astype(np.int64)).to(dev)].cpu().numpy().astype(np.float64)
    lx = local.astype(np.int32)
    w = rng.random((g.nnz, heads)).astype(np.float32)
    wd = torch.from_numpy(w).to(dev)
    ref = isa_ref.aggregate(ip, lx, xs, "src", w)
    scale = isa_ref.aggregate(ip, lx, np.abs(xs), "src", w)
    for name, y in (("plan", ops.aggregate(g, xd, "src", wd, plan=64)),
                    ("per-row", ops.aggregate(g, xd, "src", wd)),
                    ("blocked", ops.aggregate_blocked(g, xd, wd, blocks=4))):
        _check(y, ref, scale, f"{name} F={F} past 32-bit offsets")
    if F == 128:
        a = rng.standard_normal((n_cols, heads)).astype(np.float32)  # only gathered b rows matter
        ad, bd = torch.from_numpy(a).to(dev), torch.from_numpy(a[::-1].copy()).to(dev)
        y, sums = ops.gat_aggregate_blocked(g, xd, ad, bd, normalize=True, want_sums=True, blocks=4)
        rows = np.arange(n_rows)
        bs = a[::-1][uniq].astype(np.float64)
        aa = a[rows].astype(np.float64)
        gref, gsum = isa_ref.gat_aggregate(ip, lx, xs, aa, bs, "EXP_LEAKY_RELU", True)
        _check(sums, gsum, gsum, "gat sums past 32-bit offsets")
        v, _ = isa_ref.edge_softmax(ip, lx, aa, bs, "EXP_LEAKY_RELU", False)
        sc = isa_ref.aggregate(ip, lx, np.abs(xs), "src", v)
        sc = sc / np.repeat(np.where(gsum > 0, gsum, 1.0), F // heads, axis=1) * 4
        _check(y, gref, sc, "gat y past 32-bit offsets")


@pytest.mark.parametrize("n", [1, 37])
def test_degenerate_graphs_every_op(dev, n):
    """Graphs with no edges at all (and a single node): every op returns its defined value -- zero
    aggregates (or the untouched accumulator), empty edge tensors, zero tile counts -- and no launch
    fails (no zero-sized grids)."""
    g = G.from_numpy(np.zeros(n + 1, np.int64), np.zeros(0, np.int32), device=dev)
    F = 128
    x = torch.randn(n, F, device=dev)
    w8 = torch.zeros(0, 8, device=dev)
    assert torch.equal(ops.aggregate(g, x, "src", w8), torch.zeros(n, F, device=dev))
    assert torch.equal(ops.aggregate(g, x, "src", None, plan=64), torch.zeros(n, F, device=dev))
    acc = x.clone()
    assert torch.equal(ops.aggregate(g, x, "src", None, out=acc, accumulate=True), x)
    assert torch.equal(ops.aggregate_blocked(g, x, w8, blocks=4), torch.zeros(n, F, device=dev))
    assert ops.scatter(g, x, "C").shape == (0, F)
    assert torch.equal(ops.gather_add(g, torch.zeros(0, F, device=dev)), torch.zeros(n, F, device=dev))
    assert ops.apply_edge(g, "MUL", None, torch.zeros(0, F, device=dev), "edge", x, "src").shape == (0, F)
    a = torch.randn(n, 8, device=dev)
    out, sums = ops.edge_softmax(g, a, a.clone(), want_sums=True)
    assert out.shape == (0, 8) and torch.equal(sums, torch.zeros(n, 8, device=dev))
    y, _ = ops.gat_aggregate_blocked(g, x, a, a.clone(), blocks=4)
    assert y.shape == (n, F) and torch.equal(y, torch.zeros(n, F, device=dev))  # 0 / 0 rows give 0
    assert int(ops.tile_nnz(g, 16).sum()) == 0
    wm = torch.randn(F, 64, device=dev)
    assert ops.update_mm(x, wm).shape == (n, 64)
    assert ops.update_mm(x[:0], wm).shape == (0, 64)
    torch.cuda.synchronize()


@pytest.mark.parametrize("F,heads", [(100, 1), (100, 0), (100, 4), (128, 8), (64, 0), (3, 1), (602, 1)])
@pytest.mark.parametrize("plan", [None, 64])
@pytest.mark.parametrize("mode", ["src", "dst"])
def test_aggregate_bf16_rows(dev, F, heads, plan, mode):
    """bf16 node rows gathered by index (the GIN products byte model: 200-B rows at F = 100),
    widened exactly and summed in fp32: within the fp32 bound of the fp64 oracle on the bf16
    values; the 8-B-piece form (knob agg_bf16_vw8 = 0) is bitwise equal to the same kernel form on
    the fp32-widened table (F = 100: both run 32 lanes x 4 values per edge)."""
    n, e = 400, 7000
    g, ip, ix = _graph(n, e, seed=F + heads, heavy_row=900, empty_rows=4, dev=dev)
    rng = np.random.default_rng(F)
    x = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(torch.bfloat16)
    w = rng.random((g.nnz, heads)).astype(np.float32) if heads else None
    xd = x.to(dev)
    wd = None if w is None else torch.from_numpy(w).to(dev)
    y = ops.aggregate(g, xd, mode, wd, plan=plan)
    xf = x.float().numpy()
    _check(y, isa_ref.aggregate(ip, ix, xf, mode, w), isa_ref.aggregate_abs(ip, ix, xf, mode, w), f"bf16 F={F}")
    if F == 100:  # the 8-B-piece form (32 lanes x 4 values per edge) == the fp32 form on the widened table
        ops.set_debug("agg_bf16_vw8", 0)
        try:
            y8 = ops.aggregate(g, xd, mode, wd, plan=plan)
        finally:
            ops.set_debug("agg_bf16_vw8", 4)
        assert torch.equal(y8, ops.aggregate(g, xd.float(), mode, wd, plan=plan))
        assert torch.equal(y, ops.aggregate(g, xd, mode, wd, plan=plan))  # the default form: deterministic
    acc = torch.randn(n, F, device=dev)
    y2 = ops.aggregate(g, xd, mode, wd, out=acc.clone(), accumulate=True, plan=plan)
    _check(y2, acc.cpu().numpy() + isa_ref.aggregate(ip, ix, xf, mode, w),
           isa_ref.aggregate_abs(ip, ix, xf, mode, w) + np.abs(acc.cpu().numpy()), "bf16 accumulate")
    with pytest.raises(TypeError):
        ops.aggregate(g, torch.zeros(g.nnz, F, device=dev, dtype=torch.bfloat16), "edge")


@pytest.mark.parametrize("bin_kind,sf,Fa,Fb,bcast", [("MUL", None, 100, 1, True), ("ADD", "RELU", 128, 128, False),
                                                     (None, "ELU", 7, None, False), ("DIV", None, 100, 4, False)])
def test_apply_node_bf16_operand(dev, bin_kind, sf, Fa, Fb, bcast):
    """A bf16 `a` (GIN op 3: (1 + eps) x on the bf16 model input) widened exactly: bitwise equal to
    the fp32 call on the widened tensor, vector and generic forms alike."""
    rng = np.random.default_rng(Fa)
    n = 3001
    a = torch.from_numpy(rng.standard_normal((n, Fa)).astype(np.float32)).to(torch.bfloat16).to(dev)
    b = None if Fb is None else torch.from_numpy((rng.random((1 if bcast else n, Fb)) + 0.5).astype(np.float32)).to(dev)
    got = ops.apply_node(bin_kind, sf, a, b, b_broadcast_row=bcast)
    want = ops.apply_node(bin_kind, sf, a.float(), b, b_broadcast_row=bcast)
    assert got.dtype == torch.float32 and torch.equal(got, want)


@pytest.mark.parametrize("M,K,N,dt,gathered,sf", [(40000, 100, 128, "mixed", False, None), (40000, 128, 128, "mixed", False, "RELU"),
                                                  (30000, 128, 64, "bf16", False, None), (5000, 37, 200, "mixed", False, None),
                                                  (777, 256, 128, "mixed", True, "RELU"), (3001, 100, 130, "bf16", True, None),
                                                  (2449, 200, 128, "bf16", False, "ELU")])
def test_update_mm_ring_bf_bitwise(dev, M, K, N, dt, gathered, sf):
    """k_mm_ring_bf (bf16 MFMA with the x ring and W^T resident in LDS; the GIN MLP GEMMs) ==
    k_mm_rows bitwise (same k order, same RNE rounding of fp32 x, same zero padding) with 64- and
    128-row groups, and both within the fp32 bound of fp64 on the bf16-rounded operands: K tails,
    column blocks past N, gathered rows, SF epilogues."""
    rng = np.random.default_rng(M + K + N)
    x = torch.from_numpy(rng.standard_normal((M + 5, K)).astype(np.float32))
    w = torch.from_numpy((rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32)).to(torch.bfloat16)
    if dt == "bf16":
        x = x.to(torch.bfloat16)
    idx = torch.from_numpy(rng.integers(0, M + 5, M).astype(np.int32)) if gathered else None
    xd, wd = x.to(dev), w.to(dev)
    idd = None if idx is None else idx.to(dev)
    outs = []
    try:
        for ring, fr in ((0, 0), (1, 1), (1, 2)):
            ops.set_debug("mm_ring", ring)
            ops.set_debug("mm_ring_fr", fr)
            outs.append(ops.update_mm(xd, wd, idd, sf=sf, m=None if gathered else M))
    finally:
        ops.set_debug("mm_ring", 1)
        ops.set_debug("mm_ring_fr", 0)
    torch.cuda.synchronize()
    for o in outs[1:]:
        assert torch.equal(outs[0], o)
    xr = x.to(torch.bfloat16).float().numpy()
    xs = xr[idx.numpy()] if gathered else xr[:M]
    wf = w.float().numpy()
    ref = isa_ref.mm(xs, wf, sf_kind=sf)
    _check(outs[1], ref, np.abs(xs).astype(np.float64) @ np.abs(wf).astype(np.float64), "k_mm_ring_bf")


@pytest.mark.parametrize("dt", ["f32", "mixed"])
@pytest.mark.parametrize("K,N", [(1433, 128), (602, 128), (500, 128), (602, 256), (128, 64), (100, 128)])
@pytest.mark.parametrize("M", [2708, 16384, 29000, 44625])
def test_update_mm_hand_written_every_m(dev, M, K, N, dt):
    """every UPDATE row count runs a hand-written kernel (hipBLASLt is gone):
    GCN Cora's 2,708 rows (split-K ring slices + ordered slice sum), 16,384 / 29,000 / 44,625 rows
    (an 8-way row shard of Reddit / Flickr-scale tables: the persistent ring), fp32 and fp32 x with
    bf16 W (the bf16 ring), against the fp64 oracle on sampled rows (first, last, every 61st),
    with RELU on one shape per dtype; two calls bitwise equal."""
    gen = torch.Generator(device=dev)
    gen.manual_seed(M + K + N)
    x = torch.randn(M, K, device=dev, generator=gen)
    w = torch.randn(K, N, device=dev, generator=gen) / K ** 0.5
    if dt == "mixed":
        w = w.to(torch.bfloat16)
    sf = "RELU" if (K, N) == (602, 128) else None
    y = ops.update_mm(x, w, sf=sf)
    y2 = ops.update_mm(x, w, sf=sf)
    torch.cuda.synchronize()
    assert torch.equal(y, y2)
    rows = np.unique(np.concatenate([np.arange(0, M, 61), [M - 1]]))
    xs = x[torch.from_numpy(rows).to(dev)].cpu()
    if dt == "mixed":
        xs = xs.to(torch.bfloat16).float()
    xs = xs.numpy()
    wf = w.float().cpu().numpy()
    ref = isa_ref.mm(xs, wf, sf_kind=sf)
    _check(y[torch.from_numpy(rows).to(dev)], ref, np.abs(xs).astype(np.float64) @ np.abs(wf).astype(np.float64),
           f"UPDATE M={M} K={K} N={N} {dt}")


def _ring_vs_rows(dev, x, w, what):
    """(ring output, k_mm_rows output): the default ring form and k_mm_rows on the same call."""
    y_ring = ops.update_mm(x, w)
    try:
        ops.set_debug("mm_ring", 0)
        y_rows = ops.update_mm(x, w)
    finally:
        ops.set_debug("mm_ring", 1)
    torch.cuda.synchronize()
    assert torch.equal(y_ring, y_rows), f"{what}: ring != k_mm_rows"
    return y_ring


@pytest.mark.parametrize("M,K,N,sf,ldo_pad,x_off", [
    (40000, 602, 128, None, 0, 0), (232965, 602, 128, "RELU", 0, 0), (29000, 602, 256, None, 0, 0),
    (44625, 500, 128, "ELU", 0, 0), (20011, 37, 200, None, 0, 0), (3001, 61, 66, "RELU", 1, 0),
    (5000, 16, 72, None, 3, 0), (20000, 600, 128, None, 0, 1), (777, 1433, 100, "SIGMOID", 0, 3)])
def test_update_mm_wave_bitwise(dev, M, K, N, sf, ldo_pad, x_off):
    """k_mm_wave (fp32 UPDATE, one independent wave per block, both operands straight to registers;
    the default for N > 64, K >= 256 on enough rows) == k_mm_rows bitwise at every row-fragment
    count (FR 2 / 3 / 4 forced), the automatic plan (232,965 x 602: whole 64-row rounds, then the
    remainder rows as a second launch) and mm_wave = 2 (every shape): K tails of every class as the
    last register stage (37, 61, 600, 1433), K = 16 (one stage), columns past N (66, 72, 100, 200),
    unaligned output rows (ldo = N + 1 / + 3: element stores), x rows only 4-B aligned (a column
    window of a wider table), SF epilogues.  Within the fp64 bound."""
    rng = np.random.default_rng(M + K + N)
    big = torch.from_numpy(rng.standard_normal((M, K + x_off + (4 if x_off else 0))).astype(np.float32))
    x = big[:, x_off:x_off + K]
    w = torch.from_numpy((rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32))
    xd, wd = big.to(dev)[:, x_off:x_off + K], w.to(dev)
    outs = []
    try:
        ops.set_debug("mm_split", 0)
        for mode, fr in ((0, 0), (2, 2), (2, 3), (2, 4), (2, 0), (1, 0)):
            ops.set_debug("mm_ring", 0 if mode == 0 else 1)
            ops.set_debug("mm_wave", max(mode, 0))
            ops.set_debug("mm_wave_fr", fr)
            o = torch.full((M, N + ldo_pad), float("nan"), device=dev)[:, :N]
            outs.append(ops.update_mm(xd, wd, sf=sf, out=o))
    finally:
        for k, v in (("mm_split", -1), ("mm_ring", 1), ("mm_wave", 1), ("mm_wave_fr", 0)):
            ops.set_debug(k, v)
    torch.cuda.synchronize()
    for i, o in enumerate(outs[1:]):
        assert torch.equal(outs[0], o), i
    rows = np.arange(0, M, max(1, M // 2000))
    xs = x.numpy()[rows]
    ref = isa_ref.mm(xs, w.numpy(), sf_kind=sf)
    _check(outs[1][torch.from_numpy(rows).to(dev)], ref,
           np.abs(xs).astype(np.float64) @ np.abs(w.numpy()).astype(np.float64), "k_mm_wave")


@pytest.mark.parametrize("K", list(range(32, 65)))
def test_update_mm_ring_every_k_tail(dev, K):
    """Every K tail class of the fp32 ring (K % 16 = 0..15; K % 4 = 0 runs the tail as one more
    ring stage whose pieces past K read the row start and are zeroed, other K a register step) with
    the row-contiguous swizzled DMA lane map: bitwise equal to k_mm_rows, within the fp64 bound.
    N = 72: a partial second column fragment."""
    M, N = 3000, 72
    rng = np.random.default_rng(K)
    x = torch.from_numpy(rng.standard_normal((M, K)).astype(np.float32))
    w = torch.from_numpy((rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32))
    y = _ring_vs_rows(dev, x.to(dev), w.to(dev), f"fp32 K={K}")
    ref = isa_ref.mm(x.numpy(), w.numpy())
    _check(y, ref, np.abs(x.numpy()).astype(np.float64) @ np.abs(w.numpy()).astype(np.float64), f"ring K={K}")


@pytest.mark.parametrize("dt,K", [("mixed", k) for k in range(1, 97, 3)] + [("bf16", k) for k in range(8, 97, 8)])
def test_update_mm_ring_bf_every_k_tail(dev, dt, K):
    """The bf16 ring's K tails (32-k stages; a tail whose 16-B pieces lie wholly inside or past K
    is one more ring stage, otherwise a masked register step) for fp32 x rounded to bf16 (K = 1,
    4, ..., 94) and bf16 x (K = 8, ..., 96): bitwise equal to k_mm_rows, within the fp32 bound of
    fp64 on the bf16-rounded operands."""
    M, N = 2500, 128
    rng = np.random.default_rng(K + 7)
    x = torch.from_numpy(rng.standard_normal((M, K)).astype(np.float32))
    w = torch.from_numpy((rng.standard_normal((K, N)) / np.sqrt(K)).astype(np.float32)).to(torch.bfloat16)
    if dt == "bf16":
        x = x.to(torch.bfloat16)
    y = _ring_vs_rows(dev, x.to(dev), w.to(dev), f"{dt} K={K}")
    xr = x.to(torch.bfloat16).float().numpy()
    wf = w.float().numpy()
    _check(y, isa_ref.mm(xr, wf), np.abs(xr).astype(np.float64) @ np.abs(wf).astype(np.float64), f"ring_bf {dt} K={K}")


@pytest.mark.parametrize("F,H", [(128, 8), (64, 4), (256, 8)])
@pytest.mark.parametrize("blocks", [1, 2, 4])
@pytest.mark.parametrize("sf_out", ["ELU", "RELU", "EXP", "SIGMOID"])
@pytest.mark.parametrize("normalize", [True, False])
def test_gat_aggregate_fused_output_sf(dev, F, H, blocks, sf_out, normalize):
    """ABI 6 sf_out: the SF that follows GAT's aggregate (op 13) applied as y is written, by the
    ordered reduce and by k_att_h32's direct epilogue (a row's only item, B <= 2): bitwise equal
    to the aggregate followed by apply_node's SF, rows without edges included (sf(0)); per-head
    sums untouched.  Lean (F = 128, 8 heads) and generic forms."""
    n, e = 2000, 30000
    rng = np.random.default_rng(F + blocks)
    deg = np.diff(G.synthetic(n, e, seed=9).numpy()[0]).copy()
    deg[3], deg[4], deg[5] = 0, 1, 2500
    ip = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    ix = np.concatenate([np.sort(rng.integers(0, n, d)) for d in deg]).astype(np.int32)
    g = G.from_numpy(ip, ix, device=dev)
    x = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(dev)
    a = torch.from_numpy(rng.standard_normal((n, H)).astype(np.float32)).to(dev)
    b = torch.from_numpy(rng.standard_normal((n, H)).astype(np.float32)).to(dev)
    y0, s0 = ops.gat_aggregate_blocked(g, x, a, b, normalize=normalize, want_sums=True, blocks=blocks)
    y1, s1 = ops.gat_aggregate_blocked(g, x, a, b, normalize=normalize, want_sums=True, blocks=blocks, sf_out=sf_out)
    want = ops.apply_node(None, sf_out, y0)
    torch.cuda.synchronize()
    assert torch.equal(y1, want)
    assert torch.equal(s0, s1)


@pytest.mark.parametrize("dt", ["bf16", "f32"])
@pytest.mark.parametrize("F,heads", [(100, 1), (100, 0), (128, 8), (64, 0)])
@pytest.mark.parametrize("plan", [None, 64])
def test_aggregate_self_term(dev, dt, F, heads, plan):
    """ABI 7 gta_aggregate_self: y = x_self * s + sum (GIN ops 3-4 in one launch) is bitwise equal to
    apply_node("MUL", x_self, s) followed by the aggregate accumulating into it -- split rows
    (plan 64: a 900-edge row across chunks, summed by the combine kernel) and empty rows included."""
    n, e = 500, 9000
    g, ip, ix = _graph(n, e, seed=F + heads, heavy_row=900, empty_rows=5, dev=dev)
    rng = np.random.default_rng(F)
    tdt = torch.bfloat16 if dt == "bf16" else torch.float32
    x = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(tdt).to(dev)
    w = torch.from_numpy(rng.random((g.nnz, heads)).astype(np.float32)).to(dev) if heads else None
    s = torch.tensor([[1.1]], device=dev)
    t = ops.apply_node("MUL", None, x, s, b_broadcast_row=True)
    want = ops.aggregate(g, x, "src", w, out=t, accumulate=True, plan=plan)
    got = ops.aggregate(g, x, "src", w, plan=plan, self_term=(x, s))
    torch.cuda.synchronize()
    assert torch.equal(got, want)


@pytest.mark.parametrize("dt", ["bf16", "f32"])
@pytest.mark.parametrize("F,heads", [(100, 0), (128, 8), (36, 1)])
@pytest.mark.parametrize("plan", [None, 64])
def test_aggregate_self_term_bf16_out(dev, dt, F, heads, plan):
    """ABI 10 bf16 y of gta_aggregate_self (the GIN sum handed to the fused MLP) == the fp32 y rounded
    to nearest even, bitwise: per-row and split rows (the combine kernel's store), empty rows, F
    not a multiple of 8 (the fresh [N, ceil8(F)] rows); the columns past F are never written."""
    n, e = 500, 9000
    g, ip, ix = _graph(n, e, seed=F + heads + 7, heavy_row=900, empty_rows=5, dev=dev)
    rng = np.random.default_rng(F + 1)
    tdt = torch.bfloat16 if dt == "bf16" else torch.float32
    x = torch.from_numpy(rng.standard_normal((n, F)).astype(np.float32)).to(tdt).to(dev)
    w = torch.from_numpy(rng.random((g.nnz, heads)).astype(np.float32)).to(dev) if heads else None
    s = torch.tensor([[1.1]], device=dev)
    want = ops.aggregate(g, x, "src", w, plan=plan, self_term=(x, s))
    got = ops.aggregate(g, x, "src", w, plan=plan, self_term=(x, s), out_dtype=torch.bfloat16)
    assert got.dtype == torch.bfloat16 and got.shape == (n, F) and got.stride(0) % 8 == 0
    pad = torch.full((n, 48), 7.0, dtype=torch.bfloat16, device=dev)  # a caller's out with a guard band
    got2 = ops.aggregate(g, x, "src", w, plan=plan, self_term=(x, s), out_dtype=torch.bfloat16,
                         out=pad[:, :F] if F <= 40 else None)
    torch.cuda.synchronize()
    assert torch.equal(got, want.to(torch.bfloat16))
    assert torch.equal(got2, got)
    if F <= 40:
        assert bool((pad[:, F:] == 7.0).all())
    with pytest.raises(ValueError):
        ops.aggregate(g, x, "src", w, plan=plan, out_dtype=torch.bfloat16)  # no self term: fp32 only


@pytest.mark.parametrize("M,K1,N1,N2,sf1,sf2", [(20000, 100, 128, 128, "RELU", "RELU"), (4099, 36, 64, 20, None, "ELU"),
                                                (33, 128, 20, 8, "SIGMOID", None)])
def test_update_mlp_bf16_x(dev, M, K1, N1, N2, sf1, sf2):
    """ABI 10 bf16 x of gta_update_mlp (the aggregate's bf16 GIN sum) gives the bits of the fp32 x it
    was rounded from (the kernel rounds an fp32 x to bf16 on load): one 16-B piece per step, the K
    tail of a 36-wide row masked by 4-column pairs, rows padded to a multiple of 8."""
    rng = np.random.default_rng(M + K1)
    x = torch.from_numpy(rng.standard_normal((M, K1)).astype(np.float32)).to(dev)
    w1 = torch.from_numpy((rng.standard_normal((K1, N1)) / np.sqrt(K1)).astype(np.float32)).to(torch.bfloat16).to(dev)
    w2 = torch.from_numpy((rng.standard_normal((N1, N2)) / np.sqrt(N1)).astype(np.float32)).to(torch.bfloat16).to(dev)
    ld = (K1 + 7) // 8 * 8
    xbuf = torch.full((M, ld), float("nan"), dtype=torch.bfloat16, device=dev)  # NaN past K1: must not be read
    xb = xbuf[:, :K1]
    xb.copy_(x.to(torch.bfloat16))
    assert ops.update_mlp_supported(xb, w1, w2)
    want = ops.update_mlp(x, w1, w2, sf1=sf1, sf2=sf2)
    got = ops.update_mlp(xb, w1, w2, sf1=sf1, sf2=sf2)
    torch.cuda.synchronize()
    assert torch.equal(got, want)
    if K1 % 8:
        assert not ops.update_mlp_supported(torch.empty(M, K1, dtype=torch.bfloat16, device=dev)[1:], w1, w2)


@pytest.mark.parametrize("M,K1,N1,N2,sf1,sf2", [(20000, 100, 128, 128, "RELU", "RELU"), (4099, 128, 128, 128, None, "ELU"),
                                                (3001, 64, 96, 48, "SIGMOID", None), (777, 100, 128, 100, "RELU", None),
                                                (33, 36, 20, 8, "EXP", "RELU"), (5, 128, 128, 128, "RELU", "RELU")])
def test_update_mlp_bitwise(dev, M, K1, N1, N2, sf1, sf2):
    """gta_update_mlp (GIN's MM -> SF -> MM -> SF in one pass, no [M, N1] intermediate in HBM) ==
    the two unfused mixed-precision UPDATEs bitwise: fp32 x rounded to bf16 as the first GEMM stages
    it, the SF'd intermediate rounded to bf16 as the second GEMM stages it, the same k order; K and N
    tails (36, 20, 8, 100, 96, 48), an SF with sf(0) != 0 in front of zero-padded k (SIGMOID, EXP),
    row counts not a multiple of 16.  Both within the fp32 bound of fp64 on the bf16-rounded operands."""
    rng = np.random.default_rng(M + K1 + N1 + N2)
    x = torch.from_numpy(rng.standard_normal((M, K1)).astype(np.float32)).to(dev)
    w1 = torch.from_numpy((rng.standard_normal((K1, N1)) / np.sqrt(K1)).astype(np.float32)).to(torch.bfloat16).to(dev)
    w2 = torch.from_numpy((rng.standard_normal((N1, N2)) / np.sqrt(N1)).astype(np.float32)).to(torch.bfloat16).to(dev)
    assert ops.update_mlp_supported(x, w1, w2)
    fused = ops.update_mlp(x, w1, w2, sf1=sf1, sf2=sf2)
    z = ops.update_mm(x, w1, sf=sf1)
    ref2 = ops.update_mm(z, w2, sf=sf2)
    torch.cuda.synchronize()
    assert torch.equal(fused, ref2)
    xb = x.to(torch.bfloat16).double().cpu().numpy()
    zr = isa_ref.mm(xb, w1.double().cpu().numpy(), sf_kind=sf1)
    zb = torch.from_numpy(zr.astype(np.float32)).to(torch.bfloat16).double().numpy()
    # the fp64 intermediate and the GPU's fp32 one may round to neighbouring bf16 values: compare
    # against fp64 of the GPU's own bf16 intermediate, bound from |z| |W2|
    zg = z.to(torch.bfloat16).double().cpu().numpy()
    ref = isa_ref.mm(zg, w2.double().cpu().numpy(), sf_kind=sf2)
    _check(fused, ref, np.abs(zg) @ np.abs(w2.double().cpu().numpy()), "update_mlp")
    assert np.abs(zb - zg).max() <= 2 ** -7 * np.abs(zb).max() + 1e-6  # neighbouring bf16 values at most


# ---- ABI 11: the CSC view and the ISA gather with DIRECTION src (ORDER C) ----------------------
def _csc_cases():
    """(name, indptr, indices, n_cols): lognormal rows, empty rows and columns, duplicate edges, self
    loops, one heavy row, a rectangular CSR, n_cols needing 1, 2 and 3 radix passes, no edges."""
    out = []
    g = G.synthetic(3000, 40000, seed=1)
    ip, ix = g.numpy()
    out.append(("lognormal", ip, ix, 3000))
    rng = np.random.default_rng(2)
    deg = rng.integers(0, 6, 200)
    deg[[3, 50, 199]] = 0
    deg[100] = 9000  # one heavy row
    ip2 = np.concatenate([[0], np.cumsum(deg)]).astype(np.int64)
    ix2 = rng.integers(0, 200, int(ip2[-1])).astype(np.int32)  # duplicates and self loops
    ix2[ip2[10]:ip2[11]] = 10
    out.append(("dup_self_heavy", ip2, ix2, 200))
    out.append(("rect_wide", ip2, rng.integers(0, 70000, int(ip2[-1])).astype(np.int32), 70000))  # 2 passes
    out.append(("three_passes", ip2, rng.integers(0, 1 << 20, int(ip2[-1])).astype(np.int32), (1 << 20) + 3))
    out.append(("one_col", ip2, np.zeros(int(ip2[-1]), np.int32), 1))
    out.append(("no_edges", np.zeros(51, np.int64), np.zeros(0, np.int32), 50))
    return out


@pytest.mark.parametrize("case", range(6))
def test_csc_build_is_the_stable_source_sort(dev, case):
    """gta_csc_build == numpy's stable argsort by source column, bit-exact (perm, colptr, rows)."""
    name, ip, ix, nc = _csc_cases()[case]
    g = G.from_numpy(ip, ix, device=dev, n_cols=nc)
    c = ops.CSC(g)
    perm = np.argsort(ix, kind="stable")
    colptr = np.concatenate([[0], np.cumsum(np.bincount(ix, minlength=nc))]).astype(np.int64)
    assert np.array_equal(c.colptr.cpu().numpy(), colptr), name
    assert np.array_equal(c.perm.cpu().numpy(), perm), name
    assert np.array_equal(c.rows.cpu().numpy(), isa_ref.row_of_edge(ip)[perm]), name
    c2 = ops.CSC(g)  # a pure function of the graph
    assert torch.equal(c.perm, c2.perm) and torch.equal(c.colptr, c2.colptr)


@pytest.mark.parametrize("case", [0, 1, 2, 4, 5])
@pytest.mark.parametrize("F", [1, 16, 128, 130])
def test_gather_add_direction_c(dev, case, F):
    """gather C: y[j] = sum_{e: src(e) = j} xe[e] vs the fp64 oracle (per-element bound), repeat
    runs bitwise equal, accumulate; empty columns are 0 (or keep y)."""
    name, ip, ix, nc = _csc_cases()[case]
    g = G.from_numpy(ip, ix, device=dev, n_cols=nc)
    rng = np.random.default_rng(F)
    xe = rng.standard_normal((len(ix), F)).astype(np.float32)
    xd = torch.from_numpy(xe).to(dev)
    y = ops.gather_add(g, xd, direction="C")
    ref = isa_ref.gather_add(ip, xe, "C", ix, nc)
    _check(y, ref, isa_ref.gather_add(ip, np.abs(xe), "C", ix, nc), f"gather C {name} F={F}")
    assert torch.equal(y, ops.gather_add(g, xd, direction="C"))
    y0 = rng.standard_normal((nc, F)).astype(np.float32)
    yd = torch.from_numpy(y0).to(dev)
    ops.gather_add(g, xd, out=yd, accumulate=True, direction="C")
    _check(yd, y0 + ref, np.abs(y0) + isa_ref.gather_add(ip, np.abs(xe), "C", ix, nc), f"gather C acc {name}")
    # direction R through the same entry point
    if case != 5:
        _check(ops.gather_add(g, xd, direction="R"), isa_ref.gather_add(ip, xe), isa_ref.gather_add(ip, np.abs(xe)),
               f"gather R {name}")


@pytest.mark.parametrize("kind", ["dst", "src", "edge"])
def test_csc_views_aggregate(dev, kind):
    """The transposed aggregate the executor runs for gather C of a fused producer: weighted sums
    over a source column's edges of x[dst(e)] (scatter R), x[src(e)] (scatter C) or xe[e]."""
    name, ip, ix, nc = _csc_cases()[1]
    n = len(ip) - 1
    g = G.from_numpy(ip, ix, device=dev, n_cols=nc)
    c = ops.CSC(g)
    rng = np.random.default_rng(3)
    w = rng.random((len(ix), 4)).astype(np.float32)
    wc = ops.apply_edge(c.view("edge"), None, None, torch.from_numpy(w).to(dev), "src")
    assert torch.equal(wc.cpu(), torch.from_numpy(w[np.argsort(ix, kind="stable")]))  # a bit-exact permuting copy
    rows = {"dst": n, "src": nc, "edge": len(ix)}[kind]
    x = rng.standard_normal((rows, 32)).astype(np.float32)
    y = ops.aggregate(c.view(kind), torch.from_numpy(x).to(dev), "src", wc, plan=64)
    mode = {"dst": "dst", "src": "src", "edge": "edge"}[kind]
    xe = isa_ref.edge_operand(ip, ix, x.astype(np.float64), mode) * np.repeat(w, 8, axis=1)
    ref = isa_ref.gather_add(ip, xe, "C", ix, nc)
    _check(y, ref, isa_ref.gather_add(ip, np.abs(xe), "C", ix, nc), f"csc view {kind}")


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_update_mlp_one_row_products_width(dev, dtype):
    """a one-row x at GIN products' width (K1 = 100, a row stride the kernel would reject
    for bf16) runs the fused MLP; same bits as the same row inside a larger batch."""
    rng = np.random.default_rng(3)
    w1 = torch.from_numpy((rng.standard_normal((100, 128)) / 10).astype(np.float32)).to(torch.bfloat16).to(dev)
    w2 = torch.from_numpy((rng.standard_normal((128, 128)) / 11).astype(np.float32)).to(torch.bfloat16).to(dev)
    big = torch.zeros(64, 104, device=dev, dtype=dtype)[:, :100]  # rows padded to 16 B: a batch the kernel takes
    big.copy_(torch.from_numpy(rng.standard_normal((64, 100)).astype(np.float32)).to(dev).to(dtype))
    one = big[5:6].clone()  # a fresh [1, 100] tensor: stride 100
    assert ops.update_mlp_supported(one, w1, w2)
    got = ops.update_mlp(one, w1, w2, sf1="RELU", sf2="RELU")
    ref = ops.update_mlp(big, w1, w2, sf1="RELU", sf2="RELU")[5:6]
    torch.cuda.synchronize()
    assert torch.equal(got, ref)


@pytest.mark.parametrize("F", [100, 128, 36, 12, 8, 200])
@pytest.mark.parametrize("form", ["plain", "self_f32", "self_bf16"])
def test_aggregate_bf16_16B_pieces(dev, F, form):
    """bf16 rows gathered in 16-B pieces (knob agg_bf16_vw8, the default for unweighted bf16 gathers:
    GIN products' 200-B rows in 13 lanes, 4 edges per wave instruction; F % 8 == 4 clamps the last
    lane's piece inside the row) vs the fp64 oracle at the per-element bound, against the 8-B-piece
    form at the same bound, deterministic; heavy rows split by the plan, empty rows, the last table
    row gathered (its clamped piece must stay inside the allocation)."""
    g, ip, ix = _graph(500, 9000, seed=F, heavy_row=2000, empty_rows=4, dev=dev)
    ix = ix.copy()
    ix[:50] = 499  # the table's last row
    g = G.from_numpy(ip, ix, device=dev)
    rng = np.random.default_rng(F)
    x = torch.from_numpy(rng.standard_normal((500, F)).astype(np.float32)).to(dev).to(torch.bfloat16)
    xn = x.float().cpu().numpy().astype(np.float64)
    s = torch.tensor([[1.25]], device=dev)
    ref, mag = isa_ref.aggregate(ip, ix, xn, "src", None), isa_ref.aggregate_abs(ip, ix, xn, "src", None)
    if form != "plain":
        ref, mag = ref + 1.25 * xn, mag + 1.25 * np.abs(xn)
    outs = {}
    for vw8 in (4, 8, 0):
        ops.set_debug("agg_bf16_vw8", vw8)
        try:
            kw = {} if form == "plain" else {"self_term": (x, s),
                                             "out_dtype": torch.bfloat16 if form == "self_bf16" else torch.float32}
            y = ops.aggregate(g, x, "src", None, plan=64, **kw)
            y2 = ops.aggregate(g, x, "src", None, plan=64, **kw)
        finally:
            ops.set_debug("agg_bf16_vw8", 4)
        torch.cuda.synchronize()
        assert torch.equal(y, y2)
        got = y.float().cpu().numpy().astype(np.float64)
        bound = 1e-5 * mag + 1e-6 + (2.0 ** -8 * np.abs(ref) if form == "self_bf16" else 0)
        err = np.abs(got - ref)
        assert (err <= bound).all(), f"vw8={vw8}: max err {err.max():.3e}"
        outs[vw8] = y


@pytest.mark.parametrize("F,dtype,mode", [(100, "bf16", "src"), (100, "bf16", "dst"), (100, "f32", "src"),
                                          (128, "f32", "src"), (602, "f32", "dst"), (16, "f32", "src"),
                                          (3, "f32", "edge"), (36, "bf16", "src")])
@pytest.mark.parametrize("plan", [None, 64])
def test_aggregate_one_weight_per_edge(dev, F, dtype, mode, plan):
    """One weight per edge ([E, 1]: GCN's normalisation, GIN's edge operand) takes 64 weights per
    load beside the indices, broadcast like them (knob agg_w1, default): bitwise equal to the
    per-lane weight loads it replaces (agg_w1 = 0) in the same lane layout, and within the fp64
    bound in every form (bf16: also the 16-B-piece form, GIN products' layer)."""
    n, e = 450, 8000
    g, ip, ix = _graph(n, e, seed=F + 7, heavy_row=1500, empty_rows=3, dev=dev)
    rng = np.random.default_rng(F)
    rows = g.nnz if mode == "edge" else n
    xf = rng.standard_normal((rows, F)).astype(np.float32)
    x = torch.from_numpy(xf).to(dev)
    if dtype == "bf16":
        x = x.to(torch.bfloat16)
        xf = x.float().cpu().numpy()
    w = (rng.random((g.nnz, 1)) + 0.5).astype(np.float32)
    wd = torch.from_numpy(w).to(dev)
    ref, mag = isa_ref.aggregate(ip, ix, xf, mode, w), isa_ref.aggregate_abs(ip, ix, xf, mode, w)
    outs = {}
    for w1 in (1, 0):
        ops.set_debug("agg_w1", w1)
        ops.set_debug("agg_bf16_vw8", 0)
        try:
            outs[w1] = ops.aggregate(g, x, mode, wd, plan=plan)
        finally:
            ops.set_debug("agg_w1", 1)
            ops.set_debug("agg_bf16_vw8", 4)
    y = ops.aggregate(g, x, mode, wd, plan=plan)  # the defaults (bf16: 16-B pieces)
    torch.cuda.synchronize()
    assert torch.equal(outs[1], outs[0])
    for name, t in (("edge1", outs[1]), ("default", y)):
        err = np.abs(t.cpu().numpy().astype(np.float64) - ref)
        assert (err <= 1e-5 * mag + 1e-6).all(), f"{name}: max err {err.max():.3e}"


@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("form", ["plain", "self_bf16"])
def test_aggregate_line_pitched_table(dev, weighted, form):
    """A node table on line-pitched storage (ops.pitched: GIN products' 200-B bf16 rows at a 256-B
    pitch, what workloads.make_tensors builds) gives bitwise the sums of the same values stored
    contiguously: the pitch changes addresses only.  The table's last row is gathered too."""
    g, ip, ix = _graph(500, 9000, seed=11, heavy_row=2000, empty_rows=4, dev=dev)
    ix = ix.copy()
    ix[:40] = 499
    g = G.from_numpy(ip, ix, device=dev)
    rng = np.random.default_rng(5)
    x = torch.from_numpy(rng.standard_normal((500, 100)).astype(np.float32)).to(dev).to(torch.bfloat16)
    xp = ops.pitched(x)
    assert xp.stride(0) == 128 and torch.equal(xp, x)
    wd = torch.from_numpy((rng.random((g.nnz, 1)) + 0.5).astype(np.float32)).to(dev) if weighted else None
    s = torch.tensor([[1.1]], device=dev)
    res = []
    for t in (x, xp):
        kw = {} if form == "plain" else {"self_term": (t, s), "out_dtype": torch.bfloat16}
        res.append(ops.aggregate(g, t, "src", wd, plan=64, **kw))
    torch.cuda.synchronize()
    assert torch.equal(res[0], res[1])


@pytest.mark.parametrize("pf", [1, 2, 3, 4, 5])
@pytest.mark.parametrize("n,e,blocks", [(900, 30000, 8), (3000, 600000, 2), (5, 2000, 1)])
def test_aggregate_blocked_scalar_prefetch_bitwise(dev, pf, n, e, blocks):
    """k_agg_h32pf (round 6, knob seg_pf: alpha / index lines pre-fetched into L2 by scalar loads,
    indices broadcast by DPP row_newbcast instead of ds_swizzle) == k_agg_h32's 8-head form bitwise,
    on short items, multi-chunk items (several prefetch steps and index chunks) and 256-edge items
    of a few very heavy rows; and == the fp64 oracle."""
    g = G.synthetic(n, e, seed=n + pf, device=dev)
    ip, ix = g.numpy()
    rng = np.random.default_rng(n)
    x = torch.from_numpy(rng.standard_normal((n, 128)).astype(np.float32)).to(dev)
    w = torch.from_numpy(rng.random((g.nnz, 8)).astype(np.float32)).to(dev)
    old = ops.get_debug("seg_pf")
    try:
        ops.set_debug("seg_pf", 0)
        y0 = ops.aggregate_blocked(g, x, w, blocks=blocks)
        ops.set_debug("seg_pf", pf)
        y = ops.aggregate_blocked(g, x, w, blocks=blocks)
    finally:
        ops.set_debug("seg_pf", old)
    torch.cuda.synchronize()
    xn, wn = x.cpu().numpy(), w.cpu().numpy()
    _check(y, isa_ref.aggregate(ip, ix, xn, "src", wn), isa_ref.aggregate_abs(ip, ix, xn, "src", wn), f"seg_pf={pf}")
    assert torch.equal(y, y0)
