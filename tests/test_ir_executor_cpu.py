"""IR parsing of every golden stream/op graph, and the executor's block planning on CPU.

The executor is driven through tests/fake_ops.py (oracle-backed, CPU) so the
mapping of blocks/fused COMPs to kernels is checked here without a GPU; the
same streams run on the real kernels in test_gpu_executor.py.
"""
import os

import numpy as np
import pytest
import torch

from gta_graph_tensor_acclelrator_for_general_gnn_amd import executor, graph as G, ir, workloads
from gta_graph_tensor_acclelrator_for_general_gnn_amd.semantics import Semantics
from oracle.exec_ref import execute_ref

from . import fake_ops
from .conftest import load_manifest


def _streams(manifest, dataset="cora"):
    return [s for s in manifest["streams"] if "file" in s and s["dataset"] == dataset]


def test_every_op_yaml_parses(golden_dir, manifest):
    for rec in manifest["ops"]:
        g = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["file"]),
                            Semantics.for_network(rec["network"], rec["reorder"]).inputs)
        assert len(g) >= 4
        g.topo()  # acyclic after resolution


def test_parse_metric_stream(golden_dir):
    s = ir.Stream.load(os.path.join(golden_dir, "streams", "GAT-reddit-layer1-original-h512.yaml"))
    blk = [b for b in s if set(b.ops) == {3, 11, 12}][0]
    assert blk.fused == [(11, 12, ["MUL", "ADD"])]
    comp = [i for i in blk.insts if i.kind == "comp"][0]
    assert comp.type == "COMP_MUL_COMP_ADD" and comp.id == "11_applyedge_0_12_gather_0"
    assert comp.tile_times == 106232040 and comp.tile_size == 512
    assert not any(i.type == "FETCH" for i in blk.insts)  # fuse_fetch removed the scatter's FETCH
    assert blk.stored == [12]


def test_block_order_is_dependency_order(golden_dir, manifest):
    for rec in _streams(manifest):
        sem = Semantics.for_network(rec["network"], rec["reorder"])
        g = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
        s = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
        ex = executor.Executor(g, s, None, {}, sem)
        order = ex.block_order()
        seen = set()
        for bi in order:
            b = s.blocks[bi]
            for o in b.ops:
                for p in g.producers(o):
                    assert p in seen or p in b.ops, (rec["file"], o, p)
            seen.update(b.ops)


def _cora_graph(golden_dir):
    z = np.load(os.path.join(golden_dir, "cora_graph.npz"))
    return G.from_numpy(z["indptr"], z["indices"]), z["indptr"], z["indices"]


def compare(values_ex, ref, ops_to_check, rtol=1e-4):
    for i in ops_to_check:
        got = values_ex[i].detach().cpu().double().numpy()
        exp = ref[i][1]
        assert got.shape == exp.shape, (i, got.shape, exp.shape)
        nan_g, nan_e = ~np.isfinite(got), ~np.isfinite(exp)
        assert np.array_equal(nan_g, nan_e), f"op {i}: non-finite pattern differs"
        got, exp = got[~nan_e], exp[~nan_e]
        if exp.size == 0:
            continue
        scale = np.abs(exp).max() + 1e-30
        err = np.abs(got - exp).max() / scale
        assert err <= rtol, f"op {i}: normalised max err {err:.2e}"


CORA_STREAMS = _streams(load_manifest())


@pytest.mark.parametrize("idx", range(len(CORA_STREAMS)), ids=[r["file"][:-5] for r in CORA_STREAMS])
def test_executor_plans_every_golden_stream(golden_dir, manifest, monkeypatch, idx):
    rec = CORA_STREAMS[idx]
    monkeypatch.setattr(executor, "ops", fake_ops)
    g, ip, ix = _cora_graph(golden_dir)
    sem = Semantics.for_network(rec["network"], rec["reorder"])
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    tensors = workloads.make_tensors(og, g, rec["network"], seed=idx)
    ex = executor.Executor(og, st, g, tensors, sem, plan_chunk=0)
    outs = ex.run()
    ref = execute_ref(og, sem, ip, ix, {k: v.numpy() for k, v in tensors.items()})
    vals = {i: ex.tensor_of(i) for i in range(len(og))}
    compare(vals, ref, range(len(og)))
    assert set(outs) == {op.idx for op in og.ops if not op.out_list}
    # the GPU tests' op-local per-element check (oracle/sampled.py), here over the fp64 stand-in
    from oracle.sampled import SampledChecker
    SampledChecker(ex, ip, ix).check(n_samples=200, n_gather=200, seed=idx)


@pytest.mark.parametrize("network,reorder,expect", [
    ("GAT", False, {6: {"A": 6, "V": 7, "G": 8, "D": 9, "S": 10}}),
    ("GAT", True, {6: {"A": 6, "V": 8, "G": 9, "D": None}}),
    ("GCN", False, {}), ("GIN", False, {}), ("GraphSAGE", True, {}),
])
def test_softmax_chain_matching(golden_dir, network, reorder, expect):
    """GAT ops 6-10 (genGraphOP.py:51-60) are recognised as one edge-softmax; nothing else is."""
    sem = Semantics.for_network(network, reorder)
    g = ir.OpGraph.load(os.path.join(golden_dir, "ops", f"{network}-cora-layer1-{'trans' if reorder else 'original'}.yaml"),
                        sem.inputs)
    assert executor.Executor(g, None, None, {}, sem).softmax == expect


@pytest.mark.parametrize("reorder", [False, True])
def test_softmax_fusion_cpu_equivalence(golden_dir, manifest, monkeypatch, reorder):
    monkeypatch.setattr(executor, "ops", fake_ops)
    rec = [s for s in _streams(manifest) if s["network"] == "GAT" and s["reorder"] == reorder][1]
    sem = Semantics.for_network("GAT", reorder)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    gc, ip, ix = _cora_graph(golden_dir)
    tensors = workloads.make_tensors(og, gc, "GAT", seed=1)
    runs = []
    for fuse in (True, False):
        ex = executor.Executor(og, st, gc, tensors, sem)
        ex.fuse_softmax = fuse
        runs.append((ex.run(), ex.launches))
    assert runs[0][1] < runs[1][1]
    ref = execute_ref(og, sem, ip, ix, {k: v.double().numpy() for k, v in tensors.items()})
    for outs, _ in runs:
        compare(outs, ref, outs.keys())


@pytest.mark.parametrize("network", ["GraphSAGE", "GCN", "SGC"])
def test_mm_first_reordering_cpu(golden_dir, manifest, monkeypatch, network):
    """gather -> narrowing MM runs as MM -> aggregate: fewer algorithmic bytes, the MM's value
    equal to the oracle's (sum_e w x) W within fp32 rounding, the gather itself still available."""
    monkeypatch.setattr(executor, "ops", fake_ops)
    rec = [s for s in _streams(manifest) if s["network"] == network and not s["reorder"]][0]
    sem = Semantics.for_network(network, False)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    gc, ip, ix = _cora_graph(golden_dir)
    tensors = workloads.make_tensors(og, gc, network, seed=2)
    ref = execute_ref(og, sem, ip, ix, {k: v.double().numpy() for k, v in tensors.items()})
    nbytes = {}
    for on in (True, False):
        ex = executor.Executor(og, st, gc, tensors, sem)
        ex.mm_first = on
        assert ex.reorder
        ex.run()
        nbytes[on] = ex.alg_bytes
        compare({i: ex.tensor_of(i) for i in range(len(og))}, ref, range(len(og)))
    assert nbytes[True] < nbytes[False]


@pytest.mark.parametrize("reorder", [False, True])
def test_attention_fusion_cpu(golden_dir, manifest, monkeypatch, reorder):
    """GAT's alpha|v * scatter_C(h) -> gather runs as one fused attention aggregate (forced on the
    small graph with attention_blocks); every op, fused-away ones included, matches the oracle."""
    monkeypatch.setattr(executor, "ops", fake_ops)
    sem = Semantics.for_network("GAT", reorder)
    for rec in [s for s in _streams(manifest) if s["network"] == "GAT" and s["reorder"] == reorder][:3]:
        og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
        st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
        gc, ip, ix = _cora_graph(golden_dir)
        tensors = workloads.make_tensors(og, gc, "GAT", seed=4)
        ex = executor.Executor(og, st, gc, tensors, sem)
        ex.attention_blocks = 2
        calls = []
        monkeypatch.setattr(fake_ops, "gat_aggregate_blocked",
                            lambda *a, _real=fake_ops.gat_aggregate_blocked, **k: calls.append(1) or _real(*a, **k))
        ex.run()
        monkeypatch.undo()
        monkeypatch.setattr(executor, "ops", fake_ops)
        F, H = og.ops[3].out_width, og.ops[1].out_width
        assert bool(calls) == fake_ops.BlockedPlan.supports_att(F, H), (rec["file"], F, H)
        ref = execute_ref(og, sem, ip, ix, {k: v.double().numpy() for k, v in tensors.items()})
        compare({i: ex.tensor_of(i) for i in range(len(og))}, ref, range(len(og)))


def test_chrome_trace_cpu(golden_dir, manifest, monkeypatch, tmp_path):
    """trace=True: one complete ("X") event per evaluated op in the reference's Chrome schema
    (vTCAD/code/simulator.py:360-382), names from the stream's COMP instructions, bytes summed."""
    import json
    monkeypatch.setattr(executor, "ops", fake_ops)
    rec = [s for s in _streams(manifest) if s["network"] == "GAT" and not s["reorder"]][0]
    sem = Semantics.for_network("GAT", False)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    gc, ip, ix = _cora_graph(golden_dir)
    res, ex = executor.run_stream(og, st, gc, workloads.make_tensors(og, gc, "GAT"), sem, trace=True)
    ev = ex.trace_events
    assert ev and all(e["ph"] == "X" and e["dur"] >= 0 and {"name", "cat", "ts", "pid", "tid"} <= set(e) for e in ev)
    assert sum(e["args"]["alg_bytes"] for e in ev) == ex.alg_bytes
    assert any(e["name"].startswith("COMP_") for e in ev)
    path = tmp_path / "trace" / "chrome_timeline.json"
    executor.save_chrome_trace(ev, str(path))
    assert json.load(open(path)) == ev
    agg = executor.aggregate_trace(ev)
    assert sum(c for c, _, _ in agg.values()) == len(ev)


@pytest.mark.parametrize("network", ["DGN", "PNA"])
def test_node_mm_and_pushdown_cpu(golden_dir, manifest, monkeypatch, network):
    """Edge GEMMs of scattered node rows run over the nodes ((x W)[r(e)]), and DGN's MM of a sum of
    two scatters is pushed through the sum: fewer algorithmic bytes, every op still matches the oracle."""
    monkeypatch.setattr(executor, "ops", fake_ops)
    rec = [s for s in _streams(manifest) if s["network"] == network and not s["reorder"]][0]
    sem = Semantics.for_network(network, False)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    gc, ip, ix = _cora_graph(golden_dir)
    tensors = workloads.make_tensors(og, gc, network, seed=2)
    ref = execute_ref(og, sem, ip, ix, {k: v.double().numpy() for k, v in tensors.items()})
    nbytes = {}
    for on in (True, False):
        ex = executor.Executor(og, st, gc, tensors, sem)
        ex.node_mm = ex.mm_pushdown = on
        ex.run()
        nbytes[on] = ex.alg_bytes
        compare({i: ex.tensor_of(i) for i in range(len(og))}, ref, range(len(og)))
    assert nbytes[True] < nbytes[False]


def test_gather_acc_fusion_cpu(golden_dir, manifest, monkeypatch):
    """GIN op 4 = ADD(gather, (1+eps) x) runs as the aggregate accumulating into op 3's buffer: every
    op (op 3 and the gather included, recomputed on demand) still matches the oracle, and the ADD's
    [N, F] pass is gone from the algorithmic bytes."""
    monkeypatch.setattr(executor, "ops", fake_ops)
    recs = [s for s in _streams(manifest) if s["network"] == "GIN" and not s["reorder"]]
    assert recs
    for rec in recs:
        sem = Semantics.for_network("GIN", False)
        og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
        st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
        gc, ip, ix = _cora_graph(golden_dir)
        tensors = workloads.make_tensors(og, gc, "GIN", seed=5)
        ref = execute_ref(og, sem, ip, ix, {k: v.double().numpy() for k, v in tensors.items()})
        nbytes = {}
        for on in (True, False):
            ex = executor.Executor(og, st, gc, tensors, sem)
            ex.gather_acc = on
            if on:
                assert ex.gacc, "GIN's ADD(gather, MUL) not matched"
            calls = fake_ops.SELF_TERM_CALLS[0]
            ex.run()
            if on and len(st.blocks) < len(og):  # op 3 = (1 + eps) x formed by the aggregate's epilogue
                assert fake_ops.SELF_TERM_CALLS[0] == calls + 1  # (gta_aggregate_self; a stream of one-op
                # blocks materialises op 1's edge tensor, and the gather then accumulates into op 3)
            nbytes[on] = ex.alg_bytes
            compare({i: ex.tensor_of(i) for i in range(len(og))}, ref, range(len(og)))
        assert nbytes[True] < nbytes[False]


EXPR_SHAPES = {("DGN", False): (3, False, ["ADD", "ADD", "ADD"]), ("DGN", True): (3, False, ["ADD", "ADD", "ADD"]),
               ("PNA", False): (2, True, ["ADD", "ADD"]), ("PNA", True): (2, True, ["ADD", "ADD"])}


@pytest.mark.parametrize("network", ["DGN", "PNA"])
def test_edge_expr_fusion_cpu(golden_dir, manifest, monkeypatch, network):
    """DGN's op 2-7 tree (the MM of op 3 pushed to the node rows) and PNA's ops 5-7 run as one
    expression gather (gta_aggregate_expr): matched with the expected shape, every op of every golden
    stream (the tree's ops recomputed on demand) equal to the fp64 oracle, no [E, F] tensor of the
    tree in the algorithmic bytes, and the GAT / GCN / GIN / SGC / GraphSAGE streams left alone."""
    monkeypatch.setattr(executor, "ops", fake_ops)
    recs = [s for s in _streams(manifest) if s["network"] == network]
    assert recs
    gc, ip, ix = _cora_graph(golden_dir)
    for rec in recs:
        sem = Semantics.for_network(network, rec["reorder"])
        og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
        st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
        tensors = workloads.make_tensors(og, gc, network, seed=6)
        ref = execute_ref(og, sem, ip, ix, {k: v.double().numpy() for k, v in tensors.items()})
        nbytes = {}
        for on in (True, False):
            ex = executor.Executor(og, st, gc, tensors, sem)
            ex.edge_expr = on
            (e,) = ex.expr.values()
            assert (e["shape"], e["swap"], e["bins"]) == EXPR_SHAPES[(network, rec["reorder"])], rec["file"]
            calls = fake_ops.EXPR_CALLS[0]
            ex.run()
            assert fake_ops.EXPR_CALLS[0] == calls + (1 if on else 0), rec["file"]
            nbytes[on] = ex.alg_bytes
            compare({i: ex.tensor_of(i) for i in range(len(og))}, ref, range(len(og)))
        assert nbytes[True] < nbytes[False], rec["file"]
    for s in _streams(manifest):
        if s["network"] in ("DGN", "PNA"):
            continue
        sem = Semantics.for_network(s["network"], s["reorder"])
        og = ir.OpGraph.load(os.path.join(golden_dir, "ops", s["op_yaml"]), sem.inputs)
        st = ir.Stream.load(os.path.join(golden_dir, "streams", s["file"]))
        tensors = workloads.make_tensors(og, gc, s["network"], seed=0)
        assert not executor.Executor(og, st, gc, tensors, sem).expr, s["file"]


def test_two_hop_mm_first_cpu(golden_dir, manifest, monkeypatch):
    """SGC's gather -> scatter C -> MUL -> gather -> MM runs as A (A (x W)): where both weight MULs
    are fused into their gathers, the first gather's [N, F_in] value is never formed (it stays unforced
    through the run), the layer output and every op (recomputed on demand) match the fp64 oracle,
    and fewer algorithmic bytes move than with mm_first off."""
    monkeypatch.setattr(executor, "ops", fake_ops)
    recs = [s for s in _streams(manifest) if s["network"] == "SGC"]
    assert recs
    gc, ip, ix = _cora_graph(golden_dir)
    taken = 0
    for rec in recs:
        sem = Semantics.for_network("SGC", rec["reorder"])
        og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
        st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
        tensors = workloads.make_tensors(og, gc, "SGC", seed=7)
        ref = execute_ref(og, sem, ip, ix, {k: v.double().numpy() for k, v in tensors.items()})
        ex = executor.Executor(og, st, gc, tensors, sem)
        assert ex.two_hop == {2: 5}, rec["file"]
        ex.run()
        fused = all(any(pair <= set(b.ops) for b in st.blocks) for pair in ({1, 2}, {4, 5}))  # both MULs deferred
        first = ex.values[2]
        if fused:
            assert isinstance(first, executor.Lazy) and first.v is None, rec["file"]
            taken += 1
        compare({i: ex.tensor_of(i) for i in range(len(og))}, ref, range(len(og)))
    assert taken >= len(recs) // 2


def test_gin_bf16_model_input_cpu(golden_dir, manifest, monkeypatch):
    """The bf16 GIN configuration (x stored in bf16: BASELINE.md's 200-B rows, bf16 MLP weights):
    every op of the stream, the gather-accumulate fusion included, equals the fp64 oracle run on
    the same bf16 values (the executor widens a bf16 table only where an element-wise edge op
    materialises it)."""
    monkeypatch.setattr(executor, "ops", fake_ops)
    rec = [s for s in _streams(manifest) if s["network"] == "GIN" and not s["reorder"]][0]
    sem = Semantics.for_network("GIN", False)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    gc, ip, ix = _cora_graph(golden_dir)
    tensors = workloads.make_tensors(og, gc, "GIN", seed=6, dtype_w=torch.bfloat16, dtype_x=torch.bfloat16)
    assert tensors["x"].dtype == torch.bfloat16
    ref = execute_ref(og, sem, ip, ix, {k: v.double().numpy() for k, v in tensors.items()})
    ex = executor.Executor(og, st, gc, tensors, sem)
    ex.run()
    compare({i: ex.tensor_of(i) for i in range(len(og))}, ref, range(len(og)))


def test_sibling_weight_concat_is_cached_and_follows_in_place_updates(golden_dir, manifest, monkeypatch):
    """GAT's sibling MMs of x (W and the attention projections) share one [W | W_s] concatenation:
    a second forward reuses the cached tensor (no cat, and so no new W^T), and a sibling weight
    changed in place makes the next forward re-concatenate (results follow the oracle)."""
    monkeypatch.setattr(executor, "ops", fake_ops)
    executor._WCAT.clear()
    rec = [s for s in _streams(manifest) if s["network"] == "GAT" and not s["reorder"]][0]
    sem = Semantics.for_network("GAT", False)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    g, ip, ix = _cora_graph(golden_dir)
    tensors = workloads.make_tensors(og, g, "GAT", seed=5)
    executor.Executor(og, st, g, tensors, sem, plan_chunk=0).run()
    assert len(executor._WCAT) == 1
    (refs, vers, wc), = executor._WCAT.values()
    executor.Executor(og, st, g, tensors, sem, plan_chunk=0).run()
    assert next(iter(executor._WCAT.values()))[2] is wc  # reused, not rebuilt
    sib = refs[-1]()
    sib.mul_(-0.75)  # in place: the version moves, the cached concatenation is stale
    ex = executor.Executor(og, st, g, tensors, sem, plan_chunk=0)
    ex.run()
    wc2 = [e[2] for e in executor._WCAT.values() if e[0][-1]() is sib][0]
    assert wc2 is not wc and torch.equal(wc2[:, -sib.shape[1]:], sib)
    ref = execute_ref(og, sem, ip, ix, {k: v.numpy() for k, v in tensors.items()})
    compare({i: ex.tensor_of(i) for i in range(len(og))}, ref, range(len(og)))


def test_sampled_checker_always_checks_the_special_rows(golden_dir, manifest, monkeypatch):
    """oracle/sampled.py (the full-size config check): the heaviest, lightest, empty, first and
    last rows are checked in every op whatever the random sample, so an error confined to the
    heaviest row of an aggregate is caught even with a tiny random sample."""
    from oracle.sampled import SampledChecker
    rec = [s for s in _streams(manifest) if s["network"] == "GCN" and not s["reorder"]][0]
    monkeypatch.setattr(executor, "ops", fake_ops)
    g, ip, ix = _cora_graph(golden_dir)
    sem = Semantics.for_network("GCN", False)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    ex = executor.Executor(og, st, g, workloads.make_tensors(og, g, "GCN", seed=2), sem, plan_chunk=0)
    ex.run()
    chk = SampledChecker(ex, ip, ix)
    assert chk.check(n_samples=2, seed=0, n_gather=2)
    sp = chk.special
    deg = np.diff(ip)
    assert set(sp) >= {"first", "last", "heaviest", "lightest"}
    assert deg[sp["heaviest"][0]] == deg.max() and sp["last"][0] == len(deg) - 1
    vals = {op.idx: ex.values.get(op.idx) for op in og.ops if op.type == "gather"}
    vals = {i: (v.force() if isinstance(v, executor.Lazy) else v) for i, v in vals.items()}
    gat = [i for i, v in vals.items() if isinstance(v, executor.NodeT)]
    assert gat, "a materialised aggregate to corrupt"
    t = vals[gat[0]].t
    t[int(sp["heaviest"][0])] += 1.0
    with pytest.raises(AssertionError, match="heaviest"):
        chk.check(n_samples=2, seed=0, n_gather=2)


@pytest.mark.parametrize("layer", ["layer2", "layer3"])
def test_mlp_chain_fusion_cpu(golden_dir, manifest, monkeypatch, layer):
    """GIN's MLP (applynode MM -> SF -> MM -> SF, genGraphOP.py:103-108) with bf16 weights and
    widths <= 128 runs as one fused launch (ops.update_mlp); every op of the stream -- the fused-away
    MM and SF values recomputed on demand -- equals the fp64 oracle; with the fusion off, no fused
    launch."""
    monkeypatch.setattr(executor, "ops", fake_ops)
    rec = [s for s in _streams(manifest) if s["network"] == "GIN" and not s["reorder"] and layer in s["file"]][0]
    sem = Semantics.for_network("GIN", False)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    gc, ip, ix = _cora_graph(golden_dir)
    tensors = workloads.make_tensors(og, gc, "GIN", seed=9, dtype_w=torch.bfloat16)
    ref = execute_ref(og, sem, ip, ix, {k: v.double().numpy() for k, v in tensors.items()})
    for fuse in (True, False):
        calls, st_calls, bf_calls = fake_ops.MLP_CALLS[0], fake_ops.SELF_TERM_CALLS[0], fake_ops.BF16_OUT_CALLS[0]
        ex = executor.Executor(og, st, gc, tensors, sem)
        ex.fuse_mlp = fuse
        ex.run()
        assert fake_ops.MLP_CALLS[0] == calls + (1 if fuse else 0)
        # ABI 10: with the fusion, the GIN sum (op 4, formed with its self term) reaches the MLP
        # in bf16 and no fp32 copy of it is made during the run; without it, no bf16 aggregate
        n_self, n_bf = fake_ops.SELF_TERM_CALLS[0] - st_calls, fake_ops.BF16_OUT_CALLS[0] - bf_calls
        assert n_bf == (n_self if fuse else 0) and (not fuse or n_self == 1), (fuse, n_self, n_bf)
        compare({i: ex.tensor_of(i) for i in range(len(og))}, ref, range(len(og)))


def _vtcad_case(golden_dir, manifest, tmp_path):
    """vTCAD/code/test.py:6-14's set-up (GIN, cora, layer3, original order): the op YAML at the
    reference path and the stream interpret() writes for the compiler's best candidate."""
    import shutil
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import lowering
    data_set, network, layer, isReorder = "cora", "GIN", "layer3", False
    path = ir.op_yaml_path(network, data_set, layer, isReorder)
    os.makedirs(os.path.dirname(path))
    shutil.copy(os.path.join(golden_dir, "ops", "GIN-cora-layer3-original.yaml"), path)
    best = manifest["compile"]["GIN-cora-layer3-original"]["top"][0]
    op_array, tile_size_list = best[0], best[1]
    lowering.interpret(data_set, network, isReorder, layer, op_array, tile_size_list)
    return data_set, network, layer, isReorder, tile_size_list, path


def test_vtcad_simulate_call_runs_unchanged(golden_dir, manifest, monkeypatch, tmp_path):
    """vTCAD's eight-argument simulate() line (vTCAD/code/test.py:15, vTCAD/code/simulator.py:423)
    runs against execute() as written once `simulate` is bound to a graph and its tensors; the
    architecture name is checked as vTCAD checks it; outputs match the fp64 oracle."""
    monkeypatch.setattr(executor, "ops", fake_ops)
    monkeypatch.chdir(tmp_path)
    data_set, network, layer, isReorder, tile_size_list, path = _vtcad_case(golden_dir, manifest, tmp_path)
    g, ip, ix = _cora_graph(golden_dir)
    sem = Semantics.for_network(network, isReorder)
    og = ir.OpGraph.load(path, sem.inputs)
    tensors = workloads.make_tensors(og, g, network, seed=0)
    simulate = executor.bind(g, tensors, model="full")
    res = simulate(tile_size_list,data_set,network,layer,isReorder,False,True,'GTA')  # noqa: E231  (verbatim)
    assert res.model_arch == ("GTA", True)
    assert res.model_cycles > 0 and res.model_rw == sum(r["rw_bytes"] for r in res.model_insts)
    ref = execute_ref(og, sem, ip, ix, {k: v.numpy() for k, v in tensors.items()})
    for k, v in res.outputs.items():
        compare({k: v}, ref, [k])
    for arch in ("HyGCN", "GCNAX", "OPU"):
        assert simulate(tile_size_list, data_set, network, layer, isReorder, False, True, arch).model_arch == (arch, False)
    with pytest.raises(ValueError):
        simulate(tile_size_list, data_set, network, layer, isReorder, False, True, "TPU")
    # the six-argument call of code/simulator.py:370 (code/start.py:51) through the same binding
    assert executor.bind(g, tensors)(tile_size_list, data_set, network, layer, isReorder, False).model_rw == res.model_rw


def test_trace_carries_the_per_instruction_model(golden_dir, manifest, monkeypatch, tmp_path):
    """execute(..., trace=...) puts each op's stream instructions, with their modelled bytes and
    busy cycles, on the measured op event; model="full" adds the modelled timeline tracks."""
    monkeypatch.setattr(executor, "ops", fake_ops)
    monkeypatch.chdir(tmp_path)
    data_set, network, layer, isReorder, tile_size_list, path = _vtcad_case(golden_dir, manifest, tmp_path)
    g, _, _ = _cora_graph(golden_dir)
    sem = Semantics.for_network(network, isReorder)
    tensors = workloads.make_tensors(ir.OpGraph.load(path, sem.inputs), g, network, seed=0)
    res = executor.execute(tile_size_list, data_set, network, layer, isReorder, graph=g, tensors=tensors,
                           trace=str(tmp_path / "trace.json"))
    measured = [e for e in res.trace if e["pid"] == "MI355X"]
    assert measured and all(e["args"]["model"] for e in measured)
    assert sum(m["bytes"] for e in measured for m in e["args"]["model"]) > 0
    assert sum(r["rw_bytes"] for r in res.model_insts) == res.model_rw
    full = executor.execute(tile_size_list, data_set, network, layer, isReorder, graph=g, tensors=tensors,
                            model="full", trace=True)
    model_ev = [e for e in full.trace if e["pid"] == "GTA model"]
    assert len(model_ev) == sum(1 for r in full.model_insts if r["starts"] > 0)
    assert max(e["ts"] + e["dur"] for e in model_ev) * 1e3 <= full.model_cycles + 1


def test_graph_pool_eviction_is_lru_and_never_recaptures(monkeypatch):
    """past AUTO_GRAPH_MAX_POOL_BYTES the least recently used captured graphs are dropped
    (not the largest other one), and a dropped entry stays eager instead of being recaptured two
    calls later (two big alternating layers used to evict each other on every capture)."""
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import executor as X
    monkeypatch.setattr(X, "_AUTO", {})
    monkeypatch.setattr(X, "AUTO_GRAPH_MAX_POOL_BYTES", 100)
    ents = []
    for k, (b, use) in enumerate([(60, 3), (50, 1), (30, 2)]):
        e = X._AutoEntry((), {})
        e.run, e.pool_bytes, e.last_use, e.calls = object(), b, use, 2
        X._AUTO[k] = e
        ents.append(e)
    X._evict_pools(keep=ents[2])  # 140 > 100: drop the LRU entry other than the new one (not the largest)
    assert ents[1].run is None and ents[1].evicted and 1 in X._AUTO
    assert ents[0].run is not None and ents[2].run is not None  # 90 <= 100: done
    X._AUTO[3] = e = X._AutoEntry((), {})
    e.run, e.pool_bytes, e.last_use = object(), 40, 4
    X._evict_pools(keep=e)  # 130: the least recently used live graph now is entry 2
    assert ents[2].evicted and ents[0].run is not None and e.run is not None
