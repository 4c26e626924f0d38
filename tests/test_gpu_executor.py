"""Executor on the real libgta kernels vs the fp64 op-by-op oracle, for every golden stream.

Tolerance: per op, max |got - ref| / max |ref| <= 2e-4 (fp32 kernels through
chains of up to 14 ops incl. exp / division / MFMA GEMMs vs fp64), and the
non-finite pattern (0/0 at isolated nodes in GAT-trans op 11) must match.
"""
import os

import numpy as np
import pytest
import torch

from gta_graph_tensor_acclelrator_for_general_gnn_amd import executor, graph as G, ir, ops, workloads
from gta_graph_tensor_acclelrator_for_general_gnn_amd.semantics import Semantics
from oracle import isa_ref
from oracle.exec_ref import execute_ref
from oracle.sampled import SampledChecker

from .conftest import load_manifest
from .test_ir_executor_cpu import compare

pytestmark = pytest.mark.gpu


def _all_streams(manifest):
    return [s for s in manifest["streams"] if "file" in s]


@pytest.fixture(scope="module")
def cora(golden_dir):
    z = np.load(os.path.join(golden_dir, "cora_graph.npz"))
    return z["indptr"], z["indices"]


def _run(golden_dir, rec, ip, ix, dev, seed, plan_chunk):
    sem = Semantics.for_network(rec["network"], rec["reorder"])
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    gd = G.from_numpy(ip, ix, device=dev)
    gc = G.from_numpy(ip, ix)
    tensors_c = workloads.make_tensors(og, gc, rec["network"], seed=seed)
    tensors = {k: v.to(dev) for k, v in tensors_c.items()}
    res, ex = executor.run_stream(og, st, gd, tensors, sem, plan_chunk=plan_chunk)
    ref = execute_ref(og, sem, ip, ix, {k: v.double().numpy() for k, v in tensors_c.items()})
    vals = {i: ex.tensor_of(i) for i in range(len(og))}
    compare(vals, ref, range(len(og)), rtol=2e-4)  # end to end, through the whole op chain
    # op-local and per element, at every row and edge: |d| <= 1e-5 sum|terms| + 1e-6 (oracle/sampled.py)
    chk = SampledChecker(ex, ip, ix)
    chk.check(n_samples=1 << 30, n_gather=1 << 30)
    print(rec["file"], {k: round(v[2], 4) for k, v in chk.detail.items()})  # max err / bound per op
    return res


STREAMS = _all_streams(load_manifest())


@pytest.mark.parametrize("idx", range(len(STREAMS)), ids=[r["file"][:-5] for r in STREAMS])
def test_executor_golden_stream_on_gpu(golden_dir, manifest, cora, dev, idx):
    rec = STREAMS[idx]
    ip, ix = cora
    res = _run(golden_dir, rec, ip, ix, dev, seed=idx, plan_chunk=64 if idx % 2 else 512)
    assert res.launches > 0 and res.alg_bytes > 0


def test_executor_drop_in_signature(golden_dir, manifest, cora, dev, tmp_path, monkeypatch):
    """execute(tile_size_list, dataset, network, layer, isReorder, isSinput, ...) reads the same
    Results/Insts and Network/ paths as simulate()/interpret() (code/simulator.py:398, interpreter.py:821)."""
    rec = [s for s in manifest["streams"] if s.get("file") == "GCN-cora-layer1-original-c0.yaml"][0]
    monkeypatch.chdir(tmp_path)
    os.makedirs("Results/Insts")
    os.makedirs("Network/GCN/GCN-cora/GCN-original")
    import shutil
    shutil.copy(os.path.join(golden_dir, "streams", rec["file"]), "Results/Insts/GCN-cora-layer1-original.yaml")
    shutil.copy(os.path.join(golden_dir, "ops", rec["op_yaml"]), "Network/GCN/GCN-cora/GCN-original/GCN-layer1-original.yaml")
    ip, ix = cora
    gd = G.from_numpy(ip, ix, device=dev)
    og = ir.OpGraph.load("Network/GCN/GCN-cora/GCN-original/GCN-layer1-original.yaml")
    tensors = workloads.make_tensors(og, gd, "GCN", seed=0)
    res = executor.execute(rec["tile_size_list"], "cora", "GCN", "layer1", False, False, graph=gd, tensors=tensors)
    out = res.outputs[3]
    assert out.shape == (2708, 128) and torch.isfinite(out).all()


def test_execute_reports_reference_simulate_numbers(golden_dir, manifest, cora, dev, tmp_path, monkeypatch):
    """Same call, same stream, same graph: model (cycles, rw) == the reference simulate() output."""
    import shutil
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import lowering
    ip, ix = cora
    gd = G.from_numpy(ip, ix, device=dev)
    monkeypatch.chdir(tmp_path)
    for case in manifest["simulate"]:
        net, ds, layer, m = case["key"].split("-")
        os.makedirs(f"Network/{net}/{net}-{ds}/{net}-{m}", exist_ok=True)
        shutil.copy(os.path.join(golden_dir, "ops", f"{net}-{ds}-{layer}-{m}.yaml"),
                    f"Network/{net}/{net}-{ds}/{net}-{m}/{net}-{layer}-{m}.yaml")
        lowering.interpret(ds, net, m == "trans", layer, case["op_array"], case["tile_size_list"])
        og = ir.OpGraph.load(f"Network/{net}/{net}-{ds}/{net}-{m}/{net}-{layer}-{m}.yaml")
        tensors = workloads.make_tensors(og, gd, net, seed=1)
        res = executor.execute(case["tile_size_list"], ds, net, layer, m == "trans", False, graph=gd,
                               tensors=tensors, model="full")
        assert res.simulate_tuple() == (case["cycles"], case["rw"]), case["key"]


def test_executor_deterministic(golden_dir, manifest, cora, dev):
    rec = [s for s in manifest["streams"] if s.get("file") == "GAT-reddit-layer1-original-h512.yaml"][0]
    ip, ix = cora
    sem = Semantics.for_network("GAT", False)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    gd = G.from_numpy(ip, ix, device=dev)
    tensors = workloads.make_tensors(og, gd, "GAT", seed=3)
    a, _ = executor.run_stream(og, st, gd, tensors, sem)
    b, _ = executor.run_stream(og, st, gd, tensors, sem)
    for k in a.outputs:
        assert torch.equal(a.outputs[k], b.outputs[k])


@pytest.mark.parametrize("reorder", [False, True])
def test_gat_softmax_fusion_on_gpu(golden_dir, manifest, cora, dev, reorder):
    """GAT ops 6-10 run as one gta_edge_softmax launch: fewer launches, same values (fp32 rounding)
    as the unfused op-by-op path, and both match the fp64 oracle."""
    rec = [s for s in _all_streams(manifest) if s["network"] == "GAT" and s["reorder"] == reorder][0]
    ip, ix = cora
    sem = Semantics.for_network("GAT", reorder)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    gd = G.from_numpy(ip, ix, device=dev)
    tensors = {k: v.to(dev) for k, v in workloads.make_tensors(og, G.from_numpy(ip, ix), "GAT", seed=5).items()}
    outs = {}
    for fuse in (True, False):
        ex = executor.Executor(og, st, gd, tensors, sem)
        ex.fuse_softmax = fuse
        assert bool(ex.softmax) is True
        outs[fuse] = ({k: v.clone() for k, v in ex.run().items()}, ex.launches)
    (fo, fl), (uo, ul) = outs[True], outs[False]
    assert fl < ul, (fl, ul)
    for k in uo:
        a, b = fo[k].double().cpu(), uo[k].double().cpu()
        fin = torch.isfinite(b)
        assert torch.equal(torch.isfinite(a), fin)
        assert (a[fin] - b[fin]).abs().max() <= 1e-4 * b[fin].abs().max() + 1e-6


@pytest.mark.parametrize("k", [0, 1, 4, 5, 6])
def test_legacy_v2_stream_on_gpu(golden_dir, dev, k):
    """BASELINE config 0's stream (V2 create_list lowering) executed on libgta vs the fp64 oracle."""
    import json
    from .test_legacy_v2 import run_v2
    case = json.load(open(os.path.join(golden_dir, "v2", "manifest.json")))[k]
    res = run_v2(golden_dir, case, dev=dev)
    assert res.launches > 0


@pytest.mark.parametrize("reorder", [False, True])
def test_gat_attention_fusion_on_gpu(golden_dir, manifest, cora, dev, reorder, monkeypatch):
    """alpha|v * scatter_C(h) -> gather as one gta_gat_aggregate_blocked launch (forced on Cora with
    attention_blocks): every op, fused-away ones included, matches the fp64 oracle."""
    sem = Semantics.for_network("GAT", reorder)
    ip, ix = cora
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops
    calls = []
    monkeypatch.setattr(ops, "gat_aggregate_blocked",
                        lambda *a, _real=ops.gat_aggregate_blocked, **k: calls.append(1) or _real(*a, **k))
    for rec in [s for s in _all_streams(manifest) if s["network"] == "GAT" and s["reorder"] == reorder
                and s["dataset"] == "cora"][:4]:
        og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
        st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
        gd = G.from_numpy(ip, ix, device=dev)
        tc = workloads.make_tensors(og, G.from_numpy(ip, ix), "GAT", seed=6)
        ex = executor.Executor(og, st, gd, {k: v.to(dev) for k, v in tc.items()}, sem)
        ex.attention_blocks = 3
        ex.run()
        ref = execute_ref(og, sem, ip, ix, {k: v.double().numpy() for k, v in tc.items()})
        compare({i: ex.tensor_of(i) for i in range(len(og))}, ref, range(len(og)), rtol=2e-4)
    assert calls


def test_execute_chrome_trace_on_gpu(golden_dir, manifest, cora, dev, tmp_path, monkeypatch):
    """execute(..., trace=path) writes the measured per-op timeline (HIP events) as Chrome JSON."""
    import json
    import shutil
    rec = [s for s in manifest["streams"] if s.get("file") == "GCN-cora-layer1-original-c0.yaml"][0]
    monkeypatch.chdir(tmp_path)
    os.makedirs("Results/Insts")
    os.makedirs("Network/GCN/GCN-cora/GCN-original")
    shutil.copy(os.path.join(golden_dir, "streams", rec["file"]), "Results/Insts/GCN-cora-layer1-original.yaml")
    shutil.copy(os.path.join(golden_dir, "ops", rec["op_yaml"]), "Network/GCN/GCN-cora/GCN-original/GCN-layer1-original.yaml")
    ip, ix = cora
    gd = G.from_numpy(ip, ix, device=dev)
    og = ir.OpGraph.load("Network/GCN/GCN-cora/GCN-original/GCN-layer1-original.yaml")
    tensors = workloads.make_tensors(og, gd, "GCN", seed=0)
    res = executor.execute(rec["tile_size_list"], "cora", "GCN", "layer1", False, False, graph=gd, tensors=tensors,
                           trace="trace/chrome_timeline.json")
    ev = json.load(open("trace/chrome_timeline.json"))
    assert ev == res.trace and len(ev) >= 1
    assert all(e["ph"] == "X" and e["dur"] >= 0 for e in ev) and sum(e["dur"] for e in ev) > 0


def test_gcn_cora_2layer_fused_template_on_gpu(golden_dir, cora, dev):
    """BASELINE config 2 through the fused_template (V2 create_list) lowering, both layers chained on
    libgta, vs the fp64 oracle."""
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import frontend, legacy
    ip, ix = cora
    gd, gc = G.from_numpy(ip, ix, device=dev), G.from_numpy(ip, ix)
    x_c = None
    for layer, fin in ((1, 1433), (2, 128)):
        ops_ = frontend.gen_ops("GCN", layer, 2708, 10556, 1433, False, 16)
        recs = legacy.lower_v2("cora", ops_, [[o["OP_NO"]] for o in ops_], [64] * len(ops_), 2708)
        og = ir.OpGraph(legacy.typed_records(ops_))
        tc = workloads.make_tensors(og, gc, "GCN", seed=layer)
        if x_c is not None:
            tc["x"] = x_c
        res, ex = legacy.execute_v2(ops_, recs, gd, {k: v.to(dev) for k, v in tc.items()}, "GCN")
        ref = execute_ref(og, Semantics.for_network("GCN"), ip, ix, {k: v.double().numpy() for k, v in tc.items()})
        compare({i: ex.tensor_of(i) for i in range(len(og))}, ref, range(len(og)), rtol=2e-4)
        x_c = res.outputs[sorted(res.outputs)[-1]].cpu()


@pytest.mark.parametrize("network,reorder", [("GCN", False), ("GAT", False), ("GAT", True), ("GraphSAGE", False),
                                             ("GIN", False)])
def test_graphed_run_replays_the_stream(golden_dir, manifest, cora, dev, network, reorder):
    """The stream captured as one HIP graph: a replay equals a fresh execution bitwise, and follows
    in-place updates of the inputs."""
    rec = [s for s in _all_streams(manifest) if s["network"] == network and s["reorder"] == reorder
           and s["dataset"] == "cora"][0]
    sem = Semantics.for_network(network, reorder)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    ip, ix = cora
    gd = G.from_numpy(ip, ix, device=dev)
    tensors = {k: v.to(dev) for k, v in workloads.make_tensors(og, G.from_numpy(ip, ix), network, seed=2).items()}
    gr = executor.GraphedRun(og, st, gd, tensors, sem)
    for trial in range(2):
        if trial:
            tensors["x"].mul_(0.5).add_(0.25)  # new input values, same storage
        out = {k: v.clone() for k, v in gr.replay().items()}
        ref = executor.Executor(og, st, gd, tensors, sem).run()
        for k in ref:
            a, b = out[k], ref[k]
            assert torch.equal(torch.isfinite(a), torch.isfinite(b))
            assert torch.equal(a[torch.isfinite(a)], b[torch.isfinite(b)]), (network, k, trial)


@pytest.mark.parametrize("plan_chunk", [0, 64])
def test_gather_acc_fusion_bitwise_on_gpu(golden_dir, manifest, cora, dev, plan_chunk):
    """GIN's ADD(gather, (1+eps) x) as the aggregate accumulating into op 3's buffer gives every
    op's value bitwise equal to the unfused run (T + sum == sum + T in fp32)."""
    ip, ix = cora
    recs = [s for s in _all_streams(manifest) if s["network"] == "GIN" and not s["reorder"]]
    assert recs
    gd = G.from_numpy(ip, ix, device=dev)
    for rec in recs:
        sem = Semantics.for_network("GIN", False)
        og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
        st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
        tensors = workloads.make_tensors(og, gd, "GIN", seed=4)
        vals = {}
        for on in (True, False):
            ex = executor.Executor(og, st, gd, tensors, sem, plan_chunk=plan_chunk)
            ex.gather_acc = on
            assert bool(ex.gacc)
            ex.run()
            vals[on] = [ex.tensor_of(i) for i in range(len(og))]
        for i, (a, b) in enumerate(zip(vals[True], vals[False])):
            assert torch.equal(a, b), f"{rec['file']} op {i}"


def test_repeated_execute_replays_a_hip_graph(golden_dir, manifest, cora, dev, tmp_path, monkeypatch):
    """execute() called again with the same graph and input tensors replays one captured HIP graph
    (executor.AUTO_GRAPH): results equal the eager first call bitwise, follow in-place input
    updates, and a new input tensor object means a new eager run."""
    import shutil
    rec = [s for s in manifest["streams"] if s.get("file") == "GCN-cora-layer1-original-c0.yaml"][0]
    monkeypatch.chdir(tmp_path)
    os.makedirs("Results/Insts")
    os.makedirs("Network/GCN/GCN-cora/GCN-original")
    shutil.copy(os.path.join(golden_dir, "streams", rec["file"]), "Results/Insts/GCN-cora-layer1-original.yaml")
    shutil.copy(os.path.join(golden_dir, "ops", rec["op_yaml"]), "Network/GCN/GCN-cora/GCN-original/GCN-layer1-original.yaml")
    ip, ix = cora
    gd = G.from_numpy(ip, ix, device=dev)
    og = ir.OpGraph.load("Network/GCN/GCN-cora/GCN-original/GCN-layer1-original.yaml")
    tensors = workloads.make_tensors(og, gd, "GCN", seed=0)
    run = lambda: executor.execute(rec["tile_size_list"], "cora", "GCN", "layer1", False, False,  # noqa: E731
                                   graph=gd, tensors=tensors)
    first = {k: v.clone() for k, v in run().outputs.items()}
    n_before = sum(e.run is not None for e in executor._AUTO.values())
    second = run()
    third = run()
    assert sum(e.run is not None for e in executor._AUTO.values()) == n_before + 1
    assert second.outputs.keys() == first.keys() and second.model_rw == third.model_rw is not None
    for k in first:
        assert torch.equal(second.outputs[k], first[k]) and torch.equal(third.outputs[k], first[k])
    tensors["x"].mul_(0.5)  # same storage, new values: the replay reads them
    fresh = executor.Executor(og, ir.Stream(ir.read_yaml("Results/Insts/GCN-cora-layer1-original.yaml")), gd,
                              tensors, Semantics.for_network("GCN", False)).run()
    again = run()
    for k in fresh:
        assert torch.equal(again.outputs[k], fresh[k])
    # a weight changed in place (load_state_dict / optimizer step): the replay re-transposes it into
    # the graph's W^T instead of reading the stale one
    wkey = sorted(k for k in tensors if k.startswith("w:"))[0]
    tensors[wkey].mul_(-1.5)
    fresh = executor.Executor(og, ir.Stream(ir.read_yaml("Results/Insts/GCN-cora-layer1-original.yaml")), gd,
                              tensors, Semantics.for_network("GCN", False)).run()
    again = run()
    for k in fresh:
        assert torch.equal(again.outputs[k], fresh[k])
    # a knob change is part of the cache key: the next call runs eagerly under the new knobs
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops
    try:
        ops.set_debug("mm_ring", 0)
        ks = ops.knob_state()
        assert ks == (("mm_ring", 0),)
        later = run()
        assert any(k[5] == ks for k in executor._AUTO)  # a new entry under the new knob state
    finally:
        ops.set_debug("mm_ring", 1)
    assert ops.knob_state() == ()  # restored: the earlier entries' key again
    for k in fresh:
        assert torch.equal(later.outputs[k], fresh[k])  # k_mm_rows == k_mm_ring bitwise
    executor.set_auto_graph(False)
    try:
        assert not executor._AUTO
        for k, v in run().outputs.items():
            assert torch.equal(v, fresh[k])
    finally:
        executor.set_auto_graph(True)


def test_graphed_run_follows_weights_changed_in_place(golden_dir, manifest, cora, dev):
    """GraphedRun keeps the W^T tensors its launches read and refreshes them when a weight's
    version moves (in-place update), so replays never read a stale or freed transpose."""
    rec = [s for s in _all_streams(manifest) if s["network"] == "GraphSAGE" and not s["reorder"]
           and s["dataset"] == "cora"][0]
    sem = Semantics.for_network("GraphSAGE", False)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    ip, ix = cora
    gd = G.from_numpy(ip, ix, device=dev)
    tensors = {k: v.to(dev) for k, v in workloads.make_tensors(og, G.from_numpy(ip, ix), "GraphSAGE", seed=3).items()}
    gr = executor.GraphedRun(og, st, gd, tensors, sem)
    assert gr._wts, "the captured graph reads at least one cached W^T"
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import ops
    ops._WT_CACHE.clear()  # the cache may drop its entries: the graph still holds its own
    for trial in range(3):
        for k in tensors:
            if k.startswith("w:"):
                tensors[k].add_(0.125 * (trial + 1))
        out = {k: v.clone() for k, v in gr.replay().items()}
        ref = executor.Executor(og, st, gd, tensors, sem).run()
        for k in ref:
            assert torch.equal(out[k], ref[k]), (k, trial)


def test_graphed_run_follows_sibling_weights_changed_in_place(golden_dir, manifest, cora, dev):
    """GAT's sibling MMs read one cached [W | W_s] concatenation (and its cached W^T) inside the
    captured graph; a sibling weight changed in place between replays is re-concatenated and
    re-transposed before the next replay, which then equals a fresh eager run bitwise."""
    rec = [s for s in _all_streams(manifest) if s["network"] == "GAT" and not s["reorder"]
           and s["dataset"] == "cora"][0]
    sem = Semantics.for_network("GAT", False)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    ip, ix = cora
    gd = G.from_numpy(ip, ix, device=dev)
    tensors = {k: v.to(dev) for k, v in workloads.make_tensors(og, G.from_numpy(ip, ix), "GAT", seed=4).items()}
    gr = executor.GraphedRun(og, st, gd, tensors, sem)
    assert gr._wcats, "the captured graph reads a cached sibling concatenation"
    srcs, wc, _ = gr._wcats[0]
    assert any(wt is not None for w, wt, _ in gr._wts if w is wc), "and its cached W^T"
    first = {k: v.clone() for k, v in gr.replay().items()}
    ref = executor.Executor(og, st, gd, tensors, sem).run()
    for k in ref:
        assert torch.equal(first[k], ref[k]), k
    for trial, w in enumerate([srcs[-1], srcs[0], srcs[-1]]):  # a sibling, the main weight, a sibling
        w.mul_(-0.5 - 0.25 * trial)
        out = {k: v.clone() for k, v in gr.replay().items()}
        ref = executor.Executor(og, st, gd, tensors, sem).run()
        for k in ref:
            assert torch.equal(out[k], ref[k]), (k, trial)
        assert not all(torch.equal(out[k], first[k]) for k in ref), trial


def test_gin_bf16_model_input_on_gpu(golden_dir, manifest, cora, dev):
    """GIN with the bf16 model input (the gin-products configuration's storage) on the real kernels:
    the bf16-row aggregate accumulating into (1+eps) x (bf16 apply_node), the bf16 MFMA MLP;
    every op vs the fp64 oracle on the same bf16 values."""
    rec = [s for s in _all_streams(manifest) if s["network"] == "GIN" and not s["reorder"] and s["dataset"] == "cora"][0]
    sem = Semantics.for_network("GIN", False)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    ip, ix = cora
    gd = G.from_numpy(ip, ix, device=dev)
    tc = workloads.make_tensors(og, G.from_numpy(ip, ix), "GIN", seed=7, dtype_w=torch.bfloat16, dtype_x=torch.bfloat16)
    res, ex = executor.run_stream(og, st, gd, {k: v.to(dev) for k, v in tc.items()}, sem)
    # op-local fp64 checks (the bf16 GEMMs' inputs rounded to bf16 in the reference too)
    from oracle.sampled import SampledChecker
    assert SampledChecker(ex, ip, ix).check(n_samples=400, seed=3)


@pytest.mark.parametrize("layer", ["layer2", "layer3"])
@pytest.mark.parametrize("dtype_x", [torch.float32, torch.bfloat16])
def test_gin_sum_reaches_fused_mlp_in_bf16(golden_dir, manifest, cora, dev, monkeypatch, layer, dtype_x):
    """ABI 10: GIN's sum (1 + eps) x + aggregate, formed in one launch, is stored in bf16 when its only
    reader is the fused MLP; the layer output is bitwise the unfused run's (the MLP's first GEMM
    rounds an fp32 x to bf16 on load either way), and the sum itself, read afterwards, is the fp32
    value (recomputed)."""
    rec = [s for s in _all_streams(manifest) if s["network"] == "GIN" and not s["reorder"] and s["dataset"] == "cora"
           and layer in s["file"]][0]
    sem = Semantics.for_network("GIN", False)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    ip, ix = cora
    gd = G.from_numpy(ip, ix, device=dev)
    tc = workloads.make_tensors(og, G.from_numpy(ip, ix), "GIN", seed=11, dtype_w=torch.bfloat16, dtype_x=dtype_x)
    tensors = {k: v.to(dev) for k, v in tc.items()}
    seen = []
    real = executor.ops.aggregate

    def spy(*a, **k):
        y = real(*a, **k)
        seen.append(y.dtype)
        return y

    monkeypatch.setattr(executor.ops, "aggregate", spy)
    outs = {}
    for fuse in (True, False):
        seen.clear()
        ex = executor.Executor(og, st, gd, tensors, sem)
        ex.fuse_mlp = fuse
        outs[fuse] = {k: v.clone() for k, v in ex.run().items()}
        assert (torch.bfloat16 in seen) == fuse, seen
        sums = {i: ex.tensor_of(i) for i in ex.gacc}
        assert all(t.dtype == torch.float32 for t in sums.values())
        if fuse:
            fused_sums = sums
        else:
            for i, t in sums.items():
                assert torch.equal(t, fused_sums[i]), i
    for k in outs[False]:
        assert torch.equal(outs[True][k], outs[False][k]), k


def test_bf16_source_table_takes_the_row_chunked_aggregate(golden_dir, manifest, cora, dev):
    """a bf16 source table of a width the blocked kernels take (F = 128), above the
    blocked-form size gate, runs the bf16 row-chunked aggregate (the blocked kernels are fp32-only),
    and the gate sizes the table with its own element size.  Result vs the fp64 oracle."""
    rec = [s for s in _all_streams(manifest) if s["network"] == "GIN" and not s["reorder"] and s["dataset"] == "cora"][0]
    sem = Semantics.for_network("GIN", False)
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    ip, ix = cora
    gd = G.from_numpy(ip, ix, device=dev)
    tc = workloads.make_tensors(og, G.from_numpy(ip, ix), "GIN", seed=7)
    ex = executor.Executor(og, st, gd, {k: v.to(dev) for k, v in tc.items()}, sem)
    ex.blocked_min_table_bytes, ex.blocked_blocks = 0, 4
    x = torch.randn(gd.n_cols, 128, device=dev).to(torch.bfloat16)
    assert ex._blocked_blocks(x, "src", 0) == 0
    assert ex._blocked_blocks(x.float(), "src", 0) == 4
    ex.blocked_min_table_bytes = x.numel() * 2 + 1  # the bf16 table's own bytes decide, not 4 B/element
    assert ex._blocked_blocks(x.float(), "src", 0) == 4
    w = torch.rand(gd.nnz, 1, device=dev)
    for wt in (None, w):
        y = ex._spmm(x, "src", wt)
        xr = x.float().cpu().numpy().astype(np.float64)
        wr = None if wt is None else wt.cpu().numpy().astype(np.float64)
        ref = isa_ref.aggregate(ip, ix, xr, "src", wr)
        bound = 1e-5 * isa_ref.aggregate_abs(ip, ix, xr, "src", wr) + 1e-6
        assert np.all(np.abs(y.cpu().numpy() - ref) <= bound)


BIDIR_STREAMS = [s for s in STREAMS if s["network"] == "BIDIR"][:2]


@pytest.mark.parametrize("rec", BIDIR_STREAMS, ids=[r["file"][:-5] for r in BIDIR_STREAMS])
def test_gather_c_column_blocked_on_gpu(golden_dir, cora, dev, rec):
    """ORDER-C gather of a scatter-R operand (the transposed aggregate, BIDIR op 3) takes the
    column-blocked kernels over the CSC "dst" view when its table is large, as direction R does
    (forced on Cora: size gate 0, B = 4); every op per element within the bound at every row."""
    sem = Semantics.for_network(rec["network"], rec["reorder"])
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden_dir, "streams", rec["file"]))
    ip, ix = cora
    gd = G.from_numpy(ip, ix, device=dev)
    tc = workloads.make_tensors(og, G.from_numpy(ip, ix), rec["network"], seed=3)
    ex = executor.Executor(og, st, gd, {k: v.to(dev) for k, v in tc.items()}, sem)
    ex.blocked_min_table_bytes, ex.blocked_blocks = 0, 4
    ex.run()
    torch.cuda.synchronize()
    view = ops.csc(gd).view("dst")
    assert any(isinstance(k, tuple) and k[0] == "blocked" for k in view._plans)
    chk = SampledChecker(ex, ip, ix)
    chk.check(n_samples=1 << 30, n_gather=1 << 30)


@pytest.mark.parametrize("H", [0, 1, 8])
def test_transposed_spmm_column_blocked(cora, dev, H):
    """The executor's SpMM over the CSC "dst" view (y[j] = sum over the edges whose source is j of
    w(e) x[dst(e)]): column-blocked (B = 4) and row-chunked forms, unweighted, one weight per edge
    and 8 heads, against the fp64 restatement at the per-element bound."""
    ip, ix = cora
    gd = G.from_numpy(ip, ix, device=dev)
    rec = [s for s in STREAMS if s["network"] == "BIDIR"][0]
    sem = Semantics.for_network("BIDIR", False)
    golden = os.path.join(os.path.dirname(__file__), "golden")
    og = ir.OpGraph.load(os.path.join(golden, "ops", rec["op_yaml"]), sem.inputs)
    st = ir.Stream.load(os.path.join(golden, "streams", rec["file"]))
    tc = workloads.make_tensors(og, G.from_numpy(ip, ix), "BIDIR", seed=1)
    ex = executor.Executor(og, st, gd, {k: v.to(dev) for k, v in tc.items()}, sem)
    view = ops.csc(gd).view("dst")
    rng = np.random.default_rng(H)
    n, E = len(ip) - 1, len(ix)
    x = rng.standard_normal((n, 128)).astype(np.float32)
    w = (rng.random((E, H)) + 0.5).astype(np.float32) if H else None
    dst = np.repeat(np.arange(n), np.diff(ip))
    perm = np.argsort(ix, kind="stable")  # CSC order: a column's edges in CSR order
    xe = x[dst].astype(np.float64)
    if H:
        xe = xe * np.repeat(w.astype(np.float64), 128 // H, axis=1)
    ref = np.zeros((n, 128))
    mag = np.zeros((n, 128))
    np.add.at(ref, ix, xe)
    np.add.at(mag, ix, np.abs(xe))
    wc = None if w is None else torch.from_numpy(w[perm]).to(dev)
    xd = torch.from_numpy(x).to(dev)
    for blocked in (4, 0):
        ex.blocked_min_table_bytes, ex.blocked_blocks = 0, blocked
        y = ex._spmm(xd, "src", wc, graph=view)
        torch.cuda.synchronize()
        err = np.abs(y.cpu().numpy() - ref)
        assert (err <= 1e-5 * mag + 1e-6).all(), (blocked, float(err.max()))
