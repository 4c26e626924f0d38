"""Line-pitched node tables (ops.line_pitch / node_table / pitched): the row pitch the aggregates'
gathered tables are stored with (CPU: pure layout arithmetic, no kernel)."""
import os

import torch

from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G, ir, ops, workloads
from gta_graph_tensor_acclelrator_for_general_gnn_amd.semantics import Semantics


def _lines_brute(row_bytes, pitch_bytes, rows=4096):
    return sum((r * pitch_bytes + row_bytes - 1) // 128 - (r * pitch_bytes) // 128 + 1 for r in range(rows)) / rows


def test_lines_per_row_matches_a_brute_count():
    for row, pitch in [(200, 200), (200, 208), (200, 256), (400, 400), (2408, 2408), (2408, 2432), (64, 64), (72, 72)]:
        assert abs(ops._lines_per_row(row, pitch) - _lines_brute(row, pitch)) < 1e-9, (row, pitch)


def test_pitch_choices():
    # GIN products' bf16 rows: 200 B touch 2.5 lines, 256 B exactly 2
    assert ops._lines_per_row(200, 200) == 2.5 and ops._lines_per_row(200, 256) == 2.0
    assert ops.line_pitch(100, 2) == 128
    assert ops.line_pitch(128, 4) == 128       # whole lines already (the metric's rows)
    assert ops.line_pitch(100, 4) == 100       # 400-B rows touch 4 lines at either pitch: no padding
    assert ops.line_pitch(602, 4) == 608       # Reddit's model input: 19.75 -> 19 lines, +1 %
    assert ops.line_pitch(500, 4) == 512
    assert ops.line_pitch(16, 4) == 16         # a 64-B row never straddles at its own pitch
    assert ops.line_pitch(36, 2) == 36         # padding 72 B to 128 would cost more than max_extra
    assert ops.line_pitch(0, 4) == 0


def test_node_table_and_pitched():
    x = torch.randn(7, 100).to(torch.bfloat16)
    p = ops.pitched(x)
    assert p.shape == x.shape and p.stride() == (128, 1) and torch.equal(p, x)
    base = p.as_strided((7, 128), (128, 1))
    assert torch.count_nonzero(base[:, 100:]) == 0  # zero padding
    assert ops.pitched(p) is p and ops.pitched(p[2:5]).data_ptr() == p[2:5].data_ptr()  # already pitched: no copy
    q = ops.pitched(torch.randn(5, 128))
    assert q.is_contiguous()
    flat = torch.randn(6, 100).to(torch.bfloat16)
    assert ops.pitched(flat).stride(0) == 128 and ops.pitched(flat).data_ptr() != flat.data_ptr()
    t = ops.node_table(3, 602, torch.float32)
    assert t.shape == (3, 602) and t.stride(0) == 608


def test_make_tensors_builds_a_pitched_model_input(golden_dir, manifest):
    rec = [s for s in manifest["streams"] if s.get("network") == "GIN" and "op_yaml" in s and not s["reorder"]][0]
    og = ir.OpGraph.load(os.path.join(golden_dir, "ops", rec["op_yaml"]), Semantics.for_network("GIN", False).inputs)
    g = G.synthetic(300, 2000, seed=1)
    t = workloads.make_tensors(og, g, "GIN", dtype_x=torch.bfloat16, dtype_w=torch.bfloat16)
    F = t["x"].shape[1]
    assert t["x"].shape[0] == 300 and t["x"].stride(0) == ops.line_pitch(F, 2)
    # the self operand aliases the same storage
    assert any(v is t["x"] for k, v in t.items() if k.startswith("ext:"))
