"""frontend.gen_ops reproduces the reference genGraphOP YAML byte-for-byte (tests/golden/ops)."""
import os

import pytest

from gta_graph_tensor_acclelrator_for_general_gnn_amd import frontend


def test_every_golden_op_yaml(golden_dir, manifest):
    assert len(manifest["ops"]) >= 50
    for rec in manifest["ops"]:
        if rec.get("r5"):  # the hand-written ORDER-C op graphs of make_golden_r5.py: not genGraphOP output
            continue
        text = frontend.dumps(frontend.gen_ops(rec["network"], rec["layer"], rec["N"], rec["E"], rec["F"],
                                               rec["reorder"]))
        with open(os.path.join(golden_dir, "ops", rec["file"])) as f:
            assert text == f.read(), rec["file"]


def test_heads_override_changes_only_attention_width():
    ops16 = frontend.gen_ops("GAT", 1, 100, 1000, 64)
    ops8 = frontend.gen_ops("GAT", 1, 100, 1000, 64, heads=8)
    assert ops8[11]["INPUT"]["size_per_feature"] == [512, 32]   # X1 [E,128] x alpha [E,8]
    assert ops16[11]["INPUT"]["size_per_feature"] == [512, 64]
    assert ops8[0] == ops16[0]


def test_unknown_network():
    with pytest.raises(ValueError):
        frontend.gen_ops("XYZ", 1, 10, 10, 10)
