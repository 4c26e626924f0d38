"""lowering.lower() reproduces the reference interpret() streams byte-for-byte (tests/golden/streams)."""
import os

import pytest

from gta_graph_tensor_acclelrator_for_general_gnn_amd import ir, lowering

from .conftest import load_manifest

STREAMS = load_manifest()["streams"]


def _sid(rec):
    return rec.get("file") or f"{rec['network']}-{rec['dataset']}-layer{rec['layer']}-err-{rec['op_array']}"


@pytest.mark.parametrize("rec", STREAMS, ids=[_sid(r) for r in STREAMS])
def test_stream_bytes_match_reference(golden_dir, manifest, rec):
    m = "trans" if rec["reorder"] else "original"
    op_file = f"{rec['network']}-{rec['dataset']}-layer{rec['layer']}-{m}.yaml"
    records = ir.read_yaml(os.path.join(golden_dir, "ops", op_file))
    n = lowering.DATASET_NODES[rec["dataset"]]
    if "error" in rec:  # the reference raised on this partition; so must the restatement
        with pytest.raises((TypeError, ValueError, IndexError)):
            lowering.lower(records, n, rec["op_array"], rec["tile_size_list"])
        return
    text = lowering.dump(lowering.lower(records, n, rec["op_array"], rec["tile_size_list"]))
    with open(os.path.join(golden_dir, "streams", rec["file"])) as f:
        gold = f.read()
    assert text == gold


def test_interpret_writes_reference_paths(golden_dir, tmp_path, monkeypatch):
    monkeypatch.chdir(tmp_path)
    os.makedirs("Network/GCN/GCN-cora/GCN-original")
    import shutil
    shutil.copy(os.path.join(golden_dir, "ops", "GCN-cora-layer1-original.yaml"),
                "Network/GCN/GCN-cora/GCN-original/GCN-layer1-original.yaml")
    out = lowering.interpret("cora", "GCN", False, "layer1", [[0], [3], [1, 2]], [[2752, 1], [64, 1], [128, 1]])
    assert out == "Results/Insts/GCN-cora-layer1-original.yaml" and os.path.exists(out)
