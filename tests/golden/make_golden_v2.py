"""Golden fixtures for the legacy V2 lowering (V2/interpreter.py:13-271 create_list), made by
RUNNING the reference's own function (dev container only; outputs are data, no source is kept).

Cases: the committed V2/GAT_Cora.yaml and V2/simpletest.yaml op graphs under several block
partitions / tile sizes (those of V2/interpreter.py:273-295 and V2/compiler.py's candidates),
plus one op graph with an emptied output list, where the reference raises.

Round 6: also the reference's modelled triple of the legacy boundary, pipeline(data, op_fused,
isCycle) -> (total_p, record, rw) (V2/simulator.py:152-209), for every case at isCycle 1 and 0,
plus the module's own __main__ call (:236-239).  The sparse tables it reads come from the
reference's own V2/preprocessing.calculate_sparsity run on the dense adjacency of the seeded
synthetic graph of each dataset shape (graph.synthetic(n, e, seed=0)), so the count-of-zeros quirk
is the reference's.  -> v2/pipeline_triples.json

Usage (in the survey/dev container only):  python tests/golden/make_golden_v2.py [--pipeline-only]
"""
import contextlib
import importlib.util
import json
import os
import tempfile

import yaml

REF = "/root/reference"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "v2")

CASES = [  # (op graph file, dataset, op_list, tile_size, node_num)
    ("GAT_Cora.yaml", "citeseer", [[0], [1], [2], [4], [5], [6], [7], [8], [9], [10], [3], [11], [12], [13]],
     [3327] * 14, 2708),
    ("GAT_Cora.yaml", "citeseer", [[0, 1, 2], [5], [4, 6, 7, 8, 9, 10], [3, 11, 12, 13]], [579, 3327, 3327, 3327], 3327),
    ("GAT_Cora.yaml", "cora", [[0, 1, 2], [5], [4, 6, 7, 8, 9, 10], [3, 11, 12, 13]], [100, 2708, 2708, 579], 2708),
    ("GAT_Cora.yaml", "pubmed", [[0], [1], [2], [4, 5, 6], [7, 8, 9, 10], [3, 11, 12, 13]],
     [19717, 19717, 19717, 19717, 16384, 579], 19717),
    ("GAT_Cora.yaml", "citeseer", [[0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13]], [1024], 3327),
    ("simpletest.yaml", "cora", [[0], [1], [2], [3], [4], [5], [6], [7], [8]], [2708] * 9, 2708),
    ("simpletest.yaml", "cora", [[0, 1, 2], [3, 4, 5], [6, 7, 8]], [64, 512, 2708], 2708),
]


@contextlib.contextmanager
def scratch():
    cwd = os.getcwd()
    with tempfile.TemporaryDirectory() as d:
        os.chdir(d)
        try:
            yield d
        finally:
            os.chdir(cwd)


def _load(name, rel):
    spec = importlib.util.spec_from_file_location(name, os.path.join(REF, rel))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def pipeline_triples():
    """The reference's (total_p, record, rw) for every case, isCycle 1 and 0."""
    import re
    import sys

    import numpy as np
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
    from gta_graph_tensor_acclelrator_for_general_gnn_amd import graph as G
    sim = _load("v2_simulator", "V2/simulator.py")
    pre = _load("v2_preprocessing", "V2/preprocessing.py")
    manifest = json.load(open(os.path.join(OUT, "manifest.json")))
    out = []
    runs = [(m, m["op_list_records"], isc) for m in manifest if "file" in m for isc in (1, 0)]
    case0 = next(m for m in manifest if m.get("file") == "case0.yaml")
    # V2/simulator.py:236-239: the module's own call, on the committed fused.yaml (= case 0)
    runs.append((case0, [[0], [1], [2], [4], [5], [6], [7], [8], [9], [10], [3], [11], [12], [13]], 1))
    for m, op_fused, isc in runs:
        with open(os.path.join(OUT, m["file"])) as f:
            data = yaml.safe_load(f)
        n, e = G.SHAPES[m["dataset"]]
        g = G.synthetic(n, e, seed=0)
        ip, ix = g.numpy()
        tables = {}
        with scratch() as d:
            dense = np.zeros((n, n), np.uint8)
            dense[np.repeat(np.arange(n), np.diff(ip)), ix] = 1
            np.save(os.path.join(d, "adj.npy"), dense)
            del dense
            for rec in data.values():
                p = rec["sparse_path"]
                if p and p not in tables:
                    T, C = (int(v) for v in re.search(r"_(\d+)_(\d+)\.yaml$", p).groups())
                    tables[p] = [[int(v) for v in row] for row in pre.calculate_sparsity(T, C, os.path.join(d, "adj.npy"))]
        sim.read = lambda path, _t=tables: _t[path]
        sim.bw = 128 * (1024 ** 3) * (10 ** (-9))
        sim.compute_perfom = [[16, 16], [16, 16]]
        sim.load_p = sim.save_p = sim.save_start_p = sim.c_p = sim.total_p = sim.rw = 0
        sim.compute_p = [0, 0]
        total_p, record, rw = sim.pipeline(data, op_fused, isc)
        out.append({"file": m["file"], "dataset": m["dataset"], "graph": [n, e, 0], "op_fused": op_fused,
                    "isCycle": isc, "total_p": total_p, "rw": rw, "record": record})
        print(m["file"], isc, total_p, rw, len(record), flush=True)
    with open(os.path.join(OUT, "pipeline_triples.json"), "w") as f:
        json.dump(out, f)


def main():
    if "--pipeline-only" in __import__("sys").argv:
        pipeline_triples()
        return
    spec = importlib.util.spec_from_file_location("v2_interpreter", os.path.join(REF, "V2", "interpreter.py"))
    v2 = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(v2)
    os.makedirs(OUT, exist_ok=True)
    manifest = []
    for k, (src, ds, op_list, tiles, n) in enumerate(CASES):
        name = f"case{k}.yaml"
        with scratch():
            v2.create_list(ds, os.path.join(REF, "V2", src), "out.yaml", op_list, tiles, n)
            data = open("out.yaml").read()
        with open(os.path.join(OUT, name), "w") as f:
            f.write(data)
        recs, k0 = [], 0
        for blk in op_list:
            recs.append(list(range(k0, k0 + len(blk))))
            k0 += len(blk)
        manifest.append({"file": name, "op_graph": src, "dataset": ds, "op_list": op_list, "tile_size": tiles,
                         "node_num": n, "op_list_records": recs})
    # error case: op 3 (scatter) with no consumers -> the reference indexes output_list[0]
    ops = yaml.safe_load(open(os.path.join(REF, "V2", "GAT_Cora.yaml")))
    ops[3]["OUTPUT"]["output_list"] = []
    with scratch():
        yaml.safe_dump(ops, open("mut.yaml", "w"))
        try:
            v2.create_list("citeseer", "mut.yaml", "out.yaml", [[0], [1], [2], [3]], [64] * 4, 3327)
            err = None
        except Exception as ex:  # noqa: BLE001 - the reference's failure mode is the fixture
            err = type(ex).__name__
    manifest.append({"error_case": "GAT_Cora.yaml op 3 output_list = []", "op_list": [[0], [1], [2], [3]],
                     "raises": err})
    if not os.path.exists(os.path.join(os.path.dirname(OUT), "v2_simpletest.yaml")):
        import shutil
        shutil.copy(os.path.join(REF, "V2", "simpletest.yaml"), os.path.join(os.path.dirname(OUT), "v2_simpletest.yaml"))
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print(json.dumps(manifest[-1]), len(manifest) - 1, "cases")
    pipeline_triples()


if __name__ == "__main__":
    main()
