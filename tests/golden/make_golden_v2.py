"""Golden fixtures for the legacy V2 lowering (V2/interpreter.py:13-271 create_list), made by
RUNNING the reference's own function (dev container only; outputs are data, no source is kept).

Cases: the committed V2/GAT_Cora.yaml and V2/simpletest.yaml op graphs under several block
partitions / tile sizes (those of V2/interpreter.py:273-295 and V2/compiler.py's candidates),
plus one op graph with an emptied output list, where the reference raises.

Usage (in the survey/dev container only):  python tests/golden/make_golden_v2.py
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


def main():
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
        manifest.append({"file": name, "op_graph": src, "dataset": ds, "op_list": op_list, "tile_size": tiles,
                         "node_num": n})
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


if __name__ == "__main__":
    main()
