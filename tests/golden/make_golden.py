"""Generate the golden fixtures under tests/golden/ by RUNNING the reference.

Test infrastructure only (never shipped, never run on the GPU box): this script
imports the reference's own Python modules from /root/reference (read-only),
runs them in a scratch directory, and commits ONLY their outputs (YAML/JSON/npz
data) -- never reference source text.

What it pins:
  1. op-graph YAMLs       vTCAD/GraphOP/genGraphOP.py:27-154   gen_yaml()
  2. tile-nnz metadata    code/preprocessing.py:12-40,53-72     calculate_sparsity / cal_min_sparsity / gen_size
  3. fusion candidates    code/compiler.py:475-510              compile()
  4. instruction streams  code/interpreter.py:805-849           interpret()
  5. modelled (cycles,rw) code/simulator.py:370-502             simulate()   (its hard-coded
                          /Users/... record path, :499-500, is monkeypatched to a no-op)
  6. legacy V2 stream     V2/interpreter.py:13-271              create_list()

Graph used for (2),(3),(5): a seeded Cora-shaped random graph (N=2708), built
here with numpy (seed 0) and saved as CSR in golden/cora_graph.npz, so the
tests can rebuild the same dense adjacency without the reference.

Usage (in the survey/dev container only):  python tests/golden/make_golden.py
"""
import contextlib
import io
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np
import yaml

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))
HW_INFO = os.path.join(REF, "FinalVersion For Paper", "hardware_info.yaml")

NETWORKS = ["GCN", "GAT", "SGC", "GraphSAGE", "GIN", "DGN", "PNA"]
DATASETS = {  # genGraphOP.py:183-199 shapes (+ flickr from code/compiler.py:495 and the standard E)
    "cora": (2708, 10556, 1433),
    "flickr": (89250, 899756, 500),
    "reddit": (232965, 114615892, 602),
}
TILE_SIZES_CORA = [64, 128, 256, 512, 1024, 2048, 2752]


def cora_graph(seed=0, n=2708, e=10556):
    """Seeded Cora-shaped simple digraph: unique (dst,src) pairs, no self loops.
    rows = destination (R direction), cols = source (C direction)."""
    rng = np.random.default_rng(seed)
    pairs = set()
    while len(pairs) < e:
        need = e - len(pairs)
        d = rng.integers(0, n, size=need * 2)
        s = rng.integers(0, n, size=need * 2)
        for a, b in zip(d.tolist(), s.tolist()):
            if a != b:
                pairs.add((a, b))
                if len(pairs) == e:
                    break
    arr = np.array(sorted(pairs), dtype=np.int64)
    dst, src = arr[:, 0], arr[:, 1]
    indptr = np.zeros(n + 1, dtype=np.int64)
    np.add.at(indptr, dst + 1, 1)
    indptr = np.cumsum(indptr)
    return indptr, src.astype(np.int32)


@contextlib.contextmanager
def scratch():
    old = os.getcwd()
    d = tempfile.mkdtemp(prefix="gta_golden_")
    shutil.copy(HW_INFO, os.path.join(d, "hardware_info.yaml"))
    os.chdir(d)
    try:
        yield d
    finally:
        os.chdir(old)
        shutil.rmtree(d, ignore_errors=True)


def op_yaml_path(net, ds, layer, reorder):
    m = "trans" if reorder else "original"
    return f"Network/{net}/{net}-{ds}/{net}-{m}/{net}-layer{layer}-{m}.yaml"


def main():
    os.environ["PYTHONDONTWRITEBYTECODE"] = "1"
    sys.dont_write_bytecode = True
    sys.path.insert(0, os.path.join(REF, "vTCAD", "GraphOP"))
    sys.path.insert(0, os.path.join(REF, "code"))
    import genGraphOP  # noqa: E402
    import preprocessing  # noqa: E402
    import compiler  # noqa: E402
    import interpreter  # noqa: E402
    import simulator  # noqa: E402

    simulator.save_rw_record_to_file = lambda *a, **k: None  # :499-500 writes to /Users/...

    os.makedirs(os.path.join(OUT, "ops"), exist_ok=True)
    os.makedirs(os.path.join(OUT, "streams"), exist_ok=True)
    manifest = {"ops": [], "streams": [], "tiles": {}, "compile": {}, "simulate": [], "v2": None}

    # graph for tile metadata (saved so tests rebuild it without the reference)
    indptr, indices = cora_graph()
    np.savez_compressed(os.path.join(OUT, "cora_graph.npz"), indptr=indptr, indices=indices)
    n = 2708
    dense = np.zeros((n, n), dtype=np.float32)
    dst = np.repeat(np.arange(n), np.diff(indptr))
    dense[dst, indices] = 1.0

    with scratch():
        # ---- 1. op YAMLs -------------------------------------------------
        for ds, (N, E, F) in DATASETS.items():
            for net in NETWORKS:
                for layer in (1, 2, 3):
                    for reorder in (False, True):
                        if ds != "cora" and not (layer == 1 and net in ("GAT", "GCN", "GraphSAGE", "GIN")):
                            continue
                        p = op_yaml_path(net, ds, layer, reorder)
                        with contextlib.redirect_stdout(io.StringIO()):
                            genGraphOP.gen_yaml(p, N, E, F, net, layer, reorder)
                        if not os.path.exists(p):
                            continue
                        name = f"{net}-{ds}-layer{layer}-{'trans' if reorder else 'original'}.yaml"
                        shutil.copy(p, os.path.join(OUT, "ops", name))
                        manifest["ops"].append({"file": name, "network": net, "dataset": ds, "layer": layer,
                                                "reorder": reorder, "N": N, "E": E, "F": F})

        # ---- 2. tile-nnz metadata ----------------------------------------
        os.makedirs("dataset/cora", exist_ok=True)
        np.save("dataset/cora/adj_cora.npy", dense)
        tiles = {}
        sizes = preprocessing.gen_size(64, 2708)  # code/preprocessing.py:65-72
        manifest["tiles"]["gen_size_64_2708"] = sizes
        for T in sizes:
            sp = preprocessing.calculate_sparsity(T, 1, "dataset/cora/adj_cora.npy")
            with open(f"dataset/cora/adj_cora_{T}_1.yaml", "w") as f:
                yaml.dump(sp, f)
            if T in TILE_SIZES_CORA:
                tiles[f"T{T}"] = np.asarray(sp, dtype=np.int32)
        maxlist = [preprocessing.cal_min_sparsity("cora", T) for T in sizes]
        with open("dataset/cora/sizelist_cora.yaml", "w") as f:
            yaml.dump(sizes, f)
        with open("dataset/cora/maxlist_cora.yaml", "w") as f:
            yaml.dump(maxlist, f)
        np.savez_compressed(os.path.join(OUT, "cora_tiles.npz"), **tiles)
        manifest["tiles"]["maxlist"] = [int(x) for x in maxlist]

        # ---- 3+4. compile() candidates and interpret() streams (cora) -----
        for net in NETWORKS:
            for layer in (1, 2, 3):
                for reorder in (False, True):
                    p = op_yaml_path(net, "cora", layer, reorder)
                    if not os.path.exists(p):
                        continue
                    t0 = time.time()
                    try:
                        with contextlib.redirect_stdout(io.StringIO()):
                            res = compiler.compile("cora", net, f"layer{layer}", reorder, False, True)[0]
                    except Exception as ex:  # record, do not hide
                        manifest["compile"][p] = {"error": repr(ex)}
                        continue
                    key = f"{net}-cora-layer{layer}-{'trans' if reorder else 'original'}"
                    manifest["compile"][key] = {
                        "n_candidates": len(res),
                        "seconds": round(time.time() - t0, 3),
                        "top": [[r[0], r[1], int(r[2]), r[3]] for r in res[:8]],
                        "last": [[r[0], r[1], int(r[2]), r[3]] for r in res[-2:]],
                    }
                    picks = list(res[:3]) + list(res[-1:])
                    for k, r in enumerate(picks):
                        _interpret_one(interpreter, manifest, net, "cora", layer, reorder, r[0], r[1], f"c{k}")

        # ---- metric-shaped streams (hand-picked fusions, large N) ----------
        big = [
            # GAT layer1: the metric block [3,11,12] = scatter C -> applyedge MUL -> gather ADD
            ("GAT", "reddit", 1, False, [[0], [1], [2], [4, 5, 6], [7], [8], [10], [9], [3, 11, 12], [13]], 512),
            ("GAT", "flickr", 1, False, [[0], [1], [2], [4, 5, 6, 7, 8], [10, 9], [3, 11, 12], [13]], 512),
            ("GAT", "flickr", 1, False, [[0], [1], [2], [4, 5, 6, 7, 8], [10, 9], [3, 11, 12, 13]], 1024),
            ("GCN", "reddit", 1, False, [[0, 1, 2], [3]], 512),
            ("GCN", "reddit", 1, True, [[0], [1, 2, 3]], 512),
            ("GraphSAGE", "reddit", 1, False, [[0, 1, 2], [3], [4], [5, 6]], 512),
            ("GIN", "reddit", 1, False, [[0, 1, 2], [3, 4], [5], [6], [7], [8]], 512),
            ("GAT", "reddit", 1, True, [[0], [1], [2], [4, 5, 6, 8], [3, 7, 10], [9], [11, 12]], 512),
        ]
        for net, ds, layer, reorder, op_array, T in big:
            tiles_ = [[T, 1] for _ in op_array]
            _interpret_one(interpreter, manifest, net, ds, layer, reorder, op_array, tiles_, f"h{T}")

        # ---- 5. simulate() (cycles, rw) for a few cora streams ------------
        sim_cases = [("GCN", 1, False), ("GraphSAGE", 1, False), ("GIN", 1, False), ("SGC", 1, False),
                     ("GCN", 2, True)]
        for net, layer, reorder in sim_cases:
            key = f"{net}-cora-layer{layer}-{'trans' if reorder else 'original'}"
            if key not in manifest["compile"] or not manifest["compile"][key].get("top"):
                continue
            best = manifest["compile"][key]["top"][0]
            op_array, tiles_ = best[0], best[1]
            with contextlib.redirect_stdout(io.StringIO()):
                interpreter.interpret("cora", net, reorder, f"layer{layer}", op_array, tiles_)
            t0 = time.time()
            with contextlib.redirect_stdout(io.StringIO()):
                cycles, rw = simulator.simulate(tiles_, "cora", net, f"layer{layer}", reorder, False)
            manifest["simulate"].append({"key": key, "op_array": op_array, "tile_size_list": tiles_,
                                         "cycles": int(cycles), "rw": int(rw),
                                         "seconds": round(time.time() - t0, 2)})
            print("simulate", key, cycles, rw, round(time.time() - t0, 1), "s", flush=True)

    # ---- 6. legacy V2 stream (create_list) -------------------------------
    sys.path.insert(0, os.path.join(REF, "V2"))
    import importlib.util
    spec = importlib.util.spec_from_file_location("v2_interpreter", os.path.join(REF, "V2", "interpreter.py"))
    v2 = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(v2)
    op_list = [[0], [1], [2], [4], [5], [6], [7], [8], [9], [10], [3], [11], [12], [13]]
    with scratch():
        v2.create_list("citeseer", os.path.join(REF, "V2", "GAT_Cora.yaml"), "fused.yaml", op_list, [3327] * 14, 2708)
        shutil.copy("fused.yaml", os.path.join(OUT, "v2_fused.yaml"))
    shutil.copy(os.path.join(REF, "V2", "GAT_Cora.yaml"), os.path.join(OUT, "v2_GAT_Cora.yaml"))
    same = open(os.path.join(OUT, "v2_fused.yaml")).read() == open(os.path.join(REF, "V2", "fused.yaml")).read()
    manifest["v2"] = {"op_list": op_list, "tile_size": [3327] * 14, "node_num": 2708,
                      "dataset": "citeseer", "matches_committed_fused_yaml": same}

    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    print("ops", len(manifest["ops"]), "streams", len(manifest["streams"]), "sim", len(manifest["simulate"]))


def _interpret_one(interpreter, manifest, net, ds, layer, reorder, op_array, tiles_, tag):
    m = "trans" if reorder else "original"
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            interpreter.interpret(ds, net, reorder, f"layer{layer}", op_array, tiles_)
    except Exception as ex:
        manifest["streams"].append({"network": net, "dataset": ds, "layer": layer, "reorder": reorder,
                                    "op_array": op_array, "tile_size_list": tiles_, "error": repr(ex)})
        return
    src = f"Results/Insts/{net}-{ds}-layer{layer}-{m}.yaml"
    name = f"{net}-{ds}-layer{layer}-{m}-{tag}.yaml"
    shutil.copy(src, os.path.join(OUT, "streams", name))
    manifest["streams"].append({"file": name, "network": net, "dataset": ds, "layer": layer, "reorder": reorder,
                                "op_yaml": f"{net}-{ds}-layer{layer}-{m}.yaml",
                                "op_array": op_array, "tile_size_list": tiles_})


if __name__ == "__main__":
    main()
