"""End-to-end without the reference: layer -> op graph -> fusion search -> stream -> HIP execution.

  frontend.gen_ops   (genGraphOP.gen_yaml)          op graph
  tiles.metadata     (preprocessing.py)             tile sizes + max tile nnz of THIS graph
  compiler.search    (compiler.compile)             ranked fusion partitions + tiles
  lowering.lower     (interpreter.interpret)        instruction stream
  executor           (replaces simulator.simulate)  real outputs on MI355X
Each stage is pinned byte-exactly to the reference's own outputs (tests/test_frontend.py,
test_compiler.py, test_lowering.py); the executor to the fp64 oracle (test_gpu_executor.py).
"""
from . import compiler, executor, frontend, ir, lowering, tiles
from .semantics import Semantics


class Layer:
    """One compiled GNN layer bound to a graph: op graph, chosen partition, stream."""

    def __init__(self, network, layer, graph, feature, reorder=False, heads=16, candidate=0, tile_start=None,
                 op_array=None, tile_size_list=None, metadata=None, pingpang=True, sinput=False):
        """pingpang / sinput: compile()'s isPingpang / isSinput (code/compiler.py:475-510) for the
        fusion search; the reference's start.py passes its command-line flags through."""
        self.network, self.layer, self.reorder = network, layer, reorder
        self.graph = graph
        self.records = frontend.gen_ops(network, layer, graph.n_rows, graph.nnz, feature, reorder, heads)
        self.sem = Semantics.for_network(network, reorder)
        self.opgraph = ir.OpGraph(self.records, self.sem.inputs)
        if op_array is None:
            if metadata is None:
                # tile sizes 64..4096 rows: the 2 MiB buffer rules out larger row tiles
                # for every genGraphOP layer, and each size costs one tile_nnz pass
                metadata = tiles.metadata(graph, start=tile_start or 64, end=min(graph.n_rows, 4096))
            self.metadata = metadata
            sizes, maxl = metadata
            cands = compiler.search(self.records, graph.n_rows, sizes, maxl, pingpang=pingpang, sinput=sinput)
            self.candidates = cands
            if cands:
                op_array, tile_size_list = cands[min(candidate, len(cands) - 1)][:2]
            else:
                # nothing fits the modelled 2 MiB ASIC buffer (e.g. GIN/Cora layer 1 in the
                # reference too); the GPU has no such limit: fuse along the aggregate chain
                op_array, tile_size_list = self._default_partition(), None
                tile_size_list = [[sizes[0], 1] for _ in op_array]
        if not hasattr(self, "metadata"):
            self.metadata = metadata
        self.op_array, self.tile_size_list = op_array, tile_size_list
        self.stream_records = lowering.lower(self.records, graph.n_rows, op_array, tile_size_list)
        self.stream = ir.Stream(self.stream_records)

    def _default_partition(self):
        """scatter -> applyedge -> gather chains in one block each, every other op alone."""
        g, blocks, used = self.opgraph, [], set()
        for op in g.ops:
            if op.type == "gather" and op.idx not in used:
                chain = [op.idx]
                for p in g.producers(op.idx):
                    if g.ops[p].type == "applyedge":
                        chain.append(p)
                        chain += [q for q in g.producers(p) if g.ops[q].type == "scatter"]
                    elif g.ops[p].type == "scatter":
                        chain.append(p)
                chain = sorted(set(c for c in chain if c not in used))
                used.update(chain)
                blocks.append(chain)
        blocks += [[op.idx] for op in g.ops if op.idx not in used]
        return blocks

    def run(self, tensors, plan_chunk=512, model=None, sync=True):
        """sync=False: no device synchronisation around the stream (res.elapsed_s is then host time
        only); a multi-layer forward synchronises once at its end instead of twice per layer."""
        res, ex = executor.run_stream(self.opgraph, self.stream, self.graph, tensors, self.sem, plan_chunk, sync=sync)
        if model:
            executor.attach_model(res, self.stream_records, self.tile_size_list, self.graph, model)
        return res, ex


def run_layer(network, layer, graph, tensors, feature, **kw):
    lay = Layer(network, layer, graph, feature, **{k: v for k, v in kw.items() if k != "plan_chunk"})
    res, _ = lay.run(tensors, plan_chunk=kw.get("plan_chunk", 512))
    return lay, res
