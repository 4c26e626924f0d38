"""MI355X-native execution backend for GTA's graph message-passing ISA.

The reference (Jagnate/GTA_graph_tensor_acclelrator_for_general_GNN) lowers a
GNN op graph into an instruction stream (code/interpreter.py:805-849) and
"executes" it with a Python cycle model (code/simulator.py:370-502).  This
package executes the same stream on real tensors: each ISA op / fused pattern
is a hand-written gfx950 kernel in libgta.so (include/gta.h), called through
ctypes from the host-side executor.  See DESIGN.md.
"""
from . import _lib  # noqa: F401
from .graph import Graph, synthetic, dataset_graph, from_numpy  # noqa: F401

__all__ = ["Graph", "synthetic", "dataset_graph", "from_numpy"]
