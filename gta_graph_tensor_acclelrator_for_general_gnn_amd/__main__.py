"""python -m gta_graph_tensor_acclelrator_for_general_gnn_amd: start.py's flow on the GPU (cli.py)."""
import sys

from .cli import main

sys.exit(main())
