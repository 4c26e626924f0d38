"""Test-suite hygiene: a second top-level `def test_x` in a module silently replaces the first, and
pytest then collects only the survivor (the oracle edge-case test was dead code
for a round).  Every test module is parsed and checked for duplicate top-level names."""
import ast
import glob
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
MODULES = sorted(glob.glob(os.path.join(HERE, "test_*.py")))


@pytest.mark.parametrize("path", MODULES, ids=[os.path.basename(p) for p in MODULES])
def test_no_shadowed_test_names(path):
    tree = ast.parse(open(path).read(), filename=path)
    seen, dup = {}, []
    for node in tree.body:
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)) and node.name.startswith(("test", "Test")):
            if node.name in seen:
                dup.append(f"{node.name} (lines {seen[node.name]} and {node.lineno})")
            seen[node.name] = node.lineno
    assert not dup, f"{os.path.basename(path)} redefines: " + ", ".join(dup)
