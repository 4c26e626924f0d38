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


ROOT = os.path.dirname(HERE)
# the package, the entry points, and the code only a GPU box runs (GPU tests, probes) or the oracle
PRODUCT = sorted(glob.glob(os.path.join(ROOT, "gta_graph_tensor_acclelrator_for_general_gnn_amd", "*.py"))
                 + [os.path.join(ROOT, "bench.py"), os.path.join(ROOT, "__graft_entry__.py")]
                 + glob.glob(os.path.join(HERE, "*.py")) + glob.glob(os.path.join(ROOT, "scripts", "*.py"))
                 + glob.glob(os.path.join(ROOT, "oracle", "*.py")))


_SCOPES = (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda, ast.ClassDef)


def _own(node):
    """node's own scope: every sub-node except the insides of nested functions / lambdas / classes
    (their names, decorators and defaults belong to node's scope; their bodies do not)."""
    todo = list(ast.iter_child_nodes(node))
    while todo:
        sub = todo.pop()
        yield sub
        if isinstance(sub, _SCOPES):
            todo.extend(sub.decorator_list if not isinstance(sub, ast.Lambda) else [])
            if not isinstance(sub, ast.ClassDef):
                todo.extend(d for d in sub.args.defaults + sub.args.kw_defaults if d is not None)
            else:
                todo.extend(sub.bases)
        else:
            todo.extend(ast.iter_child_nodes(sub))


def _bound(node):
    """Names node's own scope binds (params, assignments, loop / with / except targets, imports,
    nested defs, comprehension targets, global / nonlocal declarations)."""
    out = set()
    if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda)):
        a = node.args
        for arg in a.posonlyargs + a.args + a.kwonlyargs + [a.vararg, a.kwarg]:
            if arg is not None:
                out.add(arg.arg)
    for sub in _own(node):
        if isinstance(sub, ast.Name) and isinstance(sub.ctx, (ast.Store, ast.Del)):
            out.add(sub.id)
        elif isinstance(sub, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            out.add(sub.name)
        elif isinstance(sub, (ast.Import, ast.ImportFrom)):
            out.update((al.asname or al.name).split(".")[0] for al in sub.names)
        elif isinstance(sub, ast.ExceptHandler) and sub.name:
            out.add(sub.name)
        elif isinstance(sub, (ast.Global, ast.Nonlocal)):
            out.update(sub.names)
    return out


@pytest.mark.parametrize("path", PRODUCT, ids=[os.path.relpath(p, ROOT) for p in PRODUCT])
def test_no_undefined_names_in_product_code(path):
    """A name read inside a function that no enclosing scope, the module or builtins binds is a
    NameError waiting for the first call -- on a GPU-only path the CPU suite never executes it
    (round 4: an `out_dtype` check pasted into ops.aggregate_blocked)."""
    import builtins
    tree = ast.parse(open(path).read(), filename=path)
    module = _bound(tree) | set(dir(builtins)) | {"__file__", "__name__", "__doc__", "__spec__"}
    missing = []

    def visit(node, outer):  # outer: the names of the enclosing function scopes and the module
        scope = outer | _bound(node) if not isinstance(node, ast.ClassDef) else outer
        for sub in _own(node):
            if isinstance(sub, ast.Name) and isinstance(sub.ctx, ast.Load) and sub.id not in scope \
                    and not isinstance(node, (ast.Module, ast.ClassDef)):
                missing.append(f"{sub.id} (line {sub.lineno})")
            if isinstance(sub, _SCOPES):
                visit(sub, scope)

    visit(tree, module)
    assert not missing, f"{os.path.basename(path)}: undefined " + ", ".join(sorted(set(missing)))
