"""The GPU test modules only run on the MI355X box: check here, on the CPU,
that every module-level name they load is defined or imported (a missing
import would otherwise surface only in the round-end GPU run)."""
import ast
import builtins
import glob
import os

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _undefined(path):
    tree = ast.parse(open(path).read())
    defined = set(dir(builtins)) | {"__file__", "__name__"}
    for n in ast.walk(tree):
        if isinstance(n, (ast.Import, ast.ImportFrom)):
            defined.update((a.asname or a.name).split(".")[0] for a in n.names)
        elif isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef, ast.Lambda)):
            if not isinstance(n, ast.Lambda):
                defined.add(n.name)
        elif isinstance(n, ast.arg):
            defined.add(n.arg)
        elif isinstance(n, ast.Name) and isinstance(n.ctx, (ast.Store, ast.Del)):
            defined.add(n.id)
        elif isinstance(n, ast.ExceptHandler) and n.name:
            defined.add(n.name)
        elif isinstance(n, (ast.Global, ast.Nonlocal)):
            defined.update(n.names)
    used = {n.id for n in ast.walk(tree) if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load)}
    return sorted(used - defined)


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(HERE, "*.py"))), ids=os.path.basename)
def test_no_undefined_names(path):
    assert _undefined(path) == []
