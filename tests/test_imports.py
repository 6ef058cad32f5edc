"""Every `from X import Y` in the test modules, bench.py and __graft_entry__.py — including the ones inside GPU test
functions, which only run on the GPU box — names something that exists (a CPU check that keeps a misspelt import
from costing a GPU run)."""
import ast
import importlib
from pathlib import Path

REPO = Path(__file__).resolve().parent.parent


def test_imported_names_exist():
    files = sorted((REPO / "tests").glob("test_*.py")) + [REPO / "bench.py", REPO / "__graft_entry__.py"]
    missing = []
    for f in files:
        for n in ast.walk(ast.parse(f.read_text())):
            if not (isinstance(n, ast.ImportFrom) and n.module and n.level == 0):
                continue
            if n.module.split(".")[0] in ("torch",):  # third-party: importable here, not ours to check
                continue
            m = importlib.import_module(n.module)
            for a in n.names:
                if a.name == "*" or hasattr(m, a.name):
                    continue
                try:
                    importlib.import_module(f"{n.module}.{a.name}")
                except ImportError:
                    missing.append(f"{f.name}:{n.lineno} from {n.module} import {a.name}")
    assert not missing, missing
