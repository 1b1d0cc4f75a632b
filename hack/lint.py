"""Repository lint: fails (exit 1) on errors, never masks them.

* ``ruff check`` when ruff is importable (CI installs it; this image has no network to);
* otherwise, and always: every Python file compiles, no unused imports (AST: a module-level or
  function-level ``import`` whose bound name is never read, outside ``__init__.py`` re-exports and
  lines marked ``# noqa``), no duplicate top-level definitions, no bare ``except:``;
* the license/header check (``hack/check_headers.py``).

    python hack/lint.py [paths...]
"""
from __future__ import annotations

import ast
import os
import subprocess
import sys
from typing import List

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEFAULT = ["walkai_nos_amd", "tests", "tools", "hack", "bench.py", "__graft_entry__.py"]


def py_files(paths: List[str]) -> List[str]:
    out = []
    for p in paths:
        p = os.path.join(ROOT, p)
        if os.path.isfile(p) and p.endswith(".py"):
            out.append(p)
        for d, _, fs in os.walk(p):
            if "__pycache__" in d or "/_native" in d:
                continue
            out += [os.path.join(d, f) for f in fs if f.endswith(".py")]
    return sorted(set(out))


def check_file(path: str) -> List[str]:
    src = open(path).read()
    rel = os.path.relpath(path, ROOT)
    try:
        tree = ast.parse(src, rel)
    except SyntaxError as e:
        return [f"{rel}:{e.lineno}: syntax error: {e.msg}"]
    lines = src.splitlines()
    errs: List[str] = []
    used = {n.id for n in ast.walk(tree) if isinstance(n, ast.Name)}
    used |= {n.value.id for n in ast.walk(tree) if isinstance(n, ast.Attribute) and isinstance(n.value, ast.Name)}
    # names listed in __all__ or used in string annotations count as used
    for n in ast.walk(tree):
        if isinstance(n, ast.Constant) and isinstance(n.value, str):
            used |= set(n.value.replace("[", " ").replace("]", " ").replace(",", " ").replace(".", " ").split())
    if not path.endswith("__init__.py"):
        for n in ast.walk(tree):
            if isinstance(n, (ast.Import, ast.ImportFrom)):
                if "noqa" in lines[n.lineno - 1] or (isinstance(n, ast.ImportFrom) and n.module == "__future__"):
                    continue
                for a in n.names:
                    name = (a.asname or a.name).split(".")[0]
                    if name != "*" and name not in used:
                        errs.append(f"{rel}:{n.lineno}: unused import {a.asname or a.name}")
    seen = {}
    for n in tree.body:
        if isinstance(n, (ast.FunctionDef, ast.AsyncFunctionDef, ast.ClassDef)):
            if n.name in seen and "noqa" not in lines[n.lineno - 1]:
                errs.append(f"{rel}:{n.lineno}: {n.name} redefines line {seen[n.name]}")
            seen[n.name] = n.lineno
    for n in ast.walk(tree):
        if isinstance(n, ast.ExceptHandler) and n.type is None and "noqa" not in lines[n.lineno - 1]:
            errs.append(f"{rel}:{n.lineno}: bare except")
    return errs


def main(argv: List[str]) -> int:
    paths = argv or DEFAULT
    rc = 0
    try:
        import ruff  # noqa: F401
        r = subprocess.run([sys.executable, "-m", "ruff", "check", *paths], cwd=ROOT)
        rc |= r.returncode
    except ImportError:
        pass
    errs = [e for f in py_files(paths) for e in check_file(f)]
    for e in errs:
        print(e)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "hack", "check_headers.py")], cwd=ROOT)
    rc |= r.returncode
    if errs:
        print(f"{len(errs)} lint error(s)")
        rc |= 1
    return rc


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
