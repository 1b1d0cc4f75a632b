#!/usr/bin/env python3
"""Source-header check (the reference's license-header CI step, ``.licenserc.yaml``): every
non-empty Python module opens with a docstring and every C++/HIP source with a comment block
that says what it is. Exits non-zero and lists the offenders.

    python hack/check_headers.py
"""
from __future__ import annotations

import ast
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PY_DIRS = ("walkai_nos_amd", "tools", "tests", "hack")
CPP_DIRS = ("csrc",)


def py_ok(path: str) -> bool:
    src = open(path, encoding="utf-8").read()
    if not src.strip():
        return True  # empty package markers
    try:
        return ast.get_docstring(ast.parse(src)) is not None
    except SyntaxError:
        return False


def cpp_ok(path: str) -> bool:
    with open(path, encoding="utf-8") as f:
        first = f.readline().strip()
    return first.startswith("//") or first.startswith("/*")


def main() -> int:
    bad = []
    for d in PY_DIRS:
        for dirpath, _, files in os.walk(os.path.join(ROOT, d)):
            if "__pycache__" in dirpath:
                continue
            bad += [os.path.join(dirpath, f) for f in files if f.endswith(".py") and not py_ok(os.path.join(dirpath, f))]
    for d in CPP_DIRS:
        for dirpath, _, files in os.walk(os.path.join(ROOT, d)):
            bad += [os.path.join(dirpath, f) for f in files
                    if f.endswith((".cpp", ".hip", ".h")) and not cpp_ok(os.path.join(dirpath, f))]
    for b in bad:
        print("missing header:", os.path.relpath(b, ROOT))
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
