"""A small Go-template/Sprig interpreter for rendering the nos Helm chart in tests (no ``helm`` here).

Covers exactly the template language the chart uses: ``{{ }}`` actions with ``{{-``/``-}}``
whitespace trimming and comments; ``if / else if / else``, ``with``, ``range`` (lists and dicts,
``$k, $v :=`` forms), ``define`` / ``include`` / ``template``; variables (``:=``, ``=``, ``$``);
pipelines and parenthesised sub-pipelines; and the Sprig/Helm functions ``toYaml nindent indent
quote default eq ne lt gt not and or hasPrefix hasSuffix dict list append set index lookup uuidv4
sha256sum print printf fail trim toString required empty int len``.  ``lookup`` returns what the test
gives it (an empty result by default, like ``helm template``).  Not a general implementation:
unknown constructs raise, so a chart change that needs more is noticed.

    python hack/helmlite.py helm-charts/nos [--namespace nos-system] [--set a.b=c]
"""
from __future__ import annotations

import copy
import glob
import hashlib
import json
import os
import re
import sys
import uuid
from typing import Any, Callable, Dict, List, Optional, Tuple

import yaml


class RenderError(Exception):
    pass


class Fail(RenderError):
    """``fail`` called by the chart."""


# -- lexing ------------------------------------------------------------------------------------
ACTION = re.compile(r"{{(-?)(.*?)(-?)}}", re.S)


def _segments(src: str) -> List[Tuple[str, str]]:
    """[("text", s) | ("action", body)] with trim markers applied."""
    out: List[Tuple[str, str]] = []
    pos = 0
    for m in ACTION.finditer(src):
        text = src[pos:m.start()]
        if m.group(1) == "-":
            text = text.rstrip()
        out.append(("text", text))
        body = m.group(2)
        out.append(("action", body.strip()))
        pos = m.end()
        if m.group(3) == "-":
            while pos < len(src) and src[pos] in " \t\r\n":
                pos += 1
    out.append(("text", src[pos:]))
    return out


TOKEN = re.compile(r'\s*(?:("(?:[^"\\]|\\.)*")|(`[^`]*`)|(\()|(\))|(\|)|(:=)|(=)|(,)|'
                   r'(\$[A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*)|(\.[A-Za-z0-9_.]*)|(-?\d+(?:\.\d+)?)|([A-Za-z_][A-Za-z0-9_]*))')


def _tokens(s: str) -> List[Tuple[str, str]]:
    out, pos = [], 0
    s = s.strip()
    while pos < len(s):
        m = TOKEN.match(s, pos)
        if not m or m.end() == pos:
            raise RenderError(f"cannot tokenize {s[pos:]!r}")
        kinds = ("str", "raw", "(", ")", "|", ":=", "=", ",", "var", "field", "num", "ident")
        for k, v in zip(kinds, m.groups()):
            if v is not None:
                out.append((k, v))
                break
        pos = m.end()
    return out


# -- parsing into a tree ------------------------------------------------------------------------
class Node:
    def __init__(self, kind: str, **kw: Any):
        self.kind = kind
        self.__dict__.update(kw)


def _parse(segs: List[Tuple[str, str]], defines: Dict[str, List[Node]]) -> List[Node]:
    pos = 0

    def block(stop: Tuple[str, ...]) -> Tuple[List[Node], str]:
        nonlocal pos
        body: List[Node] = []
        while pos < len(segs):
            kind, s = segs[pos]
            pos += 1
            if kind == "text":
                if s:
                    body.append(Node("text", s=s))
                continue
            if s.startswith("/*"):
                continue
            word = s.split(None, 1)[0] if s else ""
            rest = s[len(word):].strip()
            if word in stop or (word == "else" and "else" in stop):
                return body, s
            if word == "if":
                branches = []
                cond = rest
                while True:
                    b, term = block(("else", "end"))
                    branches.append((cond, b))
                    if term == "end":
                        break
                    t = term.split(None, 1)
                    if len(t) > 1 and t[1].startswith("if "):
                        cond = t[1][3:].strip()
                        continue
                    b, _ = block(("end",))
                    branches.append((None, b))
                    break
                body.append(Node("if", branches=branches))
            elif word in ("with", "range"):
                b, term = block(("else", "end"))
                other: List[Node] = []
                if term != "end":
                    other, _ = block(("end",))
                body.append(Node(word, expr=rest, body=b, other=other))
            elif word == "define":
                name = json.loads(rest)
                b, _ = block(("end",))
                defines[name] = b
            elif word == "template":
                body.append(Node("pipe", expr="include " + rest))
            else:
                body.append(Node("pipe", expr=s))
        return body, ""

    tree, _ = block(())
    return tree


# -- evaluation -----------------------------------------------------------------------------------
def truthy(v: Any) -> bool:
    return not (v is None or v is False or v == 0 or v == "" or v == [] or v == {})


def to_yaml(v: Any) -> str:
    if v is None or v == {} and isinstance(v, dict):
        return "{}" if v == {} else "null"
    return yaml.safe_dump(v, default_flow_style=False, sort_keys=True).rstrip("\n")


class Chart:
    def __init__(self, chart_dir: str, values: Optional[Dict[str, Any]] = None, namespace: str = "nos-system",
                 release: str = "nos", lookup: Optional[Callable[[str, str, str, str], Any]] = None):
        self.dir = chart_dir
        self.meta = yaml.safe_load(open(os.path.join(chart_dir, "Chart.yaml")))
        base = yaml.safe_load(open(os.path.join(chart_dir, "values.yaml"))) or {}
        self.values = _merge(base, values or {})
        self.name = self.meta["name"]
        self.root = {"Values": self.values, "Release": {"Name": release, "Namespace": namespace, "Service": "Helm"},
                     "Chart": {"Name": self.name, "Version": self.meta.get("version"),
                               "AppVersion": self.meta.get("appVersion", "")},
                     "Template": {"BasePath": f"{self.name}/templates"}, "Capabilities": {}}
        self.lookup_fn = lookup or (lambda *a: {})
        self.defines: Dict[str, List[Node]] = {}
        self.files: Dict[str, List[Node]] = {}
        tdir = os.path.join(chart_dir, "templates")
        for path in sorted(glob.glob(os.path.join(tdir, "**", "*"), recursive=True)):
            if os.path.isdir(path):
                continue
            rel = f"{self.name}/templates/" + os.path.relpath(path, tdir)
            tree = _parse(_segments(open(path).read()), self.defines)
            self.files[rel] = tree
            self.defines[rel] = tree

    # -- rendering ------------------------------------------------------------------------
    def render(self) -> Dict[str, str]:
        """Every non-helper template (file name -> rendered text)."""
        out = {}
        for rel, tree in self.files.items():
            if os.path.basename(rel).startswith("_") or rel.endswith(".txt"):
                continue
            out[rel] = self._run(tree, self.root, {"$": self.root})
        return out

    def objects(self) -> List[Dict[str, Any]]:
        objs = []
        for rel, text in self.render().items():
            for doc in yaml.safe_load_all(text):
                if doc:
                    doc.setdefault("__source__", rel)
                    objs.append(doc)
        return objs

    def _run(self, nodes: List[Node], dot: Any, vars_: Dict[str, Any]) -> str:
        out: List[str] = []
        for n in nodes:
            if n.kind == "text":
                out.append(n.s)
            elif n.kind == "pipe":
                v = self._pipeline(n.expr, dot, vars_)
                if v is not _NOOUT:
                    out.append(_fmt(v))
            elif n.kind == "if":
                for cond, body in n.branches:
                    if cond is None or truthy(self._pipeline(cond, dot, vars_)):
                        out.append(self._run(body, dot, vars_))
                        break
            elif n.kind == "with":
                v = self._pipeline(n.expr, dot, vars_)
                out.append(self._run(n.body, v, vars_) if truthy(v) else self._run(n.other, dot, vars_))
            elif n.kind == "range":
                out.append(self._range(n, dot, vars_))
        return "".join(out)

    def _range(self, n: Node, dot: Any, vars_: Dict[str, Any]) -> str:
        m = re.match(r"^(\$\w+)\s*(?:,\s*(\$\w+))?\s*:=\s*(.*)$", n.expr, re.S)
        kv, vv, expr = (m.group(1), m.group(2), m.group(3)) if m else (None, None, n.expr)
        coll = self._pipeline(expr, dot, vars_)
        items = sorted(coll.items()) if isinstance(coll, dict) else list(enumerate(coll or []))
        if not items:
            return self._run(n.other, dot, vars_)
        out = []
        for k, v in items:
            local = dict(vars_)
            if vv:
                local[kv], local[vv] = k, v
            elif kv:
                local[kv] = v
            out.append(self._run(n.body, v, local))
            # assignments to outer variables inside the loop persist (Go semantics)
            for name in vars_:
                if name in local and name not in (kv, vv):
                    vars_[name] = local[name]
        return "".join(out)

    # -- pipelines ---------------------------------------------------------------------------
    def _pipeline(self, expr: str, dot: Any, vars_: Dict[str, Any]) -> Any:
        toks = _tokens(expr)
        if len(toks) >= 2 and toks[0][0] == "var" and toks[1][0] in (":=", "="):
            vars_[toks[0][1]] = self._eval_tokens(toks[2:], dot, vars_)
            return _NOOUT
        return self._eval_tokens(toks, dot, vars_)

    def _eval_tokens(self, toks: List[Tuple[str, str]], dot: Any, vars_: Dict[str, Any]) -> Any:
        cmds: List[List[Tuple[str, str]]] = [[]]
        depth = 0
        for t in toks:
            if t[0] == "(":
                depth += 1
            elif t[0] == ")":
                depth -= 1
            if t[0] == "|" and depth == 0:
                cmds.append([])
            else:
                cmds[-1].append(t)
        val: Any = _NOARG
        for c in cmds:
            val = self._command(c, dot, vars_, val)
        return val

    def _args(self, toks: List[Tuple[str, str]], dot: Any, vars_: Dict[str, Any]) -> List[Any]:
        args, i = [], 0
        while i < len(toks):
            k, v = toks[i]
            if k == "(":
                depth, j = 1, i + 1
                while depth:
                    depth += {"(": 1, ")": -1}.get(toks[j][0], 0)
                    j += 1
                val = self._eval_tokens(toks[i + 1:j - 1], dot, vars_)
                if j < len(toks) and toks[j][0] == "field":  # (pipeline).Field
                    val = _path(val, toks[j][1][1:])
                    j += 1
                args.append(val)
                i = j
                continue
            args.append(self._operand(k, v, dot, vars_))
            i += 1
        return args

    def _operand(self, k: str, v: str, dot: Any, vars_: Dict[str, Any]) -> Any:
        if k == "str":
            return json.loads(v)
        if k == "raw":
            return v[1:-1]
        if k == "num":
            return float(v) if "." in v else int(v)
        if k == "field":
            return _path(dot, v[1:])
        if k == "var":
            name, _, rest = v.partition(".")
            if name not in vars_:
                raise RenderError(f"undefined variable {name}")
            return _path(vars_[name], rest)
        if k == "ident":
            if v in ("true", "false"):
                return v == "true"
            if v == "nil":
                return None
            return _FuncRef(v)
        raise RenderError(f"unexpected token {v!r}")

    def _command(self, toks: List[Tuple[str, str]], dot: Any, vars_: Dict[str, Any], piped: Any) -> Any:
        if not toks:
            raise RenderError("empty command")
        if toks[0][0] == "ident" and toks[0][1] not in ("true", "false", "nil"):
            name = toks[0][1]
            args = self._args(toks[1:], dot, vars_)
            if piped is not _NOARG:
                args.append(piped)
            return self._call(name, args, dot)
        vals = self._args(toks, dot, vars_)
        if len(vals) != 1 or piped is not _NOARG:
            raise RenderError(f"cannot evaluate {toks!r}")
        return vals[0]

    def _call(self, name: str, a: List[Any], dot: Any) -> Any:
        if name == "include":
            tname, ctx = a[0], a[1] if len(a) > 1 else None
            if tname not in self.defines:
                raise RenderError(f"no template {tname!r}")
            return self._run(self.defines[tname], ctx, {"$": self.root})
        f = FUNCS.get(name)
        if f is None:
            if name == "lookup":
                return copy.deepcopy(self.lookup_fn(*a)) or {}
            raise RenderError(f"unknown function {name}")
        return f(*a)


class _FuncRef(str):
    pass


_NOARG = object()
_NOOUT = object()


def _path(v: Any, path: str) -> Any:
    for p in [x for x in path.split(".") if x]:
        if v is None:
            return None
        v = v.get(p) if isinstance(v, dict) else getattr(v, p, None)
    return v


def _fmt(v: Any) -> str:
    if v is None:
        return "<no value>"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, (dict, list)):
        return json.dumps(v)  # Go prints maps as map[...]; the chart never does this
    return str(v)


def _indent(n: int, s: str) -> str:
    pad = " " * int(n)
    return "\n".join(pad + line if line else line for line in str(s).split("\n"))


def _default(d: Any, v: Any = _NOARG) -> Any:
    if v is _NOARG:
        return d
    return v if truthy(v) else d


def _fail(msg: str) -> Any:
    raise Fail(msg)


def _required(msg: str, v: Any) -> Any:
    if not truthy(v):
        raise Fail(msg)
    return v


def _dict(*kv: Any) -> Dict[str, Any]:
    return {str(kv[i]): kv[i + 1] for i in range(0, len(kv), 2)}


def _set(d: Dict[str, Any], k: str, v: Any) -> Dict[str, Any]:
    d[k] = v
    return d


def _index(c: Any, *keys: Any) -> Any:
    for k in keys:
        if c is None:
            return None
        c = c.get(k) if isinstance(c, dict) else c[int(k)]
    return c


FUNCS: Dict[str, Callable[..., Any]] = {
    "toYaml": to_yaml, "nindent": lambda n, s: "\n" + _indent(n, s), "indent": _indent,
    "quote": lambda *v: " ".join(json.dumps(_fmt(x)) for x in v), "default": _default,
    "eq": lambda a, *b: any(a == x for x in b), "ne": lambda a, b: a != b, "lt": lambda a, b: a < b,
    "gt": lambda a, b: a > b, "not": lambda v: not truthy(v),
    "and": lambda *v: next((x for x in v if not truthy(x)), v[-1]),
    "or": lambda *v: next((x for x in v if truthy(x)), v[-1]),
    "hasPrefix": lambda p, s: str(s).startswith(p), "hasSuffix": lambda p, s: str(s).endswith(p),
    "dict": _dict, "list": lambda *v: list(v), "append": lambda lst, v: list(lst or []) + [v], "set": _set,
    "index": _index, "uuidv4": lambda: str(uuid.uuid4()),
    "sha256sum": lambda s: hashlib.sha256(str(s).encode()).hexdigest(),
    "print": lambda *v: "".join(_fmt(x) for x in v), "printf": lambda f, *v: f.replace("%s", "{}").format(*v),
    "fail": _fail, "required": _required, "trim": lambda s: str(s).strip(), "toString": _fmt,
    "empty": lambda v: not truthy(v), "int": lambda v: int(v), "len": lambda v: len(v or []),
}


def _merge(base: Dict[str, Any], over: Dict[str, Any]) -> Dict[str, Any]:
    out = copy.deepcopy(base)
    for k, v in over.items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = _merge(out[k], v)
        else:
            out[k] = v
    return out


def set_path(values: Dict[str, Any], dotted: str, v: Any) -> Dict[str, Any]:
    cur = values
    parts = dotted.split(".")
    for p in parts[:-1]:
        cur = cur.setdefault(p, {})
    cur[parts[-1]] = v
    return values


def main(argv: List[str]) -> int:
    chart = argv[0] if argv else "helm-charts/nos"
    ns = argv[argv.index("--namespace") + 1] if "--namespace" in argv else "nos-system"
    vals: Dict[str, Any] = {}
    for i, a in enumerate(argv):
        if a == "--set":
            k, _, v = argv[i + 1].partition("=")
            set_path(vals, k, yaml.safe_load(v))
    for rel, text in Chart(chart, vals, namespace=ns).render().items():
        if text.strip():
            print(f"---\n# Source: {rel}\n{text.strip()}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
