"""Helpers over Kubernetes objects represented as JSON-shaped ``dict``s.

Objects are kept in exactly the wire shape the API server speaks (``apiVersion``, ``kind``,
``metadata``, ``spec``, ``status``) so the same controller code runs against the in-memory
API server (:mod:`walkai_nos_amd.kube.memory`) and a real cluster
(:mod:`walkai_nos_amd.kube.rest`).
"""
from __future__ import annotations

import functools

import copy
import datetime as _dt
from typing import Any, Dict, Iterable, List, Optional, Tuple

Obj = Dict[str, Any]


def deepcopy(o: Obj) -> Obj:
    return copy.deepcopy(o)


def meta(o: Obj) -> Dict[str, Any]:
    return o.setdefault("metadata", {})


def name(o: Obj) -> str:
    return o.get("metadata", {}).get("name", "")


def namespace(o: Obj) -> str:
    return o.get("metadata", {}).get("namespace", "") or ""


def key(o: Obj) -> Tuple[str, str]:
    return (namespace(o), name(o))


def labels(o: Obj) -> Dict[str, str]:
    return o.get("metadata", {}).get("labels") or {}


def annotations(o: Obj) -> Dict[str, str]:
    return o.get("metadata", {}).get("annotations") or {}


def set_label(o: Obj, k: str, v: str) -> None:
    meta(o).setdefault("labels", {})[k] = v


def set_annotation(o: Obj, k: str, v: str) -> None:
    meta(o).setdefault("annotations", {})[k] = v


def resource_version(o: Obj) -> str:
    return o.get("metadata", {}).get("resourceVersion", "")


def now_rfc3339(ts: Optional[float] = None) -> str:
    if ts is None:
        d = _dt.datetime.now(_dt.timezone.utc)
    else:
        d = _dt.datetime.fromtimestamp(ts, _dt.timezone.utc)
    return d.strftime("%Y-%m-%dT%H:%M:%SZ")


def parse_rfc3339(s: Optional[str]) -> Optional[_dt.datetime]:
    if not s:
        return None
    s = s.replace("Z", "+00:00")
    return _dt.datetime.fromisoformat(s)


# ---- Node helpers -------------------------------------------------------------------
def node_allocatable(node: Obj) -> Dict[str, Any]:
    return node.get("status", {}).get("allocatable") or {}


def node_capacity(node: Obj) -> Dict[str, Any]:
    return node.get("status", {}).get("capacity") or {}


# ---- Pod helpers --------------------------------------------------------------------
def pod_phase(pod: Obj) -> str:
    return pod.get("status", {}).get("phase", "")


def pod_node_name(pod: Obj) -> str:
    return pod.get("spec", {}).get("nodeName", "") or ""


def pod_conditions(pod: Obj) -> List[Dict[str, Any]]:
    return pod.get("status", {}).get("conditions") or []


def get_condition(pod: Obj, ctype: str) -> Optional[Dict[str, Any]]:
    for c in pod_conditions(pod):
        if c.get("type") == ctype:
            return c
    return None


def set_condition(pod: Obj, ctype: str, status: str, reason: str = "", message: str = "") -> None:
    conds = pod.setdefault("status", {}).setdefault("conditions", [])
    for c in conds:
        if c.get("type") == ctype:
            c.update(status=status, reason=reason, message=message)
            return
    conds.append({"type": ctype, "status": status, "reason": reason, "message": message})


def containers(pod: Obj) -> List[Dict[str, Any]]:
    return pod.get("spec", {}).get("containers") or []


def init_containers(pod: Obj) -> List[Dict[str, Any]]:
    return pod.get("spec", {}).get("initContainers") or []


def owner_kinds(o: Obj) -> Iterable[str]:
    for ref in o.get("metadata", {}).get("ownerReferences") or []:
        yield ref.get("kind", "")


def match_labels(selector: Optional[Dict[str, str]], lbls: Dict[str, str]) -> bool:
    if not selector:
        return True
    return all(lbls.get(k) == v for k, v in selector.items())


@functools.lru_cache(maxsize=1024)
def parse_label_selector(sel: str) -> Tuple[Tuple[str, str, Optional[str]], ...]:
    """Parse ``a=b,c!=d,e`` (equality-based + existence) selectors (memoised: controllers reuse a
    handful of selector strings on every list)."""
    return tuple(_parse_label_selector(sel))


def _parse_label_selector(sel: str) -> List[Tuple[str, str, Optional[str]]]:
    out: List[Tuple[str, str, Optional[str]]] = []
    for part in filter(None, (p.strip() for p in sel.split(","))):
        if "!=" in part:
            k, v = part.split("!=", 1)
            out.append((k.strip(), "!=", v.strip()))
        elif "==" in part:
            k, v = part.split("==", 1)
            out.append((k.strip(), "=", v.strip()))
        elif "=" in part:
            k, v = part.split("=", 1)
            out.append((k.strip(), "=", v.strip()))
        elif part.startswith("!"):
            out.append((part[1:].strip(), "!exists", None))
        else:
            out.append((part, "exists", None))
    return out


def selector_matches(sel: Optional[str], lbls: Dict[str, str]) -> bool:
    if not sel:
        return True
    for k, op, v in parse_label_selector(sel):
        if op == "=" and lbls.get(k) != v:
            return False
        if op == "!=" and lbls.get(k) == v:
            return False
        if op == "exists" and k not in lbls:
            return False
        if op == "!exists" and k in lbls:
            return False
    return True


def get_field(o: Obj, path: str) -> Any:
    cur: Any = o
    for p in path.split("."):
        if not isinstance(cur, dict):
            return None
        cur = cur.get(p)
    return cur


def field_selector_matches(sel: Optional[str], o: Obj) -> bool:
    if not sel:
        return True
    for k, op, v in parse_label_selector(sel):
        val = get_field(o, k)
        val = "" if val is None else str(val)
        if op == "=" and val != v:
            return False
        if op == "!=" and val == v:
            return False
    return True


def new_node(name_: str, labels_: Optional[Dict[str, str]] = None,
             annotations_: Optional[Dict[str, str]] = None,
             allocatable: Optional[Dict[str, Any]] = None,
             capacity: Optional[Dict[str, Any]] = None) -> Obj:
    return {
        "apiVersion": "v1",
        "kind": "Node",
        "metadata": {"name": name_, "labels": dict(labels_ or {}), "annotations": dict(annotations_ or {})},
        "spec": {},
        "status": {
            "allocatable": dict(allocatable or {}),
            "capacity": dict(capacity if capacity is not None else (allocatable or {})),
        },
    }


def new_pod(name_: str, namespace_: str = "default", requests: Optional[Dict[str, Any]] = None,
            labels_: Optional[Dict[str, str]] = None, scheduler_name: str = "default-scheduler",
            priority: int = 0, phase: str = "Pending", node_name: str = "",
            limits: Optional[Dict[str, Any]] = None) -> Obj:
    res: Dict[str, Any] = {}
    if requests:
        res["requests"] = {k: str(v) for k, v in requests.items()}
    if limits:
        res["limits"] = {k: str(v) for k, v in limits.items()}
    return {
        "apiVersion": "v1",
        "kind": "Pod",
        "metadata": {"name": name_, "namespace": namespace_, "labels": dict(labels_ or {}), "annotations": {}},
        "spec": {
            "schedulerName": scheduler_name,
            "priority": priority,
            "nodeName": node_name,
            "containers": [{"name": "main", "image": "workload", "resources": res}],
        },
        "status": {"phase": phase, "conditions": []},
    }
