"""Default kube-scheduler Filter plugins for nos-scheduler.

The reference plugs ``CapacityScheduling`` into a full kube-scheduler profile (ref
``docs/en/docs/elastic-resource-quota/configuration.md:19-42``), so every default filter still
applies to ``schedulerName: nos-scheduler`` pods.  The scheduler here is a compact Python one, so
the filters that decide *where* a pod may land are reproduced with upstream semantics:

* ``NodeUnschedulable`` — ``spec.unschedulable`` nodes only take pods tolerating
  ``node.kubernetes.io/unschedulable:NoSchedule``;
* ``TaintToleration`` — every ``NoSchedule``/``NoExecute`` taint needs a matching toleration
  (``Equal``: key, value, effect; ``Exists``: key, effect; an empty key with ``Exists`` tolerates
  everything; an empty effect matches every effect); ``PreferNoSchedule`` never filters;
* ``NodeSelector`` — every ``spec.nodeSelector`` label must match exactly;
* ``NodeAffinity`` — ``requiredDuringSchedulingIgnoredDuringExecution``: the node must match at
  least one ``nodeSelectorTerm``, a term being the AND of its ``matchExpressions`` (``In``,
  ``NotIn``, ``Exists``, ``DoesNotExist``, ``Gt``, ``Lt``) and ``matchFields`` (``metadata.name``).

``NodeResourcesFit`` is the scheduler's own ``fits`` (extended resources included).
"""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple

Obj = Dict[str, Any]

FILTER_EFFECTS = ("NoSchedule", "NoExecute")
UNSCHEDULABLE_TAINT = {"key": "node.kubernetes.io/unschedulable", "effect": "NoSchedule"}


def tolerates(toleration: Obj, taint: Obj) -> bool:
    eff = toleration.get("effect") or ""
    if eff and eff != taint.get("effect"):
        return False
    op = toleration.get("operator") or "Equal"
    key = toleration.get("key") or ""
    if op == "Exists":
        return key == "" or key == taint.get("key")
    return key == taint.get("key") and (toleration.get("value") or "") == (taint.get("value") or "")


def taint_toleration(pod: Obj, node: Obj) -> Tuple[bool, str]:
    tols = pod.get("spec", {}).get("tolerations") or []
    for t in node.get("spec", {}).get("taints") or []:
        if t.get("effect") not in FILTER_EFFECTS:
            continue
        if not any(tolerates(tol, t) for tol in tols):
            return False, f"node(s) had untolerated taint {{{t.get('key')}: {t.get('value', '')}}}"
    return True, ""


def node_unschedulable(pod: Obj, node: Obj) -> Tuple[bool, str]:
    if not node.get("spec", {}).get("unschedulable"):
        return True, ""
    if any(tolerates(tol, UNSCHEDULABLE_TAINT) for tol in pod.get("spec", {}).get("tolerations") or []):
        return True, ""
    return False, "node(s) were unschedulable"


def node_selector(pod: Obj, node: Obj) -> Tuple[bool, str]:
    sel = pod.get("spec", {}).get("nodeSelector") or {}
    labels = node.get("metadata", {}).get("labels") or {}
    if all(labels.get(k) == v for k, v in sel.items()):
        return True, ""
    return False, "node(s) didn't match Pod's node selector"


def _expr_matches(expr: Obj, value: Optional[str], present: bool) -> bool:
    op = expr.get("operator")
    vals = expr.get("values") or []
    if op == "In":
        return present and value in vals
    if op == "NotIn":
        return not present or value not in vals
    if op == "Exists":
        return present
    if op == "DoesNotExist":
        return not present
    if op in ("Gt", "Lt"):
        try:
            v, ref = int(value or ""), int(vals[0])
        except (ValueError, IndexError):
            return False
        return present and (v > ref if op == "Gt" else v < ref)
    return False


def term_matches(term: Obj, node: Obj) -> bool:
    exprs = term.get("matchExpressions") or []
    fields = term.get("matchFields") or []
    if not exprs and not fields:
        return False  # an empty term matches no objects (upstream semantics)
    labels = node.get("metadata", {}).get("labels") or {}
    for e in exprs:
        k = e.get("key", "")
        if not _expr_matches(e, labels.get(k), k in labels):
            return False
    for f in fields:
        if f.get("key") != "metadata.name":
            return False
        if not _expr_matches(f, node.get("metadata", {}).get("name"), True):
            return False
    return True


def node_affinity(pod: Obj, node: Obj) -> Tuple[bool, str]:
    req = (((pod.get("spec", {}).get("affinity") or {}).get("nodeAffinity") or {})
           .get("requiredDuringSchedulingIgnoredDuringExecution"))
    if not req:
        return True, ""
    terms = req.get("nodeSelectorTerms") or []
    if any(term_matches(t, node) for t in terms):
        return True, ""
    return False, "node(s) didn't match Pod's node affinity/selector"


FILTERS = (("NodeUnschedulable", node_unschedulable), ("NodeSelector", node_selector),
           ("NodeAffinity", node_affinity), ("TaintToleration", taint_toleration))


def filter_node(pod: Obj, node: Obj) -> Tuple[bool, str]:
    """Run every default filter; (passed, reason of the first failure)."""
    for _, f in FILTERS:
        ok, why = f(pod, node)
        if not ok:
            return False, why
    return True, ""


def feasible_nodes(pod: Obj, nodes: List[Obj]) -> Tuple[List[Obj], Dict[str, int]]:
    """Nodes passing every filter, plus a count of failure reasons (for the Unschedulable message)."""
    out, reasons = [], {}
    for n in nodes:
        ok, why = filter_node(pod, n)
        if ok:
            out.append(n)
        else:
            reasons[why] = reasons.get(why, 0) + 1
    return out, reasons
