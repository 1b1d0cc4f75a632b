"""Resource math over ``{resource_name: int}`` maps.

Reference ``pkg/resource/resource.go:30-146``: ``Sum``, ``Subtract``, ``SubtractNonNegative``,
``Abs`` and ``ComputePodRequest`` = max(sum over containers, max over init containers) + overhead.
The reference computes the overhead sum and then discards it (``quota.Add`` returns a new list,
resource.go:139-141); here overhead is really added.

Values are integers: CPU in milli-cores (key ``cpu``), memory/ephemeral-storage in bytes,
extended resources as counts.  That mirrors ``framework.Resource``.
"""
from __future__ import annotations

from typing import Any, Dict, Iterable, Mapping

from ..kube import objects as ko
from ..kube.quantity import quantity_milli, quantity_value

ResourceList = Dict[str, int]


def to_int(name: str, q: Any) -> int:
    return quantity_milli(q) if name == "cpu" else quantity_value(q)


def from_k8s(rl: Mapping[str, Any] | None) -> ResourceList:
    return {k: to_int(k, v) for k, v in (rl or {}).items()}


def add(a: Mapping[str, int], b: Mapping[str, int]) -> ResourceList:
    out = dict(a)
    for k, v in b.items():
        out[k] = out.get(k, 0) + v
    return out


def sum_all(items: Iterable[Mapping[str, int]]) -> ResourceList:
    out: ResourceList = {}
    for it in items:
        out = add(out, it)
    return out


def subtract(a: Mapping[str, int], b: Mapping[str, int]) -> ResourceList:
    out = dict(a)
    for k, v in b.items():
        out[k] = out.get(k, 0) - v
    return out


def subtract_non_negative(a: Mapping[str, int], b: Mapping[str, int]) -> ResourceList:
    return {k: max(0, v) for k, v in subtract(a, b).items()}


def abs_(a: Mapping[str, int]) -> ResourceList:
    return {k: abs(v) for k, v in a.items()}


def max_(a: Mapping[str, int], b: Mapping[str, int]) -> ResourceList:
    out = dict(a)
    for k, v in b.items():
        out[k] = max(out.get(k, 0), v)
    return out


def less_equal(a: Mapping[str, int], b: Mapping[str, int], only: Iterable[str] | None = None) -> bool:
    keys = set(a) if only is None else set(only)
    return all(a.get(k, 0) <= b.get(k, 0) for k in keys)


def compute_pod_request(pod: Dict[str, Any]) -> ResourceList:
    cont: ResourceList = {}
    for c in ko.containers(pod):
        cont = add(cont, from_k8s((c.get("resources") or {}).get("requests")))
    init: ResourceList = {}
    for c in ko.init_containers(pod):
        init = max_(init, from_k8s((c.get("resources") or {}).get("requests")))
    overhead = pod.get("spec", {}).get("overhead")
    if overhead:
        cont = add(cont, from_k8s(overhead))
    return max_(cont, init)


def filter_prefix(rl: Mapping[str, int], prefix: str) -> ResourceList:
    return {k: v for k, v in rl.items() if k.startswith(prefix)}
