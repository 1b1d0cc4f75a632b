"""Event predicates (reference ``pkg/util/predicate/predicates.go:27-76``).

``NodeResourcesChanged`` in the reference returns *false* when Allocatable changed and true only
when Allocatable is equal but Capacity changed, so the reporters effectively rely on
their periodic requeue.  Here it fires when *either* changed.
"""
from __future__ import annotations

from typing import Any, Dict

from ..kube.runtime import Predicate

Obj = Dict[str, Any]


class MatchingName(Predicate):
    def __init__(self, name: str):
        self.name = name

    def create(self, obj: Obj) -> bool:
        return obj.get("metadata", {}).get("name") == self.name

    def update(self, old: Obj, new: Obj) -> bool:
        return old.get("metadata", {}).get("name") == self.name

    def delete(self, obj: Obj) -> bool:
        return obj.get("metadata", {}).get("name") == self.name


class NodeResourcesChanged(Predicate):
    def update(self, old: Obj, new: Obj) -> bool:
        o, n = old.get("status", {}), new.get("status", {})
        return o.get("allocatable") != n.get("allocatable") or o.get("capacity") != n.get("capacity")


class AnnotationsChanged(Predicate):
    def update(self, old: Obj, new: Obj) -> bool:
        return (old.get("metadata", {}).get("annotations") or {}) != (new.get("metadata", {}).get("annotations") or {})


class LabelsChanged(Predicate):
    def update(self, old: Obj, new: Obj) -> bool:
        return (old.get("metadata", {}).get("labels") or {}) != (new.get("metadata", {}).get("labels") or {})


class ExcludeDelete(Predicate):
    def delete(self, obj: Obj) -> bool:
        return False


class HasLabel(Predicate):
    """Object carries the label (any value) — the node controller's label-exists predicate."""

    def __init__(self, key: str):
        self.key = key

    def _has(self, obj: Obj) -> bool:
        return self.key in (obj.get("metadata", {}).get("labels") or {})

    def create(self, obj: Obj) -> bool:
        return self._has(obj)

    def update(self, old: Obj, new: Obj) -> bool:
        return self._has(new)

    def delete(self, obj: Obj) -> bool:
        return self._has(obj)


class Or(Predicate):
    def __init__(self, *ps: Predicate):
        self.ps = ps

    def create(self, obj: Obj) -> bool:
        return any(p.create(obj) for p in self.ps)

    def update(self, old: Obj, new: Obj) -> bool:
        return any(p.update(old, new) for p in self.ps)

    def delete(self, obj: Obj) -> bool:
        return any(p.delete(obj) for p in self.ps)
