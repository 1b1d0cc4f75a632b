"""Geometry-partitioned GPU and node: the planning core shared by every "fixed geometry" backend.

Behaviour reproduced from ``pkg/gpu/mig/gpu.go:29-315`` and ``pkg/gpu/mig/node.go:26-222``
(SURVEY Appendix B.1-B.3), parameterised by the allowed-geometry table so that the MI355X
compute-partition table (``xcp``) is the production instance while the reference's MIG tables
can be loaded in tests to check behavioural parity of the search itself:

* ``can_apply_geometry``: allowed, and never fewer slices than are in use for any profile;
* ``update_geometry_for``: scored search over allowed geometries — provided profiles desc,
  total slices desc, L1 distance to the current geometry asc, geometry id asc;
* ``apply_geometry``: free = geometry - used; free profiles absent from the geometry dropped;
* ``init_geometry``: fewest *distinct* profiles, first wins ties;
* node ``update_geometry_for``: greedy over GPUs in index order, subtracting each GPU's free
  slices from the remaining demand.

On MI355X every allowed geometry is homogeneous, so "never shrink used" automatically forbids
flipping the mode of a GPU that has any partition in use (a flip destroys every partition).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Callable, Dict, List, Mapping, Optional, Tuple

from .geometry import (Geometry, geometry_distance, geometry_id, geometries_equal,
                       get_fewest_slices_geometry, total_slices)


@dataclass
class PartitionedGPU:
    model: str
    index: int
    allowed_geometries: List[Geometry]
    used: Dict[str, int] = field(default_factory=dict)
    free: Dict[str, int] = field(default_factory=dict)
    #: desired geometry when the spec asks for a different one than the GPU has while partitions
    #: are still in use: the GPU is *draining* — no new pod is placed on it, and it flips to
    #: ``target`` as soon as it is idle (MI355X: a flip destroys every partition)
    target: Optional[Dict[str, int]] = None
    #: the drain target is a sliced layout (SPX + CU-mask slices, ``models/xcp/slices.py``)
    target_sliced: bool = False
    #: why the agent's probe found a partition/slice of this GPU below its model's expected rate
    #: ("" = healthy or not probed): the planner places new work on other GPUs first
    degraded: str = ""

    #: served as CU-mask slices of an SPX GPU (``SlicedGPU``) rather than hardware partitions
    sliced = False

    def clone(self) -> "PartitionedGPU":
        return PartitionedGPU(self.model, self.index, [dict(g) for g in self.allowed_geometries],
                              dict(self.used), dict(self.free), dict(self.target) if self.target else None,
                              self.target_sliced, self.degraded)

    def spec_geometry(self) -> Geometry:
        """What the spec should say for this GPU: the drain target, else the geometry."""
        return dict(self.target) if self.target else self.geometry()

    def spec_sliced(self) -> bool:
        """Whether the spec asks for this GPU as slices (the drain target's layout, else its own)."""
        return self.target_sliced if self.target else self.sliced

    def geometry(self) -> Geometry:
        out: Geometry = {}
        for d in (self.used, self.free):
            for p, q in d.items():
                out[p] = out.get(p, 0) + q
        return out

    def allows_geometry(self, g: Mapping[str, int]) -> bool:
        return any(geometries_equal(g, a) for a in self.allowed_geometries)

    def can_apply_geometry(self, g: Mapping[str, int]) -> Tuple[bool, str]:
        if not self.allows_geometry(g):
            return False, f"GPU model {self.model} does not allow the provided geometry"
        for p, q in self.used.items():
            if g.get(p, 0) < q:
                return False, "cannot apply geometry: cannot delete partitions being used"
        return True, ""

    def apply_geometry(self, g: Mapping[str, int]) -> None:
        ok, reason = self.can_apply_geometry(g)
        if not ok:
            raise ValueError(reason)
        for p, q in g.items():
            self.free[p] = q - self.used.get(p, 0)
        for p in list(self.free):
            if p not in g:
                del self.free[p]

    def init_geometry(self) -> None:
        g = get_fewest_slices_geometry(self.allowed_geometries)
        if g is None:
            raise ValueError("no allowed geometries")
        self.apply_geometry(g)

    def _provided(self, candidate: Mapping[str, int], required: Mapping[str, int], current: Mapping[str, int],
                  weight: Optional[Callable[[str], float]] = None) -> float:
        provided = 0.0
        for p, rq in required.items():
            fr = self.free.get(p, 0)
            if fr >= rq:
                continue
            needed = rq - fr
            extra = candidate.get(p, 0) - current.get(p, 0)
            if extra <= 0:
                continue
            provided += min(extra, needed) * (1.0 if weight is None else weight(p))
        return provided

    def update_geometry_for(self, required: Mapping[str, int], weight: Optional[Callable[[str], float]] = None) -> bool:
        """B.1.  ``weight`` scores each provided profile (None = count pods, the reference score;
        the MI355X planner passes the GPU fraction of the profile so that a free GPU is flipped to
        the mode that puts the most *capacity* to use, not the most pods)."""
        current = self.geometry()
        best: Optional[Geometry] = None
        best_score: Optional[Tuple[float, int, int, str]] = None
        for cand in self.allowed_geometries:
            if not self.can_apply_geometry(cand)[0]:
                continue
            provided = self._provided(cand, required, current, weight)
            if provided <= 0:
                continue
            # higher is better: provided desc, slices desc, distance asc, id asc
            score = (provided, total_slices(cand), -geometry_distance(current, cand), geometry_id(cand))
            if best_score is None or _better(score, best_score):
                best, best_score = dict(cand), score
        if best is None:
            return False
        self.apply_geometry(best)
        return True

    def add_pod(self, requested: Mapping[str, int]) -> None:
        if self.target is not None:
            raise ValueError(f"GPU {self.index} is draining towards {self.target}")
        for p, q in requested.items():
            if self.free.get(p, 0) < q:
                raise ValueError(f"not enough free partitions (pod requests {q} {p}, but GPU only has "
                                 f"{self.free.get(p, 0)})")
        for p, q in requested.items():
            self.free[p] -= q
            self.used[p] = self.used.get(p, 0) + q

    def has_free_devices(self) -> bool:
        return any(q > 0 for q in self.free.values())

    def is_idle(self) -> bool:
        return not any(q > 0 for q in self.used.values())

    def used_fraction(self, partitions_of: Callable[[str], int]) -> float:
        return sum(q / partitions_of(p) for p, q in self.used.items())


def _better(a: Tuple[float, int, int, str], b: Tuple[float, int, int, str]) -> bool:
    if a[0] != b[0]:
        return a[0] > b[0]
    if a[1] != b[1]:
        return a[1] > b[1]
    if a[2] != b[2]:
        return a[2] > b[2]
    return a[3] < b[3]


@dataclass
class PartitionedNode:
    name: str
    gpus: List[PartitionedGPU]
    allocatable: Dict[str, int] = field(default_factory=dict)
    is_resource: Callable[[str], bool] = lambda r: False
    as_resource: Callable[[str], str] = lambda p: p
    weight: Optional[Callable[[str], float]] = None
    #: node-wide memory-partition mode (MI355X NPS, e.g. "nps1"): observed, and the one a plan
    #: switches the node to (every GPU of the node re-partitioned, only when all are idle)
    memory_partition: Optional[str] = None
    memory_target: Optional[str] = None
    #: xcp layout of the node (``partitions`` | ``slices`` | ``auto``, ``models/xcp/slices.py``)
    layout: str = "partitions"

    def clone(self) -> "PartitionedNode":
        return PartitionedNode(self.name, [g.clone() for g in self.gpus], dict(self.allocatable),
                               self.is_resource, self.as_resource, self.weight, self.memory_partition,
                               self.memory_target, self.layout)

    def geometry(self) -> Geometry:
        out: Geometry = {}
        for g in self.gpus:
            for p, q in g.geometry().items():
                out[p] = out.get(p, 0) + q
        return out

    def free(self) -> Geometry:
        out: Geometry = {}
        for g in self.gpus:
            for p, q in g.free.items():
                out[p] = out.get(p, 0) + q
        return out

    def has_free_capacity(self) -> bool:
        if not self.gpus:
            return False
        for g in self.gpus:
            if g.has_free_devices():
                return True
            if not g.allows_geometry(g.geometry()):
                return True
        return False

    def update_geometry_for(self, required: Mapping[str, int]) -> bool:
        if not self.gpus or not required:
            return False
        remaining = dict(required)
        any_updated = False
        for g in self.gpus:
            updated = g.update_geometry_for(remaining, self.weight)
            any_updated = any_updated or updated
            for p, q in g.free.items():
                if p in remaining:
                    remaining[p] -= q
                    if remaining[p] <= 0:
                        del remaining[p]
        self.allocatable = self._scalar_resources()
        return any_updated

    def _scalar_resources(self) -> Dict[str, int]:
        res = {r: v for r, v in self.allocatable.items() if not self.is_resource(r)}
        for p, q in self.geometry().items():
            res[self.as_resource(p)] = q
        return res

    def add_pod(self, requested: Mapping[str, int]) -> None:
        for g in self.gpus:
            try:
                g.add_pod(requested)
                return
            except ValueError:
                continue
        raise ValueError("not enough free partitions")
