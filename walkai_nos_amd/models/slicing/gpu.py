"""CU-mask slicing GPU and node models.

Reference: ``pkg/gpu/slicing/gpu.go:27-265`` and ``node.go:26-215``:
``Validate`` (each slice >= 1 GB, total <= GPU memory) and ``UpdateGeometryFor`` — process the
missing profiles smallest first; (1) create from spare capacity, (2) drop the *original* free
slices and create more, (3) try to restore the original free slices (all-or-nothing per
profile).  Generalised to two dimensions: HBM GB <= GPU memory and dedicated CUs <= CU count
(less :data:`MIN_SHARED_CUS` while memory-only slices exist), CU counts in multiples of
:data:`CU_GRANULARITY`.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, List, Mapping, Optional, Tuple

from ...kube import objects as ko
from .. import annotation as ann
from .. import gpu_util
from .. import resource as res
from ..defaults import LIBRARY_DEFAULTS, ModelDefaults
from ..geometry import Geometry
from . import profile as _profile
from .profile import (CU_GRANULARITY, MAX_SLICES_PER_GPU, MIN_SHARED_CUS, MIN_SLICE_MEMORY_GB, as_resource_name,
                      extract_profile_name, is_slice_resource, parse_profile)


@dataclass
class SlicingGPU:
    model: str
    index: int
    memory_gb: int
    cu_count: int = 256
    used: Dict[str, int] = field(default_factory=dict)
    free: Dict[str, int] = field(default_factory=dict)
    #: slices the planner may carve on this GPU (each serves one pod process; beyond 8 the hardware
    #: scheduler time-slices processes, :data:`~.profile.MAX_SLICES_PER_GPU`)
    max_slices: int = MAX_SLICES_PER_GPU
    #: memory-only slice counts never left on the GPU (None: :data:`~.profile.SKIP_SHARED_COUNTS`; a
    #: planner's node models carry its ``ModelDefaults.shared_skip_counts``)
    skip_shared: Optional[Tuple[int, ...]] = None

    @classmethod
    def full(cls, model: str, index: int, memory_gb: int, cu_count: int = 256,
             max_slices: int = MAX_SLICES_PER_GPU) -> "SlicingGPU":
        return cls(model, index, memory_gb, cu_count, max_slices=max_slices)

    def clone(self) -> "SlicingGPU":
        return SlicingGPU(self.model, self.index, self.memory_gb, self.cu_count, dict(self.used), dict(self.free),
                          self.max_slices, self.skip_shared)

    def validate(self) -> None:
        for d in (self.used, self.free):
            for p, q in d.items():
                prof = parse_profile(p)
                if prof.memory_gb < MIN_SLICE_MEMORY_GB:
                    raise ValueError(f"min allowed slice size is {MIN_SLICE_MEMORY_GB}GB, but profile {p} has "
                                     f"{prof.memory_gb}GB")
                if prof.cus % CU_GRANULARITY:
                    raise ValueError(f"profile {p}: CU count must be a multiple of {CU_GRANULARITY}")
        if self._tot_memory() > self.memory_gb:
            raise ValueError(f"total memory of profiles ({self._tot_memory()}) exceeds GPU memory ({self.memory_gb})")
        if self._tot_cus() > self._cu_budget():
            raise ValueError(f"total dedicated CUs ({self._tot_cus()}) exceed the GPU's CU budget ({self._cu_budget()})")

    def geometry(self) -> Geometry:
        out: Geometry = {}
        for d in (self.used, self.free):
            for p, q in d.items():
                out[p] = out.get(p, 0) + q
        return out

    def _tot_memory(self) -> int:
        return sum(parse_profile(p).memory_gb * q for p, q in self.geometry().items())

    def _tot_cus(self) -> int:
        return sum(parse_profile(p).cus * q for p, q in self.geometry().items())

    def _has_shared(self, extra_shared: bool = False) -> bool:
        return extra_shared or any(not parse_profile(p).dedicated and q > 0 for p, q in self.geometry().items())

    def _cu_budget(self, extra_shared: bool = False) -> int:
        return self.cu_count - (MIN_SHARED_CUS if self._has_shared(extra_shared) else 0)

    def spare_memory_gb(self) -> int:
        return self.memory_gb - self._tot_memory()

    def spare_cus(self) -> int:
        return self._cu_budget() - self._tot_cus()

    def slice_count(self) -> int:
        return sum(self.geometry().values())

    def shared_count(self) -> int:
        """Memory-only slices on the GPU (used and free)."""
        return sum(q for p, q in self.geometry().items() if not parse_profile(p).dedicated)

    def _skipped(self) -> Tuple[int, ...]:
        return _profile.SKIP_SHARED_COUNTS if self.skip_shared is None else self.skip_shared

    def can_create_more_slices(self) -> bool:
        return self.spare_memory_gb() >= MIN_SLICE_MEMORY_GB and self.slice_count() < self.max_slices

    def can_create(self, profile: str, num: int = 1) -> bool:
        """Whether ``num`` more slices of ``profile`` fit (memory, CUs, the slice cap, skipped
        memory-only counts)."""
        return self._can_create(profile, num)

    def _can_create(self, profile: str, num: int = 1) -> bool:
        prof = parse_profile(profile)
        if self.spare_memory_gb() < prof.memory_gb * num or self.slice_count() + num > self.max_slices:
            return False
        if not prof.dedicated and self.shared_count() + num in self._skipped():
            return False
        budget = self._cu_budget(extra_shared=not prof.dedicated)
        return budget - self._tot_cus() >= prof.cus * num

    def create_slices(self, profile: str, num: int = 1) -> bool:
        if not self._can_create(profile, num):
            return False
        self.free[profile] = self.free.get(profile, 0) + num
        return True

    def has_free_capacity(self) -> bool:
        return bool(self.free) or self.can_create_more_slices()

    def add_pod(self, requested: Mapping[str, int]) -> None:
        for p, q in requested.items():
            if self.free.get(p, 0) < q:
                raise ValueError(f"not enough free slices (pod requests {q} {p}, but GPU only has {self.free.get(p, 0)})")
        for p, q in requested.items():
            self.free[p] -= q
            if self.free[p] == 0:
                del self.free[p]
            self.used[p] = self.used.get(p, 0) + q

    def missing_slices(self, required: Mapping[str, int]) -> Dict[str, int]:
        out = {}
        for p, q in required.items():
            d = q - self.free.get(p, 0)
            if d > 0:
                out[p] = d
        return out

    def _create_step(self, profile: str, missing: int) -> int:
        """Create one slice of ``profile``, or two at once when one would leave a skipped
        memory-only count and two are missing; the number created."""
        if self.create_slices(profile, 1):
            return 1
        if missing >= 2 and not parse_profile(profile).dedicated and self.create_slices(profile, 2):
            return 2
        return 0

    def update_geometry_for(self, required: Mapping[str, int]) -> bool:
        missing = self.missing_slices(required)
        if not missing:
            return False
        updated = False
        original_free = dict(self.free)
        for p in sorted(missing, key=lambda x: parse_profile(x)):
            # (1) spare capacity first
            if self.can_create_more_slices():
                while missing[p] > 0:
                    n = self._create_step(p, missing[p])
                    if not n:
                        break
                    missing[p] -= n
                    updated = True
            # (2) free up room by deleting the original free slices
            for k in original_free:
                self.free.pop(k, None)
            while missing[p] > 0 and self.can_create_more_slices():
                n = self._create_step(p, missing[p])
                if not n:
                    break
                missing[p] -= n
                updated = True
            # (3) restore the original free slices (all-or-nothing per profile)
            for k, v in original_free.items():
                self.create_slices(k, v)
        return updated


@dataclass
class SlicingNode:
    name: str
    gpus: List[SlicingGPU]
    allocatable: Dict[str, int] = field(default_factory=dict)

    def clone(self) -> "SlicingNode":
        return SlicingNode(self.name, [g.clone() for g in self.gpus], dict(self.allocatable))

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
        return any(g.has_free_capacity() for g in self.gpus)

    def update_geometry_for(self, required: Mapping[str, int]) -> bool:
        if not self.gpus or not required:
            return False
        remaining = dict(required)
        any_updated = False
        for g in self.gpus:
            if not remaining:
                break
            updated = g.update_geometry_for(remaining)
            any_updated = any_updated or updated
            for p, q in g.free.items():
                if p in remaining:
                    remaining[p] -= q
                    if remaining[p] <= 0:
                        del remaining[p]
        res_ = {r: v for r, v in self.allocatable.items() if not is_slice_resource(r)}
        for p, q in self.geometry().items():
            res_[as_resource_name(p)] = q
        self.allocatable = res_
        return any_updated

    def add_pod(self, requested: Mapping[str, int]) -> None:
        for g in self.gpus:
            try:
                g.add_pod(requested)
                return
            except ValueError:
                continue
        raise ValueError("not enough free slices")


def new_node(node: Dict[str, Any], defaults: Optional[ModelDefaults] = None) -> SlicingNode:
    """Reference ``slicing.NewNode`` (node.go:48-105): also needs the GPU memory label. Every GPU
    carries ``defaults.shared_skip_counts`` (the owning planner's; none given: the library default)."""
    skip = (defaults or LIBRARY_DEFAULTS).shared_skip_counts
    model = gpu_util.get_model(node)
    count = gpu_util.get_count(node)
    mem = gpu_util.get_memory_gb(node)
    cus = gpu_util.get_cu_count(node)
    cap = max_slices_per_gpu(node)
    status, _ = ann.parse_node_annotations(ko.annotations(node))
    gpus: Dict[int, SlicingGPU] = {}
    for idx, items in sorted(ann.group_by_gpu_index(status).items()):
        used = {a.profile: a.quantity for a in items if a.is_used()}
        free = {a.profile: a.quantity for a in items if a.is_free()}
        g = SlicingGPU(model, idx, mem, cus, used, free, cap, skip)
        g.validate()
        gpus[idx] = g
    for i in range(count):
        if i not in gpus:
            gpus[i] = SlicingGPU(model, i, mem, cus, max_slices=cap, skip_shared=skip)
    return SlicingNode(ko.name(node), [gpus[i] for i in sorted(gpus)], res.from_k8s(ko.node_allocatable(node)))


def max_slices_per_gpu(node: Dict[str, Any]) -> int:
    """The node's ``nos.nebuly.com/max-slices-per-gpu`` label (a positive integer), else the default."""
    from ...api.v1alpha1 import LABEL_MAX_SLICES_PER_GPU
    v = ko.labels(node).get(LABEL_MAX_SLICES_PER_GPU)
    try:
        n = int(v) if v is not None else MAX_SLICES_PER_GPU
    except ValueError:
        return MAX_SLICES_PER_GPU
    return n if n > 0 else MAX_SLICES_PER_GPU


def get_requested_profiles(pod: Dict[str, Any]) -> Dict[str, int]:
    out: Dict[str, int] = {}
    for r, q in res.compute_pod_request(pod).items():
        p = extract_profile_name(r)
        if p is not None and q > 0:
            out[p] = out.get(p, 0) + q
    return out
