"""Compute-partition node model: a :class:`PartitionedNode` built from a Node object.

Reference ``pkg/gpu/mig/node.go:40-100`` builds GPUs from the status annotations grouped by index
and then appends empty GPUs for the *count* of missing ones starting at ``len(annotated)`` —
which silently assumes annotated indexes are ``0..n-1``.  Here missing indexes are filled exactly.
The allowed geometries are the model's geometries for the node's current NPS mode.
"""
from __future__ import annotations

from typing import Any, Dict, List, Mapping, Optional

from ...api import v1alpha1 as api
from ...kube import objects as ko
from .. import annotation as ann
from .. import gpu_util
from .. import resource as res
from ..defaults import LIBRARY_DEFAULTS, ModelDefaults
from ..partitioned import PartitionedGPU, PartitionedNode
from .known_configs import get_allowed_geometries
from .profile import as_resource_name, extract_profile_name, is_xcp_resource
from .slices import LAYOUT_PARTITIONS, LAYOUT_SLICES, LAYOUTS, SLICE_NPS, new_sliced_gpu, parse_gpu_set


def new_gpu(model: str, index: int, nps: str, used: Mapping[str, int] | None = None,
            free: Mapping[str, int] | None = None) -> PartitionedGPU:
    allowed = get_allowed_geometries(model, nps)
    if allowed is None:
        raise ValueError(f"model {model!r} is not associated with any known GPU")
    return PartitionedGPU(model, index, allowed, dict(used or {}), dict(free or {}))


def fraction_weight(profile: str) -> float:
    from .profile import parse_profile
    return 1.0 / parse_profile(profile).partitions


SCORING = {"pods": None, "fraction": fraction_weight}


def get_layout(node: Dict[str, Any], default: str = LAYOUT_PARTITIONS) -> str:
    """The node's ``nos.nebuly.com/xcp-layout`` (absent: ``default`` — the owning planner's
    ``ModelDefaults.xcp_layout``; unknown values: hardware partitions only). Slices need NPS1 (a
    sliced GPU is in SPX, which other memory modes do not offer)."""
    if default not in LAYOUTS:
        raise ValueError(f"unknown xcp layout {default!r}")
    v = (ko.labels(node).get(api.LABEL_XCP_LAYOUT) or default).lower()
    if v not in LAYOUTS or gpu_util.get_memory_partition(node) != SLICE_NPS:
        return LAYOUT_PARTITIONS
    return v


def degraded_gpus(annotations: Mapping[str, str]) -> Dict[int, str]:
    """GPU index -> the first degraded probe reason of the agent's ``status-probe`` annotation."""
    import json
    try:
        doc = json.loads(annotations.get(api.ANNOTATION_PROBE_RESULT) or "{}")
    except ValueError:
        return {}
    out: Dict[int, str] = {}
    for label, r in sorted((doc.get("slices") or {}).items()):
        if isinstance(r, dict) and r.get("degraded") and isinstance(r.get("gpu"), int):
            out.setdefault(r["gpu"], f"{label}: {r['degraded']}")
    return out


def new_node(node: Dict[str, Any], scoring: str = "fraction", defaults: Optional[ModelDefaults] = None) -> PartitionedNode:
    """The node's model; an unlabeled node takes ``defaults.xcp_layout`` (the planner's; none given:
    the library default, hardware partitions)."""
    defaults = defaults or LIBRARY_DEFAULTS
    model = gpu_util.get_model(node)
    count = gpu_util.get_count(node)
    nps = gpu_util.get_memory_partition(node)
    anns = ko.annotations(node)
    status, spec = ann.parse_node_annotations(anns)
    layout = get_layout(node, defaults.xcp_layout)
    sliced_now = parse_gpu_set(anns.get(api.ANNOTATION_SLICED_GPUS_STATUS)) if layout != LAYOUT_PARTITIONS else set()
    sliced_spec = parse_gpu_set(anns.get(api.ANNOTATION_SLICED_GPUS_SPEC))
    gpus: Dict[int, PartitionedGPU] = {}
    spec_by_gpu: Dict[int, Dict[str, int]] = {}
    for a in spec:
        spec_by_gpu.setdefault(a.index, {})[a.profile] = spec_by_gpu.get(a.index, {}).get(a.profile, 0) + a.quantity
    for idx, items in sorted(ann.group_by_gpu_index(status).items()):
        used = {a.profile: a.quantity for a in items if a.is_used()}
        free = {a.profile: a.quantity for a in items if a.is_free()}
        sliced = idx in sliced_now
        gpus[idx] = new_sliced_gpu(model, idx, used, free) if sliced else new_gpu(model, idx, nps, used, free)
        want = {p: q for p, q in spec_by_gpu.get(idx, {}).items() if q > 0}
        want_sliced = idx in sliced_spec
        busy = any(q > 0 for q in used.values())
        if want and (want != gpus[idx].geometry() or want_sliced != sliced) and (busy or (sliced and want_sliced)):
            # a change the agent cannot apply until the GPU drains; on a sliced GPU also when idle:
            # a reservation spec that no longer matches what is in use is replanned, never left in
            # place (the plugin withholds the GPU for as long as the spec says so)
            gpus[idx].target = want
            gpus[idx].target_sliced = want_sliced
    for i in range(count):
        if i not in gpus:
            # a GPU nothing is reported for yet (a fresh node): in SPX, sliced on a slices node
            gpus[i] = new_sliced_gpu(model, i) if layout == LAYOUT_SLICES else new_gpu(model, i, nps)
    # a node-wide memory-partition switch in progress (spec NPS != observed): every GPU is
    # re-partitioned, idle ones included, so none is offered to new pods until the switch lands
    spec_nps = gpu_util.get_spec_memory_partition(node)
    switching = spec_nps if spec_nps and spec_nps != nps else None
    if switching:
        for idx, g in gpus.items():
            want = {p: q for p, q in spec_by_gpu.get(idx, {}).items() if q > 0}
            if want and g.target is None and want != g.geometry():
                g.target = want
    for idx, why in degraded_gpus(anns).items():
        if idx in gpus:
            gpus[idx].degraded = why
    allocatable = res.from_k8s(ko.node_allocatable(node))
    return PartitionedNode(ko.name(node), [gpus[i] for i in sorted(gpus)], allocatable,
                           is_resource=is_xcp_resource, as_resource=as_resource_name, weight=SCORING[scoring],
                           memory_partition=nps, memory_target=switching, layout=layout)


def get_requested_profiles(pod: Dict[str, Any]) -> Dict[str, int]:
    """Compute-partition profiles requested by a pod (reference ``GetRequestedProfiles``)."""
    out: Dict[str, int] = {}
    for r, q in res.compute_pod_request(pod).items():
        p = extract_profile_name(r)
        if p is not None and q > 0:
            out[p] = out.get(p, 0) + q
    return out


def requested_profiles_list(pods: List[Dict[str, Any]]) -> Dict[str, int]:
    out: Dict[str, int] = {}
    for p in pods:
        for k, v in get_requested_profiles(p).items():
            out[k] = out.get(k, 0) + v
    return out
