"""Cluster-side partitioning: spec writer, node initializer, plan IDs, node-partitioning builder.

Reference:
* ``internal/partitioning/mig/partitioner.go:40-91`` — drop every ``spec-gpu*`` annotation, write
  one ``spec-gpu-<i>-<profile>=<qty>`` per (GPU, profile) plus ``spec-partitioning-plan``, send a
  JSON merge patch computed against the original object;
* ``initializer.go:40-79`` — GPUs with an empty geometry get the fewest-slices geometry, then the
  partitioning is applied with a fresh plan ID;
* ``state.go:25-45`` — node model -> ``NodePartitioning``;
* ``plan.go:24-26`` — plan ID = UTC UnixNano as a string.
"""
from __future__ import annotations

import itertools
import logging
import time
from typing import Any, Callable, Dict, Optional, Union

from ..api import v1alpha1 as api
from ..kube import objects as ko
from ..kube.memory import create_merge_patch
from ..models.partitioned import PartitionedNode
from ..models.slicing.gpu import SlicingNode
from ..utils.metrics import REGISTRY
from .state import GPUPartitioning, NodePartitioning

log = logging.getLogger("nos.partitioning")

_last_id = [0]


def new_plan_id(clock: Callable[[], float] = time.time) -> str:
    """UnixNano of ``clock()``; strictly increasing within the process even on a coarse or
    virtual clock (two plans in the same nanosecond would otherwise collide)."""
    t = int(clock() * 1e9)
    if t <= _last_id[0]:
        t = _last_id[0] + 1
    _last_id[0] = t
    return str(t)


def build_node_partitioning(node: Union[PartitionedNode, SlicingNode], memory_partition: Optional[str] = None) -> NodePartitioning:
    as_res = node.as_resource if isinstance(node, PartitionedNode) else None
    gpus = []
    for g in node.gpus:
        resources: Dict[str, int] = {}
        geo = g.spec_geometry() if hasattr(g, "spec_geometry") else g.geometry()
        for p, q in geo.items():
            if q <= 0:
                continue
            r = as_res(p) if as_res is not None else _slice_resource(p)
            resources[r] = resources.get(r, 0) + q
        sliced = g.spec_sliced() if hasattr(g, "spec_sliced") else False
        gpus.append(GPUPartitioning(g.index, resources, sliced))
    return NodePartitioning(gpus, memory_partition)


def _slice_resource(p: str) -> str:
    from ..models.slicing.profile import as_resource_name
    return as_resource_name(p)


def _profile_of(resource_name: str) -> Optional[str]:
    from ..models.slicing.profile import extract_profile_name as slice_profile
    from ..models.xcp.profile import extract_profile_name as xcp_profile
    return xcp_profile(resource_name) or slice_profile(resource_name)


def spec_annotations(partitioning: NodePartitioning) -> Dict[str, str]:
    out: Dict[str, str] = {}
    for g in partitioning.gpus:
        for r, q in sorted(g.resources.items()):
            p = _profile_of(r)
            if p is None:
                continue
            k = api.ANNOTATION_GPU_SPEC_FORMAT.format(index=g.gpu_index, profile=p)
            out[k] = str(int(out.get(k, "0")) + q)
    return out


class Partitioner:
    """Writes the desired partitioning of a node as spec annotations (C4)."""

    def __init__(self, client: Any):
        self.client = client

    def apply_partitioning(self, node: Dict[str, Any], plan_id: str, partitioning: NodePartitioning) -> Dict[str, Any]:
        t0 = time.perf_counter()
        original = ko.deepcopy(node)
        updated = ko.deepcopy(node)
        anns = ko.meta(updated).setdefault("annotations", {})
        for k in list(anns):
            if k.startswith(api.ANNOTATION_GPU_SPEC_PREFIX):
                del anns[k]
        anns.update(spec_annotations(partitioning))
        sliced = [g.gpu_index for g in partitioning.gpus if g.sliced]
        if sliced:
            from ..models.xcp.slices import format_gpu_set
            anns[api.ANNOTATION_SLICED_GPUS_SPEC] = format_gpu_set(sliced)
        else:
            anns.pop(api.ANNOTATION_SLICED_GPUS_SPEC, None)
        anns[api.ANNOTATION_PARTITIONING_PLAN] = plan_id
        if partitioning.memory_partition:
            anns[api.ANNOTATION_MEMORY_PARTITION_SPEC] = partitioning.memory_partition
        patch = create_merge_patch(original, updated)
        out = self.client.patch("Node", ko.name(node), patch)
        REGISTRY.phase_seconds.labels(phase="patch").observe(time.perf_counter() - t0)
        log.info("applied partitioning plan %s to node %s", plan_id, ko.name(node))
        return out


class NodeInitializer:
    """C5: initialise GPUs that have no geometry yet with the fewest-slices geometry."""

    def __init__(self, client: Any, partitioner: Optional[Partitioner] = None,
                 clock: Callable[[], float] = time.time, defaults: Any = None):
        self.client = client
        self.partitioner = partitioner or Partitioner(client)
        self.clock = clock
        self.defaults = defaults  # the planner's ModelDefaults (None: the library defaults)

    def init_node_partitioning(self, node: Dict[str, Any]) -> bool:
        from ..models.geometry import get_partitioning_kind
        from ..models.slicing import gpu as slicing_gpu
        from ..models.xcp import node as xcp_node

        kind = get_partitioning_kind(ko.labels(node))
        if kind == api.PARTITIONING_KIND_XCP:
            model = xcp_node.new_node(node, defaults=self.defaults)
            changed = False
            for g in model.gpus:
                if not g.geometry():
                    g.init_geometry()
                    changed = True
            if not changed:
                return False
            self.partitioner.apply_partitioning(node, new_plan_id(self.clock), build_node_partitioning(model))
            return True
        if kind == api.PARTITIONING_KIND_CUMASK:
            # a fresh CU-mask GPU has no slices: publish an explicit empty spec so the node counts as
            # initialised, i.e. every GPU index appears in the spec (one whole-GPU slice each)
            smodel = slicing_gpu.new_node(node, self.defaults)
            changed = False
            for g in smodel.gpus:
                if not g.geometry():
                    g.create_slices(f"{g.cu_count}cu.{g.memory_gb}gb", 1)
                    changed = True
            if not changed:
                return False
            self.partitioner.apply_partitioning(node, new_plan_id(self.clock), build_node_partitioning(smodel))
            return True
        return False


_counter = itertools.count()
