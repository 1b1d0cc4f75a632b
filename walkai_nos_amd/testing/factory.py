"""Fluent builders for Kubernetes objects (reference ``pkg/test/factory/core_factory.go``).

    node = NodeBuilder("n0").with_labels({...}).with_allocatable({"amd.com/gpu": 8}).build()
    pod = (PodBuilder("p", "ns").with_container(requests={"amd.com/cpx_nps1": 1})
           .unschedulable().with_priority(10).build())
"""
from __future__ import annotations

import copy
from typing import Any, Dict, Optional

from ..kube import objects as ko


class NodeBuilder:
    def __init__(self, name: str):
        self._obj = ko.new_node(name)

    def with_labels(self, labels: Dict[str, str]) -> "NodeBuilder":
        self._obj["metadata"]["labels"].update(labels)
        return self

    def with_annotations(self, annotations: Dict[str, str]) -> "NodeBuilder":
        self._obj["metadata"]["annotations"].update(annotations)
        return self

    def with_allocatable(self, resources: Dict[str, Any]) -> "NodeBuilder":
        self._obj["status"]["allocatable"].update({k: str(v) for k, v in resources.items()})
        self._obj["status"]["capacity"].update({k: str(v) for k, v in resources.items()})
        return self

    def with_mi355x(self, gpus: int = 8, partitioning: Optional[str] = None) -> "NodeBuilder":
        from .. import constant
        from ..api import v1alpha1 as api
        labels = {constant.LABEL_AMD_GPU_PRODUCT: "AMD_Instinct_MI355X", constant.LABEL_AMD_GPU_COUNT: str(gpus),
                  constant.LABEL_AMD_GPU_VRAM: "288G", constant.LABEL_AMD_GPU_CU_COUNT: "256"}
        if partitioning:
            labels[api.LABEL_GPU_PARTITIONING] = partitioning
        return self.with_labels(labels)

    def build(self) -> Dict[str, Any]:
        return copy.deepcopy(self._obj)


class PodBuilder:
    def __init__(self, name: str, namespace: str = "default"):
        self._obj = ko.new_pod(name, namespace)
        self._obj["spec"]["containers"] = []

    def with_container(self, name: str = "", requests: Optional[Dict[str, Any]] = None,
                       limits: Optional[Dict[str, Any]] = None) -> "PodBuilder":
        res: Dict[str, Any] = {}
        if requests:
            res["requests"] = {k: str(v) for k, v in requests.items()}
        if limits:
            res["limits"] = {k: str(v) for k, v in limits.items()}
        cs = self._obj["spec"]["containers"]
        cs.append({"name": name or f"c{len(cs)}", "resources": res})
        return self

    def with_init_container(self, requests: Dict[str, Any]) -> "PodBuilder":
        ics = self._obj["spec"].setdefault("initContainers", [])
        ics.append({"name": f"init{len(ics)}", "resources": {"requests": {k: str(v) for k, v in requests.items()}}})
        return self

    def with_labels(self, labels: Dict[str, str]) -> "PodBuilder":
        self._obj["metadata"]["labels"].update(labels)
        return self

    def with_annotations(self, annotations: Dict[str, str]) -> "PodBuilder":
        self._obj["metadata"]["annotations"].update(annotations)
        return self

    def with_phase(self, phase: str) -> "PodBuilder":
        self._obj["status"]["phase"] = phase
        return self

    def with_priority(self, priority: int) -> "PodBuilder":
        self._obj["spec"]["priority"] = priority
        return self

    def with_node(self, node: str) -> "PodBuilder":
        self._obj["spec"]["nodeName"] = node
        return self

    def with_scheduler(self, name: str) -> "PodBuilder":
        self._obj["spec"]["schedulerName"] = name
        return self

    def with_overhead(self, overhead: Dict[str, Any]) -> "PodBuilder":
        self._obj["spec"]["overhead"] = {k: str(v) for k, v in overhead.items()}
        return self

    def with_creation_timestamp(self, ts: str) -> "PodBuilder":
        self._obj["metadata"]["creationTimestamp"] = ts
        return self

    def unschedulable(self) -> "PodBuilder":
        ko.set_condition(self._obj, "PodScheduled", "False", "Unschedulable")
        return self

    def build(self) -> Dict[str, Any]:
        return copy.deepcopy(self._obj)


def build_namespace(name: str, labels: Optional[Dict[str, str]] = None) -> Dict[str, Any]:
    return {"apiVersion": "v1", "kind": "Namespace", "metadata": {"name": name, "labels": dict(labels or {})}}
