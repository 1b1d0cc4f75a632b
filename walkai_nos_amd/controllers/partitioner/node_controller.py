"""Node initialiser controller (reference ``internal/controllers/gpupartitioner/node_controller.go:36-115``).

For a node carrying ``nos.nebuly.com/gpu-partitioning`` that is not yet initialised — initialised
means ``gpu.count == #distinct GPU indexes in the spec annotations`` — require the GPU model and
count labels and run the :class:`NodeInitializer` (fewest-slices geometry, i.e. SPX on MI355X).
"""
from __future__ import annotations

import logging
from typing import Any

from ... import constant
from ...api import v1alpha1 as api
from ...kube import objects as ko
from ...kube.errors import NotFound
from ...kube.runtime import Request, Result
from ...models import annotation as ann
from ...models import gpu_util
from ...models.geometry import get_partitioning_kind
from ...partitioning.planner import NodeInitializer

log = logging.getLogger("nos.node_controller")


class NodeController:
    def __init__(self, client: Any, initializer: NodeInitializer):
        self.client = client
        self.initializer = initializer

    @staticmethod
    def is_initialized(node: dict) -> bool:
        try:
            count = gpu_util.get_count(node)
        except ValueError:
            return False
        _, spec = ann.parse_node_annotations(ko.annotations(node))
        return count == len({a.index for a in spec})

    def reconcile(self, req: Request) -> Result:
        try:
            node = self.client.get("Node", req.name)
        except NotFound:
            return Result()
        if get_partitioning_kind(ko.labels(node)) is None:
            return Result()
        if self.is_initialized(node):
            return Result()
        lbls = ko.labels(node)
        for k in (constant.LABEL_AMD_GPU_PRODUCT, constant.LABEL_AMD_GPU_COUNT):
            if k not in lbls:
                log.info("node %s: missing label %s, cannot initialise", req.name, k)
                return Result()
        self.initializer.init_node_partitioning(node)
        return Result()


LABEL = api.LABEL_GPU_PARTITIONING
