"""Wire the gpupartitioner's controllers (``cmd/gpupartitioner/gpupartitioner.go:90-104``)."""
from __future__ import annotations

from typing import Optional

from ... import constant
from ...api import v1alpha1 as api
from ...kube.runtime import Manager, Watch
from ...partitioning.planner import NodeInitializer, Partitioner
from ...utils.predicates import HasLabel
from .node_controller import NodeController
from .pod_controller import PodController


def policy_for(kind: str, policy: str) -> str:
    """``pack`` is the compute-partition policy (homogeneous GPUs, flips with an outage, drains);
    CU-mask slices are carved around the ones in use with no outage — the reference's MIG situation —
    so a ``cumask`` node is planned oldest-first (``fifo``) under ``pack``."""
    if policy == "pack" and kind == api.PARTITIONING_KIND_CUMASK:
        return "fifo"
    return policy


def setup_partitioner(mgr: Manager, kinds=(api.PARTITIONING_KIND_XCP, api.PARTITIONING_KIND_CUMASK),
                      batch_timeout: float = 0.0, batch_idle: float = 0.0, retry_after: float = 5.0,
                      partitioner: Optional[Partitioner] = None, scoring: str = "fraction",
                      policy: str = "fifo", pack=None, defaults=None):
    """``defaults``: the ``ModelDefaults`` every controller here builds node models with (the
    partitioner's ``defaultXcpLayout`` / ``sharedSliceSkipCounts``; None: the library defaults)."""
    partitioner = partitioner or Partitioner(mgr.client)
    pod_ctrls = []
    for kind in kinds:
        pc = PodController(mgr.client, kind, partitioner, clock=mgr.clock, batch_timeout=batch_timeout,
                           batch_idle=batch_idle, retry_after=retry_after, scoring=scoring,
                           policy=policy_for(kind, policy), pack=pack, defaults=defaults)
        # MaxConcurrentReconciles = 1: one writer per kind (mig_controller.go:204)
        mgr.new_controller(f"{constant.CLUSTER_PARTITIONER_CONTROLLER}-{kind}", pc.reconcile,
                           [Watch("Pod", mapper=pc.map_pod)], 1)
        pod_ctrls.append(pc)
    nc = NodeController(mgr.client, NodeInitializer(mgr.client, partitioner, clock=mgr.clock, defaults=defaults))
    mgr.new_controller(constant.NODE_INITIALIZER_CONTROLLER, nc.reconcile,
                       [Watch("Node", [HasLabel(api.LABEL_GPU_PARTITIONING)])], 5)
    return pod_ctrls, nc
