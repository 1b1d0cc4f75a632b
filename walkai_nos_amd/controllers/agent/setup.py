"""Wire the partition agent's reporter and actuator into a manager (``cmd/migagent/migagent.go:106-146``)."""
from __future__ import annotations

from typing import Any, Callable, Optional

from ... import constant
from ...kube.runtime import Manager, Watch
from ...utils.predicates import AnnotationsChanged, ExcludeDelete, MatchingName, NodeResourcesChanged
from .actuator import Actuator, BarrierFactory
from .reporter import Reporter
from .shared import SharedState


def setup_partition_agent(mgr: Manager, node_name: str, partition_client: Any, device_plugin: Any = None,
                          barrier_factory: Optional[BarrierFactory] = None, refresh_interval: float = 10.0,
                          verify: Optional[Callable[[int, str], bool]] = None,
                          extra_annotations: Optional[Callable[[], dict]] = None,
                          probe: Optional[Callable[[SharedState], Callable[[], dict]]] = None,
                          helpers: Any = None, slice_store: Any = None):
    """``probe``: factory taking the agent's SharedState and returning an extra-annotation hook
    (e.g. ``lambda sh: ProbeRunner(sh, node).annotations``) that measures each commit."""
    shared = SharedState(helpers)
    if probe is not None:
        hook = probe(shared)
        if extra_annotations is None:
            extra_annotations = hook
        else:
            user = extra_annotations
            extra_annotations = lambda: {**user(), **hook()}  # noqa: E731
    reporter = Reporter(mgr.client, partition_client, shared, refresh_interval, extra_annotations=extra_annotations,
                        slice_store=slice_store)
    actuator = Actuator(mgr.client, partition_client, shared, node_name, device_plugin, barrier_factory, verify,
                        clock=mgr.clock, slice_store=slice_store)
    mgr.new_controller(constant.AGENT_REPORTER_CONTROLLER, reporter.reconcile,
                       [Watch("Node", [ExcludeDelete(), MatchingName(node_name), NodeResourcesChanged()])])
    mgr.new_controller(constant.AGENT_ACTUATOR_CONTROLLER, actuator.reconcile,
                       [Watch("Node", [ExcludeDelete(), MatchingName(node_name), AnnotationsChanged()])])
    return shared, reporter, actuator
