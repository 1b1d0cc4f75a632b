"""Device-plugin restart client (reference ``pkg/gpu/client.go:37-135``).

``restart(node, timeout)``: list the device-plugin pod on ``node`` (label selector + the
``spec.nodeName`` field), require exactly one, delete it, then poll every ``poll_interval`` until
a *differently named*, non-terminating, Running pod exists on the node or the timeout expires.
The label is configurable; the default targets the AMD k8s-device-plugin DaemonSet.
"""
from __future__ import annotations

import logging
import time
from typing import Any, Callable, Optional

from .. import constant
from ..kube import objects as ko
from ..kube.errors import NotFound
from ..models.errors import GpuError

log = logging.getLogger("nos.deviceplugin")


class DevicePluginClient:
    def __init__(self, client: Any, label_selector: str = constant.DEFAULT_DEVICE_PLUGIN_LABEL,
                 namespace: Optional[str] = None, poll_interval: float = 5.0,
                 sleep: Callable[[float], None] = time.sleep, clock: Callable[[], float] = time.monotonic):
        self.client = client
        self.label_selector = label_selector
        self.namespace = namespace
        self.poll_interval = poll_interval
        self.sleep = sleep
        self.clock = clock

    def _pods(self, node: str):
        return self.client.list("Pod", namespace=self.namespace, label_selector=self.label_selector,
                                field_selector=f"spec.nodeName={node}")

    def restart(self, node: str, timeout: float = constant.DEFAULT_DEVICE_PLUGIN_RESTART_TIMEOUT_S) -> None:
        t0 = time.perf_counter()
        pods = self._pods(node)
        if len(pods) != 1:
            raise GpuError(f"expected exactly 1 device plugin pod on node {node}, found {len(pods)}")
        old = pods[0]
        try:
            self.client.delete("Pod", ko.name(old), ko.namespace(old))
        except NotFound:
            pass
        self.wait_until_running(node, ko.name(old), timeout)
        from ..utils.metrics import REGISTRY
        REGISTRY.phase_seconds.labels(phase="device_plugin_reregister").observe(time.perf_counter() - t0)

    def wait_until_running(self, node: str, old_name: str, timeout: float) -> None:
        end = self.clock() + timeout
        while True:
            for p in self._pods(node):
                if ko.name(p) == old_name or p.get("metadata", {}).get("deletionTimestamp"):
                    continue
                if ko.pod_phase(p) == "Running":
                    log.info("device plugin pod %s running on %s", ko.name(p), node)
                    return
            if self.clock() >= end:
                raise GpuError(f"timeout waiting for the device plugin pod to be recreated on node {node}")
            self.sleep(self.poll_interval)
