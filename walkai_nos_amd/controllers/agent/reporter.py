"""Partition agent reporter (reference ``internal/controllers/migagent/reporter.go:34-123``).

Under the shared lock: list the partition devices (used = kubelet ``List``; free = allocatable −
used), render them as ``status-gpu-<i>-<profile>-<free|used>`` annotations; when they are unchanged
*and* the reported plan ID already equals the last parsed one, only requeue after the refresh
interval; otherwise strip every ``status-gpu-*`` annotation, write the new ones plus
``status-partitioning-plan`` (and the node's NPS mode), patch, requeue.  ``on_report_done`` always
runs (deferred in the reference).
"""
from __future__ import annotations

import json
import logging
from typing import Any, Callable, Dict, List, Optional

from ...api import v1alpha1 as api
from ...kube import objects as ko
from ...kube.errors import NotFound
from ...kube.memory import create_merge_patch
from ...kube.runtime import Request, Result
from ...models.xcp.profile import extract_profile_name
from .shared import SharedState

log = logging.getLogger("nos.agent.reporter")


class Reporter:
    def __init__(self, client: Any, partition_client: Any, shared: SharedState, refresh_interval: float = 10.0,
                 profile_extractor: Callable[[str], Optional[str]] = extract_profile_name,
                 extra_annotations: Optional[Callable[[], Dict[str, str]]] = None, slice_store: Any = None,
                 observers: Optional[List[Callable[[], Any]]] = None):
        self.client = client
        self.pc = partition_client
        self.shared = shared
        self.refresh_interval = refresh_interval
        self.extract = profile_extractor
        self.extra = extra_annotations
        self.slice_store = slice_store
        self.observers = list(observers or [])   # run after every report (e.g. sliceagent/balance.py)

    def reconcile(self, req: Request) -> Result:
        with self.shared.lock:
            try:
                return self._reconcile(req)
            finally:
                self.shared.on_report_done()
                for obs in self.observers:
                    try:
                        obs()
                    except Exception as e:  # noqa: BLE001 - an observer never fails the report
                        log.warning("report observer failed: %s", e)

    def _reconcile(self, req: Request) -> Result:
        try:
            node = self.client.get("Node", req.name)
        except NotFound:
            return Result()
        devices = self.pc.get_partition_devices()
        new_status = devices.as_status_annotation(self.extract)
        anns = ko.annotations(node)
        # order-insensitive comparison of the rendered status family (reporter.go:80-85's
        # UnorderedEqual of parsed annotations, done on the key -> value map directly)
        new_map = {s.key: s.value() for s in new_status}
        old_map = {k: v for k, v in anns.items() if k.startswith(api.ANNOTATION_GPU_STATUS_PREFIX)}
        desired_extra: Dict[str, str] = {}
        nps = self._nps()
        if nps:
            desired_extra[api.ANNOTATION_MEMORY_PARTITION_STATUS] = nps
        pods = getattr(self.pc, "pods_by_gpu", None)
        if pods is not None:
            desired_extra[api.ANNOTATION_GPU_PODS_STATUS] = json.dumps({str(g): v for g, v in pods().items()},
                                                                       sort_keys=True, separators=(",", ":"))
        if self.shared.last_commit:
            desired_extra[api.ANNOTATION_COMMIT_STATUS] = self.shared.last_commit
        remove = []
        if self.slice_store is not None:
            from ...models.xcp.slices import format_gpu_set
            sliced = format_gpu_set(g for g, ss in self.slice_store.load().items() if ss)
            if sliced:
                desired_extra[api.ANNOTATION_SLICED_GPUS_STATUS] = sliced
            elif api.ANNOTATION_SLICED_GPUS_STATUS in anns:
                remove.append(api.ANNOTATION_SLICED_GPUS_STATUS)
        if self.extra is not None:
            desired_extra.update(self.extra())
        extra_same = all(anns.get(k) == v for k, v in desired_extra.items()) and not remove
        if new_map == old_map and extra_same and \
                anns.get(api.ANNOTATION_REPORTED_PARTITIONING_PLAN) == self.shared.last_parsed_plan_id:
            return Result(requeue_after=self.refresh_interval)
        updated = ko.deepcopy(node)
        a = ko.meta(updated).setdefault("annotations", {})
        for k in list(a):
            if k.startswith(api.ANNOTATION_GPU_STATUS_PREFIX):
                del a[k]
        for s in new_status:
            a[s.key] = s.value()
        a.update(desired_extra)
        for k in remove:
            a.pop(k, None)
        a[api.ANNOTATION_REPORTED_PARTITIONING_PLAN] = self.shared.last_parsed_plan_id
        self.client.patch("Node", req.name, create_merge_patch(node, updated))
        log.debug("reported status for node %s (plan %s)", req.name, self.shared.last_parsed_plan_id)
        return Result(requeue_after=self.refresh_interval)

    def _nps(self) -> Optional[str]:
        fn = getattr(self.pc, "current_profiles", None)
        if fn is None:
            return None
        cur = fn()
        if not cur:
            return None
        return next(iter(cur.values())).split("_", 1)[1]


def probe_annotation(results: Dict[str, Any]) -> Dict[str, str]:
    return {api.ANNOTATION_PROBE_RESULT: json.dumps(results, sort_keys=True, separators=(",", ":"))}
