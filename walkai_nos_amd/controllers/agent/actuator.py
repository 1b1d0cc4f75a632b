"""Partition agent actuator (reference ``internal/controllers/migagent/actuator.go:36-310``).

Reconcile, per annotation change on its own node:

1. no report since the last apply → requeue after 1 s (consumes the token);
2. under the shared lock, record ``spec-partitioning-plan`` as the last parsed plan ID;
3. spec == status (and NPS spec == status) → nothing to do;
4. plan from the *actual* state (kubelet devices + amd-smi modes); devices NotFound → re-register
   the device plugin;
5. skip an empty plan, or one identical to the last applied with an unchanged status;
6. apply: node-wide NPS change first (only on an idle node), then one mode flip per GPU; if any
   flip fails, **roll back** the GPUs already flipped in this plan to their previous mode (the
   reference re-creates deleted MIG profiles, ``actuator.go:181-184``);
7. **node-atomic commit**: every GPU is re-enumerated and verified, then all participants vote
   through the RCCL commit barrier; a failed vote rolls the plan back too;
8. re-register the device plugin when anything changed.

Fixes vs the reference: a deleted node (NotFound) is ignored instead of retried forever (Q13).
"""
from __future__ import annotations

import logging
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

from ...api import v1alpha1 as api
from ...kube import objects as ko
from ...kube.errors import NotFound
from ...kube.runtime import Request, Result
from ...models import annotation as ann
from ...models.errors import GpuError, is_not_found
from ...parallel.barrier import CommitBarrier
from ...utils.metrics import REGISTRY
from .plan import XcpConfigPlan, XcpState, new_xcp_config_plan
from .shared import SharedState

log = logging.getLogger("nos.agent.actuator")

BarrierFactory = Callable[[int], CommitBarrier]


class Actuator:
    def __init__(self, client: Any, partition_client: Any, shared: SharedState, node_name: str,
                 device_plugin: Any = None, barrier_factory: Optional[BarrierFactory] = None,
                 verify: Optional[Callable[[int, str], bool]] = None, clock: Callable[[], float] = time.time):
        self.client = client
        self.pc = partition_client
        self.shared = shared
        self.node_name = node_name
        self.device_plugin = device_plugin
        self.barrier_factory = barrier_factory
        self.verify = verify
        self.clock = clock
        self.last_applied_plan: Optional[XcpConfigPlan] = None
        self.last_applied_status: Optional[list] = None
        self.applied_plans = 0

    def reconcile(self, req: Request) -> Result:
        if not self.shared.at_least_one_report_since_last_apply():
            log.debug("last applied config not reported yet, waiting")
            return Result(requeue_after=1.0)
        with self.shared.lock:
            try:
                node = self.client.get("Node", req.name)
            except NotFound:
                return Result()
            anns = ko.annotations(node)
            self.shared.last_parsed_plan_id = anns.get(api.ANNOTATION_PARTITIONING_PLAN, "")
            status, spec = ann.parse_node_annotations(anns)
            spec_nps = anns.get(api.ANNOTATION_MEMORY_PARTITION_SPEC)
            status_nps = anns.get(api.ANNOTATION_MEMORY_PARTITION_STATUS)
            if ann.spec_matches_status(spec, status) and (not spec_nps or spec_nps == status_nps):
                log.debug("reported status matches desired partitioning")
                return Result()
            plan = self.plan(spec, spec_nps)
            if plan is None:
                return Result()
            try:
                if plan.is_empty():
                    for g, reason in plan.blocked + plan.invalid:
                        log.info("GPU %d not changed: %s", g, reason)
                    return Result()
                if plan.equal(self.last_applied_plan) and self.last_applied_status is not None and \
                        ann.annotations_equal(status, self.last_applied_status):
                    log.debug("plan already applied and status unchanged")
                    return Result()
                err = self.apply(plan)
                if err is not None:
                    # a failed plan is retried (with the runtime's back-off) instead of being
                    # remembered as applied: the reference records it anyway (defer at
                    # actuator.go:106) and then skips the identical retry until the status changes
                    plan = None
            finally:
                self.last_applied_plan, self.last_applied_status = plan, status
            self.shared.on_apply_done()
            if err is not None:
                raise err
            return Result()

    def plan(self, spec: List[ann.SpecAnnotation], spec_nps: Optional[str]) -> Optional[XcpConfigPlan]:
        try:
            devices = self.pc.get_partition_devices()
        except GpuError as e:
            if is_not_found(e):
                self._reregister()
                return None
            raise
        state = XcpState(devices)
        current = self.pc.current_profiles()
        cur_nps = next(iter(current.values())).split("_", 1)[1] if current else None
        if state.matches(spec) and (not spec_nps or spec_nps == cur_nps):
            # devices already match the spec (e.g. the previous apply succeeded but was not reported)
            if all(current.get(a.index) == a.profile for a in spec):
                return XcpConfigPlan()
        return new_xcp_config_plan(state, current, spec, spec_nps, cur_nps)

    def apply(self, plan: XcpConfigPlan) -> Optional[Exception]:
        t0 = time.perf_counter()
        errors: List[str] = []
        flipped: List[Tuple[int, Optional[str]]] = []
        changed = False
        if plan.memory_partition:
            try:
                self.pc.set_memory_partition(plan.memory_partition)
                changed = True
            except GpuError as e:
                REGISTRY.apply_errors.labels(node=self.node_name, op="memory_partition").inc()
                return e
            # the driver reload re-derived every GPU's compute mode; re-read before flipping
            current = self.pc.current_profiles()
            plan.changes = [c.__class__(c.gpu_index, current.get(c.gpu_index), c.to_profile)
                            for c in plan.changes if current.get(c.gpu_index) != c.to_profile]
        for ch in plan.changes:
            try:
                self.pc.set_profile(ch.gpu_index, ch.to_profile)
                flipped.append((ch.gpu_index, ch.from_profile))
                changed = True
            except GpuError as e:
                REGISTRY.apply_errors.labels(node=self.node_name, op="compute_partition").inc()
                errors.append(f"GPU {ch.gpu_index} -> {ch.to_profile}: {e}")
                break
        ok = not errors
        if ok and changed:
            ok = self._commit(plan)
            if not ok:
                errors.append("commit barrier vetoed the plan")
        if not ok and flipped:
            self._rollback(flipped)
        if changed:
            self._reregister()
        REGISTRY.phase_seconds.labels(phase="agent_apply_total").observe(time.perf_counter() - t0)
        self.applied_plans += 1
        self.shared.record_commit(ok)
        if plan.blocked:
            for g, reason in plan.blocked:
                log.info("GPU %d not changed: %s", g, reason)
        if errors:
            return GpuError("at least one operation failed while applying the partitioning plan: " + "; ".join(errors))
        return None

    def _commit(self, plan: XcpConfigPlan) -> bool:
        """Verify every changed GPU, then vote through the node's commit barrier."""
        current = self.pc.current_profiles()
        votes = []
        for ch in plan.changes:
            ok = current.get(ch.gpu_index) == ch.to_profile
            if ok and self.verify is not None:
                ok = bool(self.verify(ch.gpu_index, ch.to_profile))
            votes.append(ok)
        if self.barrier_factory is None:
            return all(votes)
        barrier = self.barrier_factory(max(1, len(votes)))
        try:
            vote_all = getattr(barrier, "vote_all", None)
            if vote_all is not None:
                return bool(vote_all(votes or [True]))
            return bool(barrier.vote(all(votes)))
        finally:
            barrier.close()

    def _rollback(self, flipped: List[Tuple[int, Optional[str]]]) -> None:
        log.info("rolling back %d GPU mode change(s)", len(flipped))
        for g, prev in reversed(flipped):
            if prev is None:
                continue
            try:
                self.pc.set_profile(g, prev)
            except GpuError as e:
                log.error("unable to roll back GPU %d to %s: %s", g, prev, e)

    def _reregister(self) -> None:
        if self.device_plugin is None:
            return
        try:
            self.device_plugin.restart(self.node_name)
        except GpuError as e:
            log.error("unable to re-register the device plugin: %s", e)
