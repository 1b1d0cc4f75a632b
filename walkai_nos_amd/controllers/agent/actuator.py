"""Partition agent actuator (reference ``internal/controllers/migagent/actuator.go:36-310``).

Reconcile, per annotation change on its own node:

1. no report since the last apply → requeue after 1 s (consumes the token);
2. under the shared lock, record ``spec-partitioning-plan`` as the last parsed plan ID;
3. spec == status (and NPS spec == status) → nothing to do;
4. plan from the *actual* state (kubelet devices + amd-smi modes); devices NotFound → re-register
   the device plugin;
5. skip an empty plan, or one identical to the last applied with an unchanged status;
6. apply:

   * write the plan to the ``status-partitioning-inflight`` journal annotation first (no journal,
     no flip), and stop every spawned GPU helper of this agent (a helper still holding a KFD
     context would make the flip fail);
   * node-wide NPS change first (only on an idle node);
   * one mode flip per GPU, each only if amd-smi reports **no process** on any partition of that
     GPU (the MI355X form of ref ``actuator.go:221-229``'s "never delete used devices": a flip
     destroys every partition).  A busy GPU is skipped and the plan retried with back-off;
   * if a flip fails, **roll back** the GPUs already flipped in this plan (ref re-creates deleted
     MIG profiles, ``actuator.go:181-184``);

7. **node-atomic commit**: the backend re-enumerated the device map after the flips; every
   logical device of the node gets a vote (its GPU in the planned mode, with the planned number
   of partitions, and ``verify`` passing), and the votes go through the commit barrier — in
   production a spawned helper that sees exactly those devices and all-reduces over RCCL.  A veto
   rolls the plan back;
8. re-register the device plugin when anything changed; clear the journal.

:meth:`Actuator.startup` is the start-up pass (ref ``cmd/migagent/migagent.go:165-199``'s
``initAgent``): it finds a journal left by a crash between two flips and rolls the node forward to
the current spec (or leaves it to the normal plan if the spec moved on) before the controllers run.

Fixes vs the reference: a deleted node (NotFound) is ignored instead of retried forever (Q13).
"""
from __future__ import annotations

import contextlib

import json
import logging
import time
from typing import Any, Callable, Dict, List, Optional, Tuple

from ...api import v1alpha1 as api
from ...kube import objects as ko
from ...kube.errors import NotFound
from ...kube.runtime import Request, Result
from ...models import annotation as ann
from ...models.errors import GpuError, is_not_found
from ...models.xcp.profile import parse_profile
from ...models.xcp.slices import SLICED_MODE, parse_gpu_set
from ...parallel.barrier import CommitBarrier
from ...utils.metrics import REGISTRY
from .plan import XcpConfigPlan, XcpState, new_xcp_config_plan
from .shared import SharedState

log = logging.getLogger("nos.agent.actuator")

BarrierFactory = Callable[[int], CommitBarrier]


class Actuator:
    def __init__(self, client: Any, partition_client: Any, shared: SharedState, node_name: str,
                 device_plugin: Any = None, barrier_factory: Optional[BarrierFactory] = None,
                 verify: Optional[Callable[[int, str], bool]] = None, clock: Callable[[], float] = time.time,
                 journal: bool = True, slice_store: Any = None):
        """``slice_store``: where the CU-mask slice layout of sliced GPUs lives (read by the nos
        partition plugin); None = the node has no sliced GPUs."""
        self.client = client
        self.pc = partition_client
        self.shared = shared
        self.node_name = node_name
        self.device_plugin = device_plugin
        self.barrier_factory = barrier_factory
        self.verify = verify
        self.clock = clock
        self.journal = journal
        self.slice_store = slice_store
        self.last_applied_plan: Optional[XcpConfigPlan] = None
        self.last_applied_status: Optional[list] = None
        self.applied_plans = 0
        self.last_votes: List[bool] = []
        self._vote_devices: List[Any] = []
        self._gpus_before: Dict[int, str] = {}

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
            plan_id = anns.get(api.ANNOTATION_PARTITIONING_PLAN, "")
            self.shared.last_parsed_plan_id = plan_id
            status, spec = ann.parse_node_annotations(anns)
            spec_nps = anns.get(api.ANNOTATION_MEMORY_PARTITION_SPEC)
            status_nps = anns.get(api.ANNOTATION_MEMORY_PARTITION_STATUS)
            sliced = parse_gpu_set(anns.get(api.ANNOTATION_SLICED_GPUS_SPEC))
            same_layout = sliced == parse_gpu_set(anns.get(api.ANNOTATION_SLICED_GPUS_STATUS))
            if ann.spec_matches_status(spec, status) and (not spec_nps or spec_nps == status_nps) and same_layout:
                log.debug("reported status matches desired partitioning")
                return Result()
            plan = self.plan(spec, spec_nps, sliced)
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
                err = self.apply(plan, plan_id)
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

    def plan(self, spec: List[ann.SpecAnnotation], spec_nps: Optional[str],
             sliced: Optional[set] = None) -> Optional[XcpConfigPlan]:
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
        slices = self.slice_store.load() if self.slice_store is not None else {}
        sliced = set(sliced or ()) if self.slice_store is not None else set()
        if state.matches(spec) and (not spec_nps or spec_nps == cur_nps) and not sliced and not any(slices.values()):
            # devices already match the spec (e.g. the previous apply succeeded but was not reported)
            if all(current.get(a.index) == a.profile for a in spec):
                return XcpConfigPlan()
        extra: Dict[str, Any] = {}
        if sliced or any(slices.values()):
            m = self.pc.device_map()
            extra = dict(sliced=sliced, slices=slices, used_ids=self.pc.used_ids(),
                         gpu_ids={g.index: g.bdf for g in m.gpus}, vram_bytes={g.index: g.vram_bytes for g in m.gpus})
        return new_xcp_config_plan(state, current, spec, spec_nps, cur_nps, **extra)

    # -- apply --------------------------------------------------------------------------------
    def apply(self, plan: XcpConfigPlan, plan_id: str = "") -> Optional[Exception]:
        t0 = time.perf_counter()
        errors: List[str] = []
        busy: List[int] = []
        flipped: List[Tuple[int, Optional[str]]] = []
        changed = False
        try:
            self._write_journal(plan, plan_id)
        except Exception as e:  # noqa: BLE001 - no durable record, no flip
            REGISTRY.apply_errors.labels(node=self.node_name, op="journal").inc()
            return GpuError(f"unable to journal plan {plan_id!r} before applying it: {e}")
        self._gpus_before = self._physical_gpus()
        helpers = self.shared.helpers
        gate = helpers.held() if hasattr(helpers, "held") else contextlib.nullcontext()
        with gate:  # no helper may start between the quiesce and the last switch
            stopped = self.shared.helpers.quiesce()
            if stopped:
                log.info("stopped %d GPU helper process(es) before flipping", stopped)
            if plan.memory_partition:
                try:
                    self.pc.set_memory_partition(plan.memory_partition)
                    changed = True
                except GpuError as e:
                    REGISTRY.apply_errors.labels(node=self.node_name, op="memory_partition").inc()
                    self._clear_journal()
                    return e
                # the driver reload re-derived every GPU's compute mode; re-read before flipping
                current = self.pc.current_profiles()
                plan.changes = [c.__class__(c.gpu_index, current.get(c.gpu_index), c.to_profile)
                                for c in plan.changes if current.get(c.gpu_index) != c.to_profile]
            applied = []
            for ch in plan.changes:
                if self._gpu_busy(ch.gpu_index):
                    busy.append(ch.gpu_index)
                    REGISTRY.apply_errors.labels(node=self.node_name, op="gpu_busy").inc()
                    log.info("GPU %d has processes on its partitions: not flipping it to %s", ch.gpu_index, ch.to_profile)
                    continue
                try:
                    self.pc.set_profile(ch.gpu_index, ch.to_profile)
                    flipped.append((ch.gpu_index, ch.from_profile))
                    applied.append(ch)
                    changed = True
                except GpuError as e:
                    REGISTRY.apply_errors.labels(node=self.node_name, op="compute_partition").inc()
                    errors.append(f"GPU {ch.gpu_index} -> {ch.to_profile}: {e}")
                    break
        ok = not errors
        if ok and changed:
            ok = self._commit(applied)
            if not ok:
                errors.append("commit barrier vetoed the plan")
        if ok and plan.slices and self.slice_store is not None:
            # a re-carve is a configuration change only (no device operation, nothing to vote on):
            # the plugin serves the new layout after its next sync
            # only for GPUs in SPX now: a GPU whose flip to SPX was skipped (busy) keeps its hardware
            # partitions, and a saved layout would make the reporter publish it as sliced
            modes = self.pc.current_profiles()
            ready = {g: ss for g, ss in plan.slices.items()
                     if g not in busy and (not ss or str(modes.get(g, "")).startswith(SLICED_MODE))}
            cur = self.slice_store.load()
            cur.update(ready)
            self.slice_store.save({g: ss for g, ss in cur.items() if ss})
            changed = True
        if not ok and flipped:
            gate = helpers.held() if hasattr(helpers, "held") else contextlib.nullcontext()
            with gate:
                helpers.quiesce()  # e.g. a barrier helper left behind by a timeout
                self._rollback(flipped)
        if changed:
            self._reregister()
        self._clear_journal()
        REGISTRY.phase_seconds.labels(phase="agent_apply_total").observe(time.perf_counter() - t0)
        self.applied_plans += 1
        if changed or errors:
            self.shared.record_commit(ok)
        for g, reason in plan.blocked:
            log.info("GPU %d not changed: %s", g, reason)
        if errors:
            return GpuError("at least one operation failed while applying the partitioning plan: " + "; ".join(errors))
        if busy:
            return GpuError(f"GPU(s) {busy} busy (processes on their partitions); retrying later", GpuError.BUSY)
        return None

    def _gpu_busy(self, gpu: int) -> bool:
        fn = getattr(self.pc, "gpu_busy", None)
        if fn is None:
            return False
        try:
            return bool(fn(gpu))
        except GpuError as e:
            log.warning("process list of GPU %d unavailable (%s): treating it as busy", gpu, e)
            return True

    def _commit(self, applied: List[Any]) -> bool:
        """One vote per logical device of the re-enumerated node, through the commit barrier."""
        votes = self._votes(applied)
        self.last_votes = votes
        if self.barrier_factory is None:
            return all(votes)
        try:
            # the GPUs are already switched: a barrier that cannot even be built (the native helper
            # missing, a spawn failure) is a veto, so the rollback below runs
            barrier = self.barrier_factory(max(1, len(votes)))
        except Exception as e:  # noqa: BLE001
            log.error("commit barrier unavailable (%s): vetoing the plan", e)
            REGISTRY.apply_errors.labels(node=self.node_name, op="barrier_unavailable").inc()
            return False
        participants = getattr(barrier, "set_participants", None)
        if participants is not None and self._vote_devices:
            participants(self._vote_devices)
        try:
            vote_all = getattr(barrier, "vote_all", None)
            if vote_all is not None:
                return bool(vote_all(votes or [True]))
            return bool(barrier.vote(all(votes)))
        finally:
            barrier.close()

    def _votes(self, applied: List[Any]) -> List[bool]:
        target = {ch.gpu_index: ch.to_profile for ch in applied}
        self._vote_devices = []
        dm_fn = getattr(self.pc, "device_map", None)
        if dm_fn is None:
            # a partition client without a device map: one vote per changed GPU
            current = self.pc.current_profiles()
            votes = []
            for g, p in target.items():
                ok = current.get(g) == p
                if ok and self.verify is not None:
                    ok = bool(self.verify(g, p))
                votes.append(ok)
            return votes
        m = dm_fn()
        devices = sorted(m.devices, key=lambda d: (d.hip_id, d.gpu_index, d.partition_index))
        self._vote_devices = devices
        # the physical GPUs must come back as they were: a GPU whose partitions all vanished from the
        # re-enumerated map has no device to carry its veto, and build_device_map numbers GPUs by
        # position in the sorted BDF list, so every GPU after it is renumbered and the per-GPU
        # checks below would look at the wrong hardware. Every device votes no (the barrier still
        # runs: on a multi-rank node every rank must take part in the all-reduce).
        before = getattr(self, "_gpus_before", None)
        after = {g.index: g.bdf.lower() for g in m.gpus}
        missing = [g for g in target if not m.partitions_of(g)]
        if (before and after != before) or missing:
            log.error("device map after the flip does not match the node: GPUs before %s, after %s, "
                      "target GPUs without partitions %s", before, after, missing)
            return [False] * max(1, len(devices))
        gpu_ok: Dict[int, bool] = {}
        for g, p in target.items():
            parts = m.partitions_of(g)
            ok = bool(parts) and len(parts) == parse_profile(p).partitions and \
                all(f"{d.compute_mode}_{d.memory_mode}".lower() == p for d in parts)
            if ok and self.verify is not None:
                ok = bool(self.verify(g, p))
            gpu_ok[g] = ok
        return [gpu_ok.get(d.gpu_index, True) for d in devices]

    def _physical_gpus(self) -> Dict[int, str]:
        """GPU index -> BDF of the current device map ({} without one)."""
        dm_fn = getattr(self.pc, "device_map", None)
        if dm_fn is None:
            return {}
        try:
            return {g.index: g.bdf.lower() for g in dm_fn().gpus}
        except GpuError as e:
            log.warning("device map unavailable before the flip: %s", e)
            return {}

    def _rollback(self, flipped: List[Tuple[int, Optional[str]]]) -> None:
        """Flip the GPUs of this plan back, addressed by BDF: if a GPU dropped out of the map the
        others were renumbered, and index ``g`` may now be a different card."""
        log.info("rolling back %d GPU mode change(s)", len(flipped))
        now = {bdf: i for i, bdf in self._physical_gpus().items()}
        for g, prev in reversed(flipped):
            if prev is None:
                continue
            bdf = self._gpus_before.get(g)
            if bdf is not None and now:
                if bdf not in now:
                    log.error("unable to roll back GPU %d (%s) to %s: it is gone from the device map", g, bdf, prev)
                    continue
                g = now[bdf]
            try:
                self.pc.set_profile(g, prev)
            except GpuError as e:
                log.error("unable to roll back GPU %d to %s: %s", g, prev, e)

    def _reregister(self) -> None:
        if self.device_plugin is None:
            return
        try:
            self.device_plugin.restart(self.node_name)
        except Exception as e:  # noqa: BLE001 - the change is committed; the plugin's own sync retries
            log.error("unable to re-register the device plugin: %s", e)

    # -- journal ------------------------------------------------------------------------------
    def _write_journal(self, plan: XcpConfigPlan, plan_id: str) -> None:
        if not self.journal:
            return
        entry = {"plan": plan_id, "at": round(self.clock(), 3),
                 "from": {str(c.gpu_index): c.from_profile for c in plan.changes},
                 "to": {str(c.gpu_index): c.to_profile for c in plan.changes}}
        if plan.memory_partition:
            entry["nps"] = plan.memory_partition
        self.client.patch("Node", self.node_name, {"metadata": {"annotations": {
            api.ANNOTATION_INFLIGHT_PLAN: json.dumps(entry, sort_keys=True, separators=(",", ":"))}}})

    def _clear_journal(self) -> None:
        if not self.journal:
            return
        try:
            self.client.patch("Node", self.node_name, {"metadata": {"annotations": {api.ANNOTATION_INFLIGHT_PLAN: None}}})
        except Exception as e:  # noqa: BLE001 - a stale journal is handled by the next start-up
            log.warning("unable to clear the in-flight plan journal: %s", e)

    # -- start-up -----------------------------------------------------------------------------
    def startup(self) -> Dict[str, Any]:
        """Start-up reconciliation, run once before the controllers start.

        * no journal: nothing was in flight; the normal report → apply loop takes over;
        * a journal whose plan is still the node's spec plan: the agent died between two flips of
          that plan — roll forward now (one synchronous apply against the actual devices);
        * a journal of a superseded plan: the spec moved on; apply the *current* spec now, which
          also moves any GPU left in the old plan's half-applied state.

        Either way the journal is cleared afterwards, and the outcome is returned (and logged)."""
        out: Dict[str, Any] = {"journal": None, "action": "none", "modes": {}}
        try:
            node = self.client.get("Node", self.node_name)
        except NotFound:
            return out
        anns = ko.annotations(node)
        raw = anns.get(api.ANNOTATION_INFLIGHT_PLAN)
        out["modes"] = dict(self.pc.current_profiles())
        if not raw:
            return out
        try:
            journal = json.loads(raw)
        except ValueError:
            journal = {"plan": None}
        out["journal"] = journal
        spec_plan = anns.get(api.ANNOTATION_PARTITIONING_PLAN, "")
        out["action"] = "roll-forward" if journal.get("plan") == spec_plan else "superseded"
        log.warning("found in-flight plan %s at start-up (spec plan %s, modes %s): %s",
                    journal.get("plan"), spec_plan, out["modes"], out["action"])
        REGISTRY.apply_errors.labels(node=self.node_name, op="startup_" + out["action"]).inc()
        self.shared.on_report_done()  # the devices are read fresh by the plan below
        try:
            self.reconcile(Request(self.node_name))
        except GpuError as e:
            out["error"] = str(e)
            log.error("start-up apply failed (the controllers will retry): %s", e)
        self._clear_journal()
        out["modes_after"] = dict(self.pc.current_profiles())
        return out
