"""CU-mask slice agent: reporter + actuator for nodes labelled ``gpu-partitioning=cumask``.

The reference's gpu-agent only *reports* memory slices (``internal/controllers/gpuagent/
reporter.go:34-110``; the MPS planner that wrote the device-plugin config was removed).
Here the agent also actuates, which is what the docs describe (``getting-started-mps.md``):

* plan per GPU from the spec annotations: free slices that are not wanted are deleted (free first,
  surplus *used* slices are reported as blocked), missing ones are created;
* new slices get CU rows next to the kept ones (:mod:`..models.slicing.cumask`: XCD-symmetric rows,
  used slices never move) and an HBM budget; memory and dedicated-CU budgets are validated;
* the new slice configuration is written to the :class:`SliceStore` the nos device plugin serves,
  the plugin re-registers, and the change is committed through the node commit barrier (rolled
  back to the previous configuration on a veto).

The reporter is the partition agent's reporter with the slice profile extractor (only
``amd.com/gpu-<profile>`` resources are reported, as the reference excludes plain ``nvidia.com/gpu``).
"""
from __future__ import annotations

import logging
import time
from collections import defaultdict
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from ... import constant
from ...api import v1alpha1 as api
from ...kube import objects as ko
from ...kube.errors import NotFound
from ...kube.runtime import Manager, Request, Result, Watch
from ...models import annotation as ann
from ...models.errors import GpuError
from ...models.slicing.cumask import Slice, place
from ...models.slicing.profile import MIN_SHARED_CUS, parse_profile
from ...utils.metrics import REGISTRY
from ...utils.predicates import AnnotationsChanged, ExcludeDelete, MatchingName, NodeResourcesChanged
from ..agent.reporter import Reporter
from ..agent.shared import SharedState

log = logging.getLogger("nos.sliceagent")


@dataclass
class SlicePlan:
    new: Dict[int, List[Slice]] = field(default_factory=dict)
    deleted: List[str] = field(default_factory=list)
    created: List[str] = field(default_factory=list)
    blocked: List[Tuple[int, str]] = field(default_factory=list)

    def is_empty(self) -> bool:
        return not self.deleted and not self.created


def plan_slices(current: Dict[int, List[Slice]], used_ids: set, spec: List[ann.SpecAnnotation],
                gpu_ids: Dict[int, str], memory_gb: int, cu_count: int) -> SlicePlan:
    plan = SlicePlan()
    want: Dict[int, Dict[str, int]] = defaultdict(lambda: defaultdict(int))
    for a in spec:
        want[a.index][a.profile] += a.quantity
    for g in sorted(set(current) | set(want)):
        have = list(current.get(g, []))
        if g not in want:
            plan.new[g] = have
            continue
        keep: List[Slice] = []
        by_prof: Dict[str, List[Slice]] = defaultdict(list)
        for s in have:
            by_prof[s.profile].append(s)
        for prof, ss in by_prof.items():
            target = want[g].get(prof, 0)
            ss.sort(key=lambda s: (s.id not in used_ids, s.id))  # used first: kept preferentially
            kept, extra = ss[:target], ss[target:]
            for s in extra:
                if s.id in used_ids:
                    kept.append(s)
                    plan.blocked.append((g, f"slice {s.id} ({prof}) is in use"))
                else:
                    plan.deleted.append(s.id)
            keep.extend(kept)
        serial = 1 + max([int(s.id.rsplit("::s", 1)[1]) for s in have if "::s" in s.id] or [-1])
        wanted: List[Tuple[str, str]] = []
        for prof, q in sorted(want[g].items()):
            missing = q - sum(1 for s in keep if s.profile == prof)
            for _ in range(max(0, missing)):
                wanted.append((f"{gpu_ids[g]}::s{serial}", prof))
                serial += 1
        mem = sum(parse_profile(s.profile).memory_gb for s in keep) + sum(parse_profile(p).memory_gb for _, p in wanted)
        if mem > memory_gb:
            raise GpuError(f"GPU {g}: slices need {mem} GB, the GPU has {memory_gb} GB")
        ded = sum(parse_profile(s.profile).cus for s in keep) + sum(parse_profile(p).cus for _, p in wanted)
        shared = any(not parse_profile(p).dedicated for p in [s.profile for s in keep] + [p for _, p in wanted])
        if ded > cu_count - (MIN_SHARED_CUS if shared else 0):
            raise GpuError(f"GPU {g}: slices need {ded} dedicated CUs, the GPU has {cu_count}")
        placed = place(keep, wanted, cu_count)
        plan.created.extend(s.id for s in placed)
        plan.new[g] = keep + placed
    return plan


class SliceActuator:
    def __init__(self, client: Any, slicing_client: Any, store: Any, shared: SharedState, node_name: str,
                 device_plugin: Any = None, barrier_factory: Optional[Callable[[int], Any]] = None,
                 cu_count: int = 256, memory_gb: int = 288):
        self.client = client
        self.sc = slicing_client
        self.store = store
        self.shared = shared
        self.node_name = node_name
        self.device_plugin = device_plugin
        self.barrier_factory = barrier_factory
        self.cu_count = cu_count
        self.memory_gb = memory_gb

    def reconcile(self, req: Request) -> Result:
        if not self.shared.at_least_one_report_since_last_apply():
            return Result(requeue_after=1.0)
        with self.shared.lock:
            try:
                node = self.client.get("Node", req.name)
            except NotFound:
                return Result()
            anns = ko.annotations(node)
            self.shared.last_parsed_plan_id = anns.get(api.ANNOTATION_PARTITIONING_PLAN, "")
            status, spec = ann.parse_node_annotations(anns)
            if ann.spec_matches_status(spec, status):
                return Result()
            current = self.store.load()
            gpu_ids = {g.index: g.bdf for g in self.sc.smi.list_gpus()}
            plan = plan_slices(current, self.sc.used_ids(), spec, gpu_ids, self.memory_gb, self.cu_count)
            for g, reason in plan.blocked:
                log.info("GPU %d: %s", g, reason)
            if plan.is_empty():
                return Result()
            t0 = time.perf_counter()
            ok = False
            try:
                self.store.save(plan.new)
                ok = self._commit(len(plan.new))
            finally:
                # whatever happened after the save (a veto, a barrier that could not be built or
                # raised), the store, the plugin and the shared state come out consistent: the old
                # layout back unless committed, the plugin re-read, the apply recorded
                if not ok:
                    self.store.save(current)
                if self.device_plugin is not None:
                    self.device_plugin.restart(self.node_name)
                REGISTRY.phase_seconds.labels(phase="agent_apply_total").observe(time.perf_counter() - t0)
                self.shared.record_commit(ok)
                self.shared.on_apply_done()
            if not ok:
                raise GpuError("commit barrier vetoed the slice plan")
            return Result()

    def _commit(self, n: int) -> bool:
        """The node-atomic vote over the new layout (ref ``actuator.go:181-184`` rolls back a failed
        apply): a barrier that cannot be built or fails is a veto."""
        if self.barrier_factory is None:
            return True
        try:
            b = self.barrier_factory(max(1, n))
        except Exception as e:  # noqa: BLE001
            log.error("commit barrier unavailable (%s): vetoing the slice plan", e)
            REGISTRY.apply_errors.labels(node=self.node_name, op="barrier_unavailable").inc()
            return False
        try:
            vote_all = getattr(b, "vote_all", None)
            return bool(vote_all([True] * n)) if vote_all is not None else bool(b.vote(True))
        except Exception as e:  # noqa: BLE001
            log.error("commit barrier failed (%s): vetoing the slice plan", e)
            return False
        finally:
            b.close()


def setup_slice_agent(mgr: Manager, node_name: str, slicing_client: Any, store: Any, device_plugin: Any = None,
                      barrier_factory: Optional[Callable[[int], Any]] = None, refresh_interval: float = 10.0,
                      cu_count: int = 256, memory_gb: int = 288,
                      probe: Optional[Callable[[SharedState], Callable[[], dict]]] = None,
                      skip_counts: Optional[List[int]] = None,
                      on_release: Optional[Callable[[str], None]] = None):
    from ...models.slicing.profile import SKIP_SHARED_COUNTS, extract_profile_name
    from .balance import SharedBalance, node_event
    shared = SharedState()
    extra = probe(shared) if probe is not None else None
    balance = SharedBalance(node_name, store.load, slicing_client.used_ids, node_event(mgr.client, node_name),
                            SKIP_SHARED_COUNTS if skip_counts is None else skip_counts, on_release=on_release)
    reporter = Reporter(mgr.client, slicing_client, shared, refresh_interval, profile_extractor=extract_profile_name,
                        extra_annotations=extra, observers=[balance.check])
    reporter.balance = balance
    actuator = SliceActuator(mgr.client, slicing_client, store, shared, node_name, device_plugin, barrier_factory,
                             cu_count, memory_gb)
    mgr.new_controller(constant.SLICE_AGENT_REPORTER_CONTROLLER, reporter.reconcile,
                       [Watch("Node", [ExcludeDelete(), MatchingName(node_name), NodeResourcesChanged()])])
    mgr.new_controller(constant.SLICE_AGENT_ACTUATOR_CONTROLLER, actuator.reconcile,
                       [Watch("Node", [ExcludeDelete(), MatchingName(node_name), AnnotationsChanged()])])
    return shared, reporter, actuator



def slice_probe_targets(store: Any, cu_count: int = 256) -> Callable[[], list]:
    """Probe targets for :class:`~walkai_nos_amd.controllers.agent.probe.ProbeRunner`: every live
    slice's CU set on its physical GPU (a CU-masked stream), labelled by the slice id."""
    from ...models.slicing.cumask import cus_of

    def targets() -> list:
        out = []
        for gpu, slices in sorted(store.load().items()):
            for sl in slices:
                out.append((gpu, cus_of(sl, slices, cu_count), sl.id))
        return out
    return targets
