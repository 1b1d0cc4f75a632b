"""nos-scheduler: a scheduler for ``schedulerName: nos-scheduler`` pods with the
``CapacityScheduling`` plugin (docs ``elastic-resource-quota/configuration.md``).

The reference documents a kube-scheduler build with the plugin at PreFilter, PostFilter
(preemption; all other PostFilter plugins disabled) and Reserve; neither the plugin nor the
scheduler ships in the fork.  No kube-scheduler can be built here, so this is a compact scheduler
with the same extension points:

* **PreFilter** — the pod's quota (by namespace) must not exceed ``max``; above ``min`` it may only
  *borrow* while the cluster has unused guaranteed quota (sum used + req <= sum min);
* **Filter** — the default kube-scheduler filters that still run next to the plugin in the
  reference's profile (``quota/filters.py``: NodeUnschedulable, NodeSelector, NodeAffinity,
  TaintToleration), then NodeResourcesFit on every requested resource (allocatable minus the
  requests of the pods bound to the node, terminal pods excluded), extended resources included;
* **Score** — most-allocated on GPU resources (bin packing keeps whole GPUs free for mode flips);
* **PostFilter** — preemption: on each node, victims are over-quota pods of quotas the preemptor
  may reclaim from under the fair-share rule, or lower-priority pods of the same quota; the node
  needing the fewest victims wins, victims are evicted and the pod is nominated;
* **PostFilter, partitioned GPUs** (MI355X) — when no node offers the pod's partition profile at
  all (a team reclaiming a whole ``spx`` GPU while borrowers hold every GPU in ``cpx``), evicting
  pods of that profile cannot help: the profile only appears after a mode flip, and a GPU flips
  only once it is idle.  The scheduler then evicts *every* pod of one GPU — read from the agent's
  ``status-pods`` annotation; a GPU whose pods the borrowers can give up while keeping their own
  ``min``, preferring one the partitioner is already draining for that profile, then the fewest
  victims — and marks the pod ``quota-reclaim``; the partitioner flips the now idle GPU as for
  any pending pod;
* **PostFilter, sliced GPUs** (MI355X, ``models/xcp/slices.py``) — a sliced GPU frees a slice for a
  new profile by re-carving, not by a flip: the scheduler evicts only as many evictable pods of one
  sliced GPU as free the row groups the reclaiming pod's slice needs (fewest victims, cheapest
  first), marks it ``quota-reclaim``, and the partitioner re-carves the freed groups for it;
* **Reserve** — the pod's request is added to its quota's ``used`` for the rest of the cycle.
  A pod that preemption was done for (nominated, or ``quota-reclaim``) holds its request against
  its quota while it waits, so borrowers cannot take the freed capacity back in the meantime.
"""
from __future__ import annotations

import json
import logging
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..api import v1alpha1 as api
from ..kube import objects as ko
from ..kube.errors import Conflict, NotFound
from ..kube.runtime import Manager, Request, Result, Watch
from ..models import resource as res
from ..models.annotation import parse_node_annotations
from ..models.xcp.profile import extract_profile_name, is_xcp_resource, parse_profile
from ..utils import pod as podutil
from ..utils.metrics import REGISTRY
from .elasticquota import QuotaInfo, QuotaSet, capacity_labels, compute_used
from .filters import feasible_nodes
from .gpu_memory import GpuMemoryCalculator
from .operator import list_quotas

log = logging.getLogger("nos.scheduler")

SCHEDULER_NAME = "nos-scheduler"


@dataclass
class CycleState:
    quotas: QuotaSet
    node_free: Dict[str, Dict[str, int]]
    node_pods: Dict[str, List[Dict[str, Any]]]
    requests: Dict[str, Dict[str, int]] = field(default_factory=dict)
    nodes: Dict[str, Dict[str, Any]] = field(default_factory=dict)
    held: Dict[str, Dict[str, int]] = field(default_factory=dict)   # preemptor -> request held in its quota
    labels: Optional[Dict[str, str]] = None                         # pod -> in-quota / over-quota


def is_reclaiming(p: Dict[str, Any]) -> bool:
    return bool(ko.annotations(p).get(api.ANNOTATION_QUOTA_RECLAIM)) or podutil.is_preempting(p)


def _pkey(p: Dict[str, Any]) -> str:
    return ko.namespace(p) + "/" + ko.name(p)


class CapacityScheduling:
    name = "CapacityScheduling"

    def __init__(self, calculator: GpuMemoryCalculator):
        self.calc = calculator

    def request(self, state: CycleState, pod: Dict[str, Any]) -> Dict[str, int]:
        k = _pkey(pod)
        if k not in state.requests:
            state.requests[k] = self.calc.pod_request(pod)
        return state.requests[k]

    def pre_filter(self, state: CycleState, pod: Dict[str, Any]) -> Tuple[bool, str]:
        q = state.quotas.for_namespace(ko.namespace(pod))
        if q is None:
            return True, ""
        req = self.request(state, pod)
        if q.exceeds_max(req):
            return False, f"{podutil.QUOTA_UNSCHEDULABLE_PREFIX}{q.name}: max would be exceeded"
        if q.over_min(req) and not state.quotas.can_borrow(q, req):
            return False, f"{podutil.QUOTA_UNSCHEDULABLE_PREFIX}{q.name}: over min and no quota left to borrow"
        return True, ""

    def reserve(self, state: CycleState, pod: Dict[str, Any]) -> None:
        q = state.quotas.for_namespace(ko.namespace(pod))
        if q is not None:
            req = self.request(state, pod)
            q.used = res.add(q.used, {r: v for r, v in req.items() if r in q.resources()})

    def hold(self, state: CycleState, pod: Dict[str, Any]) -> None:
        """Count a waiting preemptor's request against its quota (see the module docstring)."""
        q = state.quotas.for_namespace(ko.namespace(pod))
        if q is not None and _pkey(pod) not in state.held:
            req = {r: v for r, v in self.request(state, pod).items() if r in q.resources()}
            state.held[_pkey(pod)] = req
            q.used = res.add(q.used, req)

    def unhold(self, state: CycleState, pod: Dict[str, Any]) -> None:
        q = state.quotas.for_namespace(ko.namespace(pod))
        req = state.held.pop(_pkey(pod), None)
        if q is not None and req is not None:
            q.used = res.subtract(q.used, req)

    def _labels(self, state: CycleState) -> Dict[str, str]:
        if state.labels is None:
            state.labels = {}
            every = [p for ps in state.node_pods.values() for p in ps]
            for q in state.quotas.quotas:
                qpods = [p for p in every if ko.namespace(p) in q.namespaces]
                state.labels.update(capacity_labels(qpods, q, lambda p: self.request(state, p)))
        return state.labels

    def candidates(self, state: CycleState, pod: Dict[str, Any], node: str) -> List[Dict[str, Any]]:
        """Running pods of ``node`` that ``pod`` may preempt, cheapest first."""
        qa = state.quotas.for_namespace(ko.namespace(pod))
        req = self.request(state, pod)
        labels = self._labels(state)
        cands = []
        for v in state.node_pods.get(node, []):
            # a terminating pod already frees its capacity for whoever evicted it: counting it
            # again would let a second preemptor claim capacity the first one paid for
            if not podutil.is_running(v) or podutil.is_terminating(v):
                continue
            qb = state.quotas.for_namespace(ko.namespace(v))
            if qb is None:
                continue
            if qa is not None and qb is not qa and labels.get(_pkey(v)) == api.CAPACITY_OVER_QUOTA \
                    and state.quotas.may_preempt(qa, req, qb):
                cands.append(v)
            elif qb is qa and podutil.priority(v) < podutil.priority(pod):
                cands.append(v)
        return sorted(cands, key=lambda p: (podutil.priority(p), _neg_ts(p)))

    def victims_on_node(self, state: CycleState, pod: Dict[str, Any], node: str,
                        fits: Callable[[Dict[str, int], Dict[str, int]], bool]) -> Optional[List[Dict[str, Any]]]:
        req = self.request(state, pod)
        cands = self.candidates(state, pod, node)
        free = dict(state.node_free.get(node, {}))
        victims: List[Dict[str, Any]] = []
        for v in cands:
            if fits(req, free):
                break
            victims.append(v)
            free = res.add(free, res.compute_pod_request(v))
        return victims if fits(req, free) and victims else None

    @staticmethod
    def _xcp_view(state: CycleState, pod: Dict[str, Any], node: str):
        profile = next((extract_profile_name(r) for r in res.compute_pod_request(pod) if is_xcp_resource(r)), None)
        n = state.nodes.get(node)
        if profile is None or n is None:
            return None
        anns = ko.annotations(n)
        nps = anns.get(api.ANNOTATION_MEMORY_PARTITION_STATUS, "").lower()
        if nps and parse_profile(profile).nps != nps:
            return None   # a different NPS is a whole-node switch: the partitioner's alone
        status, spec = parse_node_annotations(anns)
        return profile, anns, status, spec

    @staticmethod
    def _sliced_room(anns: Dict[str, str], status: List[Any]) -> Dict[int, int]:
        """Sliced GPU -> row groups not in use (free slices can be re-carved)."""
        from ..models.xcp.slices import GROUPS, groups_of, parse_gpu_set
        out = {g: GROUPS for g in parse_gpu_set(anns.get(api.ANNOTATION_SLICED_GPUS_STATUS))}
        for a in status:
            if a.index in out and a.is_used():
                out[a.index] -= groups_of(a.profile) * a.quantity
        return out

    def slice_victims(self, state: CycleState, pod: Dict[str, Any], node: str
                      ) -> Optional[Tuple[Tuple[int, int], int, List[Dict[str, Any]]]]:
        """The fewest evictable pods of one sliced GPU of ``node`` whose slices, with the groups
        already free, make room for the pod's slice: ``(rank, gpu index, victims)``, or None."""
        from ..models.xcp.slices import groups_of, is_slice_profile
        view = self._xcp_view(state, pod, node)
        if view is None or not is_slice_profile(view[0]):
            return None
        profile, anns, status, _ = view
        need = groups_of(profile)
        room = self._sliced_room(anns, status)
        try:
            pods_by_gpu = json.loads(anns.get(api.ANNOTATION_GPU_PODS_STATUS) or "{}")
        except ValueError:
            return None
        cands = self.candidates(state, pod, node)
        best = None
        for g, free in sorted(room.items()):
            if free >= need:
                return None                    # room already: the partitioner re-carves it, no eviction
            on_gpu = set(pods_by_gpu.get(str(g), []))
            victims: List[Dict[str, Any]] = []
            got = free
            for v in cands:
                if got >= need:
                    break
                if _pkey(v) not in on_gpu:
                    continue
                vp = next((extract_profile_name(r) for r in res.compute_pod_request(v) if is_xcp_resource(r)), None)
                if vp is None or not is_slice_profile(vp):
                    continue
                victims.append(v)
                got += groups_of(vp)
            if got < need or not victims or not self._evictable_together(state, pod, victims):
                continue
            rank = (len(victims), g)
            if best is None or rank < best[0]:
                best = (rank, g, victims)
        return best

    def gpu_available(self, state: CycleState, pod: Dict[str, Any], node: str) -> bool:
        """``node`` has a GPU already in the pod's profile, or an idle one the partitioner can flip."""
        view = self._xcp_view(state, pod, node)
        if view is None:
            return False
        profile, anns, status, _ = view
        gpus = {a.index for a in status}
        busy = {a.index for a in status if a.is_used() and a.quantity > 0}
        try:
            pods_by_gpu = json.loads(anns.get(api.ANNOTATION_GPU_PODS_STATUS) or "{}")
        except ValueError:
            pods_by_gpu = {}
        on_node = {_pkey(v) for v in state.node_pods.get(node, [])}
        # pods the agent last saw on a GPU that are all gone since: idle once the agent reports again
        emptied = {int(g) for g, keys in pods_by_gpu.items() if keys and not any(k in on_node for k in keys)}
        return any(a.profile == profile for a in status) or bool(gpus - busy) or bool(emptied & busy)

    def gpu_victims(self, state: CycleState, pod: Dict[str, Any], node: str
                    ) -> Optional[Tuple[Tuple[int, int, int], int, List[Dict[str, Any]]]]:
        """The cheapest whole GPU of ``node`` to free for a profile the node does not offer:
        ``(rank, gpu index, victims)``, or None.  Only GPUs of the node's memory-partition mode
        that have no partition of the profile, whose pods (per the agent's ``status-pods``) may all
        be evicted together (``_evictable_together``)."""
        view = self._xcp_view(state, pod, node)
        if view is None:
            return None
        profile, anns, status, spec = view
        try:
            pods_by_gpu = json.loads(anns.get(api.ANNOTATION_GPU_PODS_STATUS) or "{}")
        except ValueError:
            return None
        serving = {a.index for a in status if a.profile == profile}
        draining = {a.index for a in spec if a.profile == profile and a.quantity > 0}
        on_node = {_pkey(v): v for v in state.node_pods.get(node, [])}
        best = None
        for g, keys in pods_by_gpu.items():
            gi = int(g)
            live = [on_node[k] for k in keys if k in on_node]   # pods already gone need no eviction
            if any(podutil.is_terminating(v) for v in live):
                continue   # being freed already (for another preemptor, or shutting down)
            if gi in serving or not live or not self._evictable_together(state, pod, live):
                continue
            rank = (0 if gi in draining else 1, len(live), gi)
            if best is None or rank < best[0]:
                best = (rank, gi, live)
        return best

    def _evictable_together(self, state: CycleState, pod: Dict[str, Any], victims: List[Dict[str, Any]]) -> bool:
        """Per-pod in/over-quota labels follow creation order, not GPU placement, so a GPU's pods
        are judged by amount: every victim is a lower-priority pod of the preemptor's own quota,
        or belongs to a quota the preemptor may reclaim from (fair-share rule) whose victims add
        up to no more than what it uses over its ``min`` — a borrower keeps its guarantee."""
        qa = state.quotas.for_namespace(ko.namespace(pod))
        req = self.request(state, pod)
        take: Dict[int, Tuple[QuotaInfo, Dict[str, int]]] = {}
        for v in victims:
            if not podutil.is_running(v):
                return False
            qb = state.quotas.for_namespace(ko.namespace(v))
            if qb is None:
                return False
            if qb is qa:
                if podutil.priority(v) >= podutil.priority(pod):
                    return False
                continue
            if qa is None or not state.quotas.may_preempt(qa, req, qb):
                return False
            cur = take.setdefault(id(qb), (qb, {}))
            take[id(qb)] = (qb, res.add(cur[1], self.request(state, v)))
        return all(amt.get(r, 0) <= qb.used_over_quota(r) for qb, amt in take.values() for r in qb.resources())


def _neg_ts(p: Dict[str, Any]) -> str:
    # newest first among equal priority: invert the timestamp ordering
    ts = p["metadata"].get("creationTimestamp", "")
    return "".join(chr(0x10FFFF - ord(c)) for c in ts)


class NosScheduler:
    def __init__(self, client: Any, calculator: Optional[GpuMemoryCalculator] = None,
                 on_bind: Optional[Callable[[Dict[str, Any], str], None]] = None, scheduler_name: str = SCHEDULER_NAME,
                 clock: Callable[[], float] = time.time):
        self.client = client
        self.calc = calculator or GpuMemoryCalculator()
        self.plugin = CapacityScheduling(self.calc)
        self.on_bind = on_bind
        self.scheduler_name = scheduler_name
        self.clock = clock
        self.bound = 0
        self.preempted = 0
        self._preempted_for: Dict[str, float] = {}  # preemptor -> when its first victims were evicted
        self._victims_of: Dict[str, set] = {}       # preemptor -> keys of the pods it evicted
        self.reclaim_latency_s: List[float] = []    # preemption -> preemptor bound

    KEY = Request("nos-scheduler-cycle")

    def snapshot(self) -> CycleState:
        quotas = [QuotaInfo.from_object(o) for o in list_quotas(self.client)]
        pods = self.client.list("Pod")
        for q in quotas:
            q.used = {r: v for r, v in compute_used([p for p in pods if ko.namespace(p) in q.namespaces],
                                                   self.calc.pod_request).items() if r in q.resources()}
        node_free: Dict[str, Dict[str, int]] = {}
        node_pods: Dict[str, List[Dict[str, Any]]] = {}
        nodes: Dict[str, Dict[str, Any]] = {}
        for n in self.client.list("Node"):
            node_free[ko.name(n)] = res.from_k8s(ko.node_allocatable(n))
            node_pods[ko.name(n)] = []
            nodes[ko.name(n)] = n
        for p in pods:
            nn = ko.pod_node_name(p)
            if nn in node_free and not podutil.is_terminated(p):
                node_free[nn] = res.subtract(node_free[nn], res.compute_pod_request(p))
                node_pods[nn].append(p)
        state = CycleState(QuotaSet(quotas), node_free, node_pods, nodes=nodes)
        for p in pods:
            if p["spec"].get("schedulerName") == self.scheduler_name and not podutil.is_scheduled(p) \
                    and podutil.is_pending(p) and is_reclaiming(p):
                self.plugin.hold(state, p)
        return state

    @staticmethod
    def fits(req: Dict[str, int], free: Dict[str, int]) -> bool:
        return all(free.get(r, 0) >= v for r, v in req.items() if v > 0 and r != api.RESOURCE_GPU_MEMORY)

    def score(self, node: str, free: Dict[str, int], req: Dict[str, int], state: CycleState) -> Tuple[int, str]:
        gpu_free = sum(v for r, v in free.items() if r.startswith("amd.com/"))
        return (gpu_free, node)  # least free GPU capacity first = most allocated

    def _mark_unschedulable(self, pod: Dict[str, Any], msg: str) -> None:
        cur = next((c for c in pod.get("status", {}).get("conditions") or [] if c.get("type") == "PodScheduled"), {})
        if cur.get("reason") == "Unschedulable" and cur.get("message") == msg:
            return
        st = {"conditions": [{"type": "PodScheduled", "status": "False", "reason": "Unschedulable", "message": msg}]}
        try:
            self.client.patch("Pod", ko.name(pod), {"status": st}, ko.namespace(pod))
        except NotFound:
            pass

    def reconcile(self, req: Request) -> Result:
        pending = [p for p in self.client.list("Pod", field_selector="status.phase=Pending")
                   if p["spec"].get("schedulerName") == self.scheduler_name and not podutil.is_scheduled(p)]
        # preemptors that left the queue without being bound (deleted, bound elsewhere) stop being timed
        waiting = {_pkey(p) for p in pending}
        for k in [k for k in self._preempted_for if k not in waiting]:
            del self._preempted_for[k]
        for k in [k for k in self._victims_of if k not in waiting]:
            del self._victims_of[k]
        if not pending:
            return Result()
        pending.sort(key=lambda p: (-podutil.priority(p), p["metadata"].get("creationTimestamp", ""), ko.name(p)))
        state = self.snapshot()
        retry = False
        for pod in pending:
            self.plugin.unhold(state, pod)    # its own hold does not count against itself
            ok, why = self.plugin.pre_filter(state, pod)
            if not ok:
                self._mark_unschedulable(pod, why)
                if is_reclaiming(pod):
                    self.plugin.hold(state, pod)
                continue
            req_ = res.compute_pod_request(pod)
            allowed, reasons = feasible_nodes(pod, list(state.nodes.values()))
            allowed_names = {ko.name(n) for n in allowed}
            feasible = [n for n, free in state.node_free.items() if n in allowed_names and self.fits(req_, free)]
            if not feasible and self._victims_terminating(state, pod):
                # its victims are still shutting down (graceful deletion): wait for them instead of
                # preempting again (kube-scheduler's PodEligibleToPreemptOthers)
                self.plugin.hold(state, pod)
                retry = True
                continue
            if not feasible:
                preempted = bool(allowed_names) and (self._preempt(state, pod, allowed_names) or
                                                     self._preempt_gpu(state, pod, allowed_names))
                if preempted:
                    retry = True
                else:
                    why = ", ".join(f"{c} {r}" for r, c in sorted(reasons.items()))
                    self._mark_unschedulable(pod, f"0/{len(state.node_free)} nodes are available" +
                                             (f": {why}" if why else ""))
                if preempted or is_reclaiming(pod):
                    self.plugin.hold(state, pod)
                continue
            node = min(feasible, key=lambda n: self.score(n, state.node_free[n], req_, state))
            self.plugin.reserve(state, pod)
            try:
                self.client.bind(ko.name(pod), ko.namespace(pod), node)
            except (Conflict, NotFound):
                continue
            state.node_free[node] = res.subtract(state.node_free[node], req_)
            state.node_pods[node].append(pod)
            self.bound += 1
            t = self._preempted_for.pop(_pkey(pod), None)
            if t is not None:
                self.reclaim_latency_s.append(self.clock() - t)
                REGISTRY.phase_seconds.labels(phase="quota_reclaim").observe(self.clock() - t)
            if self.on_bind is not None:
                self.on_bind(pod, node)
        return Result(requeue_after=1.0) if retry else Result()

    def _preempt(self, state: CycleState, pod: Dict[str, Any], allowed: Optional[set] = None) -> bool:
        """Victims only on nodes the pod may run on at all (preemption cannot fix a taint)."""
        best: Optional[Tuple[int, str, List[Dict[str, Any]]]] = None
        for node in sorted(state.node_free):
            if allowed is not None and node not in allowed:
                continue
            victims = self.plugin.victims_on_node(state, pod, node, self.fits)
            if victims is not None and (best is None or len(victims) < best[0]):
                best = (len(victims), node, victims)
        if best is None:
            return False
        _, node, victims = best
        self._evict(state, pod, node, victims)
        try:
            self.client.patch("Pod", ko.name(pod), {"status": {"nominatedNodeName": node}}, ko.namespace(pod))
        except NotFound:
            pass
        return True

    def _preempt_gpu(self, state: CycleState, pod: Dict[str, Any], allowed: Optional[set] = None) -> bool:
        """Free a whole GPU for a profile no allowed node offers (module docstring).  The pod is
        not nominated — the partitioner ignores nominated pods, and this one needs its flip."""
        xcp = [r for r, v in res.compute_pod_request(pod).items() if v > 0 and is_xcp_resource(r)]
        nodes = [n for n in sorted(state.nodes) if allowed is None or n in allowed]
        if not xcp or any(res.from_k8s(ko.node_allocatable(state.nodes[n])).get(r, 0) > 0 for n in nodes for r in xcp):
            return False   # some node offers the profile: ordinary preemption's case
        sliced = None
        for node in nodes:
            cand = self.plugin.slice_victims(state, pod, node)
            if cand is not None and (sliced is None or cand[0] < sliced[1][0]):
                sliced = (node, cand)
        if sliced is not None:
            node, (_, gpu, victims) = sliced
            log.info("freeing %d pod(s) of sliced GPU %d of %s for %s/%s", len(victims), gpu, node,
                     ko.namespace(pod), ko.name(pod))
            self._evict(state, pod, node, victims)
            self._mark_reclaim(pod, node)
            return True
        if any(self.plugin.gpu_available(state, pod, n) for n in nodes):
            return False   # an idle GPU (or one already flipped) will serve it without evictions
        best = None
        for node in nodes:
            cand = self.plugin.gpu_victims(state, pod, node)
            if cand is not None and (best is None or cand[0] < best[1][0]):
                best = (node, cand)
        if best is None:
            return False
        node, (_, gpu, victims) = best
        log.info("freeing GPU %d of %s for %s/%s (%d pods)", gpu, node, ko.namespace(pod), ko.name(pod), len(victims))
        self._evict(state, pod, node, victims)
        self._mark_reclaim(pod, node)
        return True

    def _mark_reclaim(self, pod: Dict[str, Any], node: str) -> None:
        try:
            self.client.patch("Pod", ko.name(pod), {"metadata": {"annotations": {api.ANNOTATION_QUOTA_RECLAIM: node}}},
                              ko.namespace(pod))
        except NotFound:
            pass

    def _victims_terminating(self, state: CycleState, pod: Dict[str, Any]) -> bool:
        mine = self._victims_of.get(_pkey(pod))
        if not mine:
            return False
        return any(_pkey(v) in mine and podutil.is_terminating(v) for ps in state.node_pods.values() for v in ps)

    def _evict(self, state: CycleState, pod: Dict[str, Any], node: str, victims: List[Dict[str, Any]]) -> None:
        self._preempted_for.setdefault(_pkey(pod), self.clock())
        gone = {_pkey(v) for v in victims}
        self._victims_of.setdefault(_pkey(pod), set()).update(gone)
        for v in victims:
            try:
                self.client.delete("Pod", ko.name(v), ko.namespace(v))
                self.preempted += 1
                REGISTRY.preemptions.inc()
                log.info("preempted %s/%s for %s/%s", ko.namespace(v), ko.name(v), ko.namespace(pod), ko.name(pod))
            except NotFound:
                pass
        # the victims' quota usage is released for the rest of the cycle
        for v in victims:
            q = state.quotas.for_namespace(ko.namespace(v))
            if q is not None:
                q.used = res.subtract(q.used, {r: x for r, x in self.plugin.request(state, v).items()
                                               if r in q.resources()})
        state.node_pods[node] = [p for p in state.node_pods.get(node, []) if _pkey(p) not in gone]
        state.labels = None


def setup_nos_scheduler(mgr: Manager, calculator: Optional[GpuMemoryCalculator] = None,
                        on_bind: Optional[Callable[[Dict[str, Any], str], None]] = None) -> NosScheduler:
    s = NosScheduler(mgr.client, calculator, on_bind, clock=mgr.clock)
    to_cycle = lambda o: [NosScheduler.KEY]  # noqa: E731
    mgr.new_controller("nos-scheduler", s.reconcile,
                       [Watch("Pod", mapper=to_cycle), Watch("Node", mapper=to_cycle),
                        Watch(api.KIND_ELASTIC_QUOTA, mapper=to_cycle),
                        Watch(api.KIND_COMPOSITE_ELASTIC_QUOTA, mapper=to_cycle)], 1)
    return s
