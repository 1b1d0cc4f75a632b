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
* **Reserve** — the pod's request is added to its quota's ``used`` for the rest of the cycle.
"""
from __future__ import annotations

import logging
import time
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from ..api import v1alpha1 as api
from ..kube import objects as ko
from ..kube.errors import Conflict, NotFound
from ..kube.runtime import Manager, Request, Result, Watch
from ..models import resource as res
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
            return False, f"quota {q.name}: max would be exceeded"
        if q.over_min(req) and not state.quotas.can_borrow(q, req):
            return False, f"quota {q.name}: over min and no quota left to borrow"
        return True, ""

    def reserve(self, state: CycleState, pod: Dict[str, Any]) -> None:
        q = state.quotas.for_namespace(ko.namespace(pod))
        if q is not None:
            req = self.request(state, pod)
            q.used = res.add(q.used, {r: v for r, v in req.items() if r in q.resources()})

    def victims_on_node(self, state: CycleState, pod: Dict[str, Any], node: str,
                        fits: Callable[[Dict[str, int], Dict[str, int]], bool]) -> Optional[List[Dict[str, Any]]]:
        qa = state.quotas.for_namespace(ko.namespace(pod))
        req = self.request(state, pod)
        labels: Dict[str, str] = {}
        for q in state.quotas.quotas:
            qpods = [p for ns_pods in [state.node_pods.get(n, []) for n in state.node_pods] for p in ns_pods
                     if ko.namespace(p) in q.namespaces]
            labels.update(capacity_labels(qpods, q, lambda p: self.request(state, p)))
        cands = []
        for v in state.node_pods.get(node, []):
            if not podutil.is_running(v):
                continue
            qb = state.quotas.for_namespace(ko.namespace(v))
            if qb is None:
                continue
            if qa is not None and qb is not qa and labels.get(_pkey(v)) == api.CAPACITY_OVER_QUOTA \
                    and state.quotas.may_preempt(qa, req, qb):
                cands.append(v)
            elif qb is qa and podutil.priority(v) < podutil.priority(pod):
                cands.append(v)
        cands = sorted(cands, key=lambda p: (podutil.priority(p), _neg_ts(p)))
        free = dict(state.node_free.get(node, {}))
        victims: List[Dict[str, Any]] = []
        for v in cands:
            if fits(req, free):
                break
            victims.append(v)
            free = res.add(free, res.compute_pod_request(v))
        return victims if fits(req, free) and victims else None


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
        return CycleState(QuotaSet(quotas), node_free, node_pods, nodes=nodes)

    @staticmethod
    def fits(req: Dict[str, int], free: Dict[str, int]) -> bool:
        return all(free.get(r, 0) >= v for r, v in req.items() if v > 0 and r != api.RESOURCE_GPU_MEMORY)

    def score(self, node: str, free: Dict[str, int], req: Dict[str, int], state: CycleState) -> Tuple[int, str]:
        gpu_free = sum(v for r, v in free.items() if r.startswith("amd.com/"))
        return (gpu_free, node)  # least free GPU capacity first = most allocated

    def _mark_unschedulable(self, pod: Dict[str, Any], msg: str) -> None:
        if podutil.is_unschedulable(pod):
            return
        st = {"conditions": [{"type": "PodScheduled", "status": "False", "reason": "Unschedulable", "message": msg}]}
        try:
            self.client.patch("Pod", ko.name(pod), {"status": st}, ko.namespace(pod))
        except NotFound:
            pass

    def reconcile(self, req: Request) -> Result:
        pending = [p for p in self.client.list("Pod", field_selector="status.phase=Pending")
                   if p["spec"].get("schedulerName") == self.scheduler_name and not podutil.is_scheduled(p)]
        if not pending:
            return Result()
        pending.sort(key=lambda p: (-podutil.priority(p), p["metadata"].get("creationTimestamp", ""), ko.name(p)))
        state = self.snapshot()
        retry = False
        for pod in pending:
            ok, why = self.plugin.pre_filter(state, pod)
            if not ok:
                self._mark_unschedulable(pod, why)
                continue
            req_ = res.compute_pod_request(pod)
            allowed, reasons = feasible_nodes(pod, list(state.nodes.values()))
            allowed_names = {ko.name(n) for n in allowed}
            feasible = [n for n, free in state.node_free.items() if n in allowed_names and self.fits(req_, free)]
            if not feasible:
                if allowed_names and self._preempt(state, pod, allowed_names):
                    retry = True
                else:
                    why = ", ".join(f"{c} {r}" for r, c in sorted(reasons.items()))
                    self._mark_unschedulable(pod, f"0/{len(state.node_free)} nodes are available" +
                                             (f": {why}" if why else ""))
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
        self._preempted_for.setdefault(_pkey(pod), self.clock())
        for v in victims:
            try:
                self.client.delete("Pod", ko.name(v), ko.namespace(v))
                self.preempted += 1
                REGISTRY.preemptions.inc()
                log.info("preempted %s/%s for %s/%s", ko.namespace(v), ko.name(v), ko.namespace(pod), ko.name(pod))
            except NotFound:
                pass
        try:
            self.client.patch("Pod", ko.name(pod), {"status": {"nominatedNodeName": node}}, ko.namespace(pod))
        except NotFound:
            pass
        return True


def setup_nos_scheduler(mgr: Manager, calculator: Optional[GpuMemoryCalculator] = None,
                        on_bind: Optional[Callable[[Dict[str, Any], str], None]] = None) -> NosScheduler:
    s = NosScheduler(mgr.client, calculator, on_bind, clock=mgr.clock)
    to_cycle = lambda o: [NosScheduler.KEY]  # noqa: E731
    mgr.new_controller("nos-scheduler", s.reconcile,
                       [Watch("Pod", mapper=to_cycle), Watch("Node", mapper=to_cycle),
                        Watch(api.KIND_ELASTIC_QUOTA, mapper=to_cycle),
                        Watch(api.KIND_COMPOSITE_ELASTIC_QUOTA, mapper=to_cycle)], 1)
    return s
