"""Elastic Resource Quota model: ``ElasticQuota`` / ``CompositeElasticQuota`` and fair sharing.

Spec (docs-only in the reference fork, SURVEY §2.L1-L5 / Appendix A.8;
``docs/en/docs/elastic-resource-quota/{getting-started,key-concepts}.md``):

* ``ElasticQuota`` (namespaced, at most one per namespace) and ``CompositeElasticQuota`` (a list of
  namespaces); ``spec.min`` guaranteed, optional ``spec.max`` >= min, ``status.used``;
* a namespace is subject to one EQ *or* one CEQ, never both;
* ``used`` = requests of **Running** pods only;
* over-quota labelling: pods sorted by creation time, then fewer requested resources; pods whose
  cumulative request exceeds ``min`` are ``over-quota``, the others ``in-quota``;
* fair sharing: ``tot_avail_over = sum_i max(0, min_i - used_i)``,
  ``guaranteed_over_X = min_X / sum_i min_i * tot_avail_over``; Pod-A (quota A) may preempt Pod-B
  (quota B) iff B is over-quota, ``used_A + req_A <= min_A + guaranteed_over_A`` and
  ``used_B - min_B > guaranteed_over_B`` (the docs' worked example reads condition 2 with
  ``min_A +``, which is the consistent form).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Any, Dict, Iterable, List, Mapping, Optional, Set

from ..api import v1alpha1 as api
from ..models import resource as res
from ..utils import pod as podutil

ResourceList = Dict[str, int]


def _rl(x: Optional[Mapping[str, Any]]) -> ResourceList:
    return res.from_k8s(x) if x else {}


@dataclass
class QuotaInfo:
    name: str
    namespace: str                      # where the quota object lives
    namespaces: Set[str]                # namespaces it governs
    min: ResourceList
    max: Optional[ResourceList]
    used: ResourceList = field(default_factory=dict)
    composite: bool = False

    @staticmethod
    def from_object(o: Dict[str, Any]) -> "QuotaInfo":
        md = o.get("metadata", {})
        spec = o.get("spec", {})
        composite = o.get("kind") == api.KIND_COMPOSITE_ELASTIC_QUOTA
        nss = set(spec.get("namespaces") or []) if composite else {md.get("namespace", "default")}
        mx = spec.get("max")
        return QuotaInfo(md.get("name", ""), md.get("namespace", "default"), nss, _rl(spec.get("min")),
                         _rl(mx) if mx is not None else None, _rl((o.get("status") or {}).get("used")), composite)

    def key(self) -> str:
        return f"{'ceq' if self.composite else 'eq'}/{self.namespace}/{self.name}"

    def resources(self) -> Set[str]:
        return set(self.min) | set(self.max or {})

    def over_min(self, extra: Mapping[str, int]) -> bool:
        return any(self.used.get(r, 0) + extra.get(r, 0) > self.min.get(r, 0) for r in self.resources())

    def exceeds_max(self, extra: Mapping[str, int]) -> bool:
        if self.max is None:
            return False
        return any(self.used.get(r, 0) + extra.get(r, 0) > self.max[r] for r in self.max)

    def used_over_quota(self, r: str) -> int:
        return max(0, self.used.get(r, 0) - self.min.get(r, 0))


def validate_quota(o: Dict[str, Any]) -> List[str]:
    q = QuotaInfo.from_object(o)
    errs = []
    if q.max is not None:
        for r, v in q.min.items():
            if r in q.max and q.max[r] < v:
                errs.append(f"max[{r}]={q.max[r]} < min[{r}]={v}")
    if q.composite and not q.namespaces:
        errs.append("spec.namespaces must not be empty")
    return errs


def validate_cluster(quotas: Iterable[QuotaInfo]) -> List[str]:
    """At most one EQ per namespace; a namespace under one EQ *or* one CEQ."""
    errs = []
    seen: Dict[str, str] = {}
    for q in quotas:
        for ns in q.namespaces:
            if ns in seen:
                errs.append(f"namespace {ns} is subject to both {seen[ns]} and {q.key()}")
            else:
                seen[ns] = q.key()
    return errs


class QuotaSet:
    """All quotas of the cluster with namespace lookup and the fair-share arithmetic."""

    def __init__(self, quotas: Iterable[QuotaInfo]):
        self.quotas = list(quotas)
        self.by_ns: Dict[str, QuotaInfo] = {}
        for q in self.quotas:
            for ns in q.namespaces:
                self.by_ns.setdefault(ns, q)

    def for_namespace(self, ns: str) -> Optional[QuotaInfo]:
        return self.by_ns.get(ns)

    def total_min(self, r: str) -> int:
        return sum(q.min.get(r, 0) for q in self.quotas)

    def total_used(self, r: str) -> int:
        return sum(q.used.get(r, 0) for q in self.quotas)

    def available_over_quota(self, r: str) -> int:
        return sum(max(0, q.min.get(r, 0) - q.used.get(r, 0)) for q in self.quotas)

    def guaranteed_over_quota(self, q: QuotaInfo, r: str) -> float:
        tot = self.total_min(r)
        if tot <= 0:
            return 0.0
        return q.min.get(r, 0) / tot * self.available_over_quota(r)

    def can_borrow(self, q: QuotaInfo, req: Mapping[str, int]) -> bool:
        """An over-min request is admitted while the cluster has unused guaranteed quota to lend:
        sum(used) + req <= sum(min) for every quota-managed resource of the request."""
        for r in q.resources():
            if req.get(r, 0) <= 0:
                continue
            if q.used.get(r, 0) + req.get(r, 0) <= q.min.get(r, 0):
                continue
            if self.total_used(r) + req[r] > self.total_min(r):
                return False
        return True

    def may_preempt(self, preemptor: QuotaInfo, req: Mapping[str, int], victim: QuotaInfo) -> bool:
        """Fair-share conditions 2 and 3 (condition 1, victim over-quota, is per pod).

        A preemptor that stays within its own ``min`` is reclaiming what it lent: any quota using
        more than its ``min`` may lose pods to it (as the upstream capacity-scheduling plugin
        lets an in-min preemptor take from over-min quotas).  Condition 3's guaranteed share is
        computed from the *unused* guarantees, and the preemptor's is about to be used: counting
        it as lendable would let the borrower keep part of the very quota being reclaimed."""
        if preemptor is victim:
            return False
        relevant = [r for r in preemptor.resources() if req.get(r, 0) > 0]
        if not relevant:
            return False
        if all(preemptor.used.get(r, 0) + req[r] <= preemptor.min.get(r, 0) for r in relevant):
            return any(victim.used_over_quota(r) > 0 for r in relevant)
        for r in relevant:
            if preemptor.used.get(r, 0) + req[r] > preemptor.min.get(r, 0) + self.guaranteed_over_quota(preemptor, r):
                return False
        return any(victim.used_over_quota(r) > self.guaranteed_over_quota(victim, r) for r in relevant)


def pod_sort_key(pod: Dict[str, Any], request: Mapping[str, int]):
    """Creation time first, then fewer requested resources (key-concepts.md:21-25)."""
    return (pod.get("metadata", {}).get("creationTimestamp", ""), sum(request.values()), pod["metadata"]["name"])


def compute_used(pods: Iterable[Dict[str, Any]], request_fn) -> ResourceList:
    used: ResourceList = {}
    for p in pods:
        if podutil.is_running(p):
            used = res.add(used, request_fn(p))
    return used


def capacity_labels(pods: List[Dict[str, Any]], q: QuotaInfo, request_fn) -> Dict[str, str]:
    """pod name -> in-quota / over-quota for the Running pods governed by ``q``."""
    running = [p for p in pods if podutil.is_running(p)]
    reqs = {p["metadata"]["namespace"] + "/" + p["metadata"]["name"]: request_fn(p) for p in running}
    running.sort(key=lambda p: pod_sort_key(p, reqs[p["metadata"]["namespace"] + "/" + p["metadata"]["name"]]))
    cum: ResourceList = {}
    out: Dict[str, str] = {}
    for p in running:
        k = p["metadata"]["namespace"] + "/" + p["metadata"]["name"]
        cum = res.add(cum, reqs[k])
        over = any(cum.get(r, 0) > q.min.get(r, 0) for r in q.min)
        out[k] = api.CAPACITY_OVER_QUOTA if over else api.CAPACITY_IN_QUOTA
    return out
