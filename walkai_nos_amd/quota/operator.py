"""nos-operator: keeps ``status.used`` of every (Composite)ElasticQuota and the
``nos.nebuly.com/capacity`` label of every governed pod up to date.

Reconciles on quota changes and on pod phase transitions (a pod event maps to the quota governing
its namespace).  Invalid quotas (max < min, a namespace claimed twice) are reported through a
``Ready=False`` status condition instead of being silently used.
"""
from __future__ import annotations

import logging
from typing import Any, Dict, List, Optional

from .. import constant
from ..api import v1alpha1 as api
from ..kube import objects as ko
from ..kube.errors import NotFound
from ..kube.quantity import format_quantity
from ..kube.runtime import Manager, Request, Result, Watch
from ..utils.metrics import REGISTRY
from .elasticquota import QuotaInfo, capacity_labels, compute_used, validate_cluster, validate_quota
from .gpu_memory import GpuMemoryCalculator

log = logging.getLogger("nos.quota.operator")

QUOTA_KINDS = (api.KIND_ELASTIC_QUOTA, api.KIND_COMPOSITE_ELASTIC_QUOTA)


def list_quotas(client: Any) -> List[Dict[str, Any]]:
    out: List[Dict[str, Any]] = []
    for k in QUOTA_KINDS:
        out.extend(client.list(k))
    return out


class QuotaOperator:
    def __init__(self, client: Any, calculator: Optional[GpuMemoryCalculator] = None):
        self.client = client
        self.calc = calculator or GpuMemoryCalculator()

    # requests are keyed "<kind>|<namespace>|<name>" so one controller serves both kinds
    @staticmethod
    def request_for(o: Dict[str, Any]) -> Request:
        return Request(f"{o['kind']}|{ko.name(o)}", ko.namespace(o))

    def map_pod(self, pod: Dict[str, Any]) -> List[Request]:
        ns = ko.namespace(pod)
        out = []
        for q in list_quotas(self.client):
            if ns in QuotaInfo.from_object(q).namespaces:
                out.append(self.request_for(q))
        return out

    def reconcile(self, req: Request) -> Result:
        kind, name = req.name.split("|", 1)
        try:
            obj = self.client.get(kind, name, req.namespace)
        except NotFound:
            return Result()
        q = QuotaInfo.from_object(obj)
        errs = validate_quota(obj)
        others = [QuotaInfo.from_object(o) for o in list_quotas(self.client)]
        errs += [e for e in validate_cluster(others) if q.key() in e]
        pods: List[Dict[str, Any]] = []
        for ns in sorted(q.namespaces):
            pods.extend(p for p in self.client.list("Pod", namespace=ns))
        used = compute_used(pods, self.calc.pod_request)
        used = {r: v for r, v in used.items() if r in q.resources()}
        status = {"used": {r: format_quantity(v) for r, v in sorted(used.items())},
                  "conditions": [{"type": "Ready", "status": "False" if errs else "True",
                                  "reason": "Invalid" if errs else "Valid", "message": "; ".join(errs)}]}
        if (obj.get("status") or {}) != status:
            self.client.patch(kind, name, {"status": status}, req.namespace)
        for r, v in used.items():
            REGISTRY.quota_used.labels(namespace=req.namespace, quota=name, resource=r).set(v)
        q.used = used
        labels = capacity_labels(pods, q, self.calc.pod_request)
        for p in pods:
            k = ko.namespace(p) + "/" + ko.name(p)
            want = labels.get(k)
            have = ko.labels(p).get(api.LABEL_CAPACITY_INFO)
            if want is not None and want != have:
                self.client.patch("Pod", ko.name(p), {"metadata": {"labels": {api.LABEL_CAPACITY_INFO: want}}},
                                  ko.namespace(p))
            elif want is None and have is not None and not ko.pod_phase(p) == "Running":
                self.client.patch("Pod", ko.name(p), {"metadata": {"labels": {api.LABEL_CAPACITY_INFO: None}}},
                                  ko.namespace(p))
        return Result()


def setup_quota_operator(mgr: Manager, calculator: Optional[GpuMemoryCalculator] = None) -> QuotaOperator:
    op = QuotaOperator(mgr.client, calculator)
    watches = [Watch(k, mapper=lambda o: [QuotaOperator.request_for(o)]) for k in QUOTA_KINDS]
    watches.append(Watch("Pod", mapper=op.map_pod))
    mgr.new_controller(constant.QUOTA_OPERATOR_CONTROLLER, op.reconcile, watches, 1)
    return op
