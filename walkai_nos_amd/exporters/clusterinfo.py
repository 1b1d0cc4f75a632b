"""Cluster-info snapshot collector and exporter (walkai addition; reference
``pkg/clusterinfo/{collector,types}.go`` and ``cmd/clusterinfoexporter/clusterinfoexporter.go``).

Snapshot JSON (wire-compatible)::

    {"ts": RFC3339, "gpus": [{"gpu": profile, "allocated": n, "available": n}],
     "pods": [{"name", "namespace", "status", "gpu", "start_time", "finish_time"}]}

Inventory (Appendix B.9): status annotations first (``used`` -> allocated, ``free`` -> available);
if none exist, node ``status.capacity`` partition resources minus the requests of *all* pods,
capped at capacity.  Pod summaries: only pods requesting partitions/slices, sorted by
(namespace, name); status = first container waiting/terminated reason, then "Running", then the
phase; finish time = latest container ``finishedAt`` once Succeeded/Failed; profiles rendered as
``"cpx_nps1 x2, spx_nps1"``.  MI355X additions: every snapshot also carries the node-level
utilisation and pod density (the north-star metrics), and ``probes``: what every partition or
CU-mask slice measured in the agent's probe-on-commit (``status-probe``) — bf16/fp32 TFLOP/s,
TFLOP/s per CU, HBM GB/s and, for one below its model's expected rate, why it is withheld — so the
inventory says what the capacity can actually deliver, not only how much of it is allocated.
"""
from __future__ import annotations

import datetime as _dt
import json
import logging
import time
import urllib.request
from dataclasses import asdict, dataclass, field
from typing import Any, Callable, Dict, List, Optional

from ..kube import objects as ko
from ..models import annotation as ann
from ..models import resource as res
from ..models.slicing.profile import extract_profile_name as slice_profile, parse_profile as parse_slice
from ..models.xcp.profile import COMPUTE_MODES, extract_profile_name as xcp_profile

log = logging.getLogger("nos.clusterinfo")


def profile_of(resource_name: str) -> Optional[str]:
    return xcp_profile(resource_name) or slice_profile(resource_name)


def gpu_fraction(profile: str) -> float:
    if "_nps" in profile:
        return 1.0 / COMPUTE_MODES[profile.split("_", 1)[0]]
    p = parse_slice(profile)
    return max(p.cus / 256.0, p.memory_gb / 288.0)


@dataclass
class GPUInventory:
    gpu: str
    allocated: int
    available: int


@dataclass
class PodSummary:
    name: str
    namespace: str
    status: str
    gpu: str
    start_time: Optional[str]
    finish_time: Optional[str]


@dataclass
class ProbeSummary:
    node: str
    target: str                    # "gpu<i>.p<k>" (a partition) or a slice id
    gpu: Optional[int]
    n_cus: int
    bf16_tflops: Optional[float]
    fp32_tflops: Optional[float]
    bf16_tflops_per_cu: Optional[float]
    hbm_gbps: Optional[float]
    degraded: str = ""


@dataclass
class Snapshot:
    ts: str
    gpus: List[GPUInventory] = field(default_factory=list)
    pods: List[PodSummary] = field(default_factory=list)
    utilization: Dict[str, float] = field(default_factory=dict)
    probes: List[ProbeSummary] = field(default_factory=list)

    def to_json(self) -> str:
        return json.dumps(asdict(self), sort_keys=False)


def requested_profiles(pod: Dict[str, Any]) -> Dict[str, int]:
    out: Dict[str, int] = {}
    for r, q in res.compute_pod_request(pod).items():
        p = profile_of(r)
        if p is not None and q > 0:
            out[p] = out.get(p, 0) + q
    return out


def inventory_from_annotations(nodes: List[Dict[str, Any]]) -> List[GPUInventory]:
    totals: Dict[str, List[int]] = {}
    for n in nodes:
        status, _ = ann.parse_node_annotations(ko.annotations(n))
        for a in status:
            e = totals.setdefault(a.profile, [0, 0])
            if a.is_used():
                e[0] += a.quantity
            elif a.is_free():
                e[1] += a.quantity
    return [GPUInventory(p, v[0], v[1]) for p, v in sorted(totals.items()) if p]


def inventory_from_capacity(nodes: List[Dict[str, Any]], pods: List[Dict[str, Any]]) -> List[GPUInventory]:
    cap: Dict[str, int] = {}
    for n in nodes:
        for r, q in res.from_k8s(ko.node_capacity(n)).items():
            p = profile_of(r)
            if p is not None:
                cap[p] = cap.get(p, 0) + q
    if not cap:
        return []
    alloc: Dict[str, int] = {}
    for p in pods:  # all pods regardless of phase (reference behaviour)
        for prof, q in requested_profiles(p).items():
            alloc[prof] = alloc.get(prof, 0) + q
    return [GPUInventory(p, min(alloc.get(p, 0), t), t - min(alloc.get(p, 0), t)) for p, t in sorted(cap.items())]


def _container_reason(statuses: List[Dict[str, Any]]) -> str:
    for s in statuses or []:
        st = s.get("state") or {}
        if (st.get("waiting") or {}).get("reason"):
            return st["waiting"]["reason"]
        if (st.get("terminated") or {}).get("reason"):
            return st["terminated"]["reason"]
        if st.get("running") is not None:
            return "Running"
    return ""


def pod_status(pod: Dict[str, Any]) -> str:
    st = pod.get("status") or {}
    return (_container_reason(st.get("containerStatuses")) or _container_reason(st.get("initContainerStatuses"))
            or st.get("phase") or "Unknown")


def _ts(s: Optional[str]) -> Optional[str]:
    d = ko.parse_rfc3339(s)
    return d.astimezone(_dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ") if d else None


def pod_finish_time(pod: Dict[str, Any]) -> Optional[str]:
    st = pod.get("status") or {}
    if st.get("phase") not in ("Succeeded", "Failed"):
        return None
    latest: Optional[str] = None
    for key in ("initContainerStatuses", "containerStatuses", "ephemeralContainerStatuses"):
        for s in st.get(key) or []:
            for state in (s.get("state") or {}, s.get("lastState") or {}):
                fin = (state.get("terminated") or {}).get("finishedAt")
                t = _ts(fin)
                if t and (latest is None or t > latest):
                    latest = t
    return latest


def format_profiles(profiles: Dict[str, int]) -> str:
    return ", ".join(p if q <= 1 else f"{p} x{q}" for p, q in sorted(profiles.items()))


def pod_summaries(pods: List[Dict[str, Any]]) -> List[PodSummary]:
    out = []
    for p in pods:
        profs = requested_profiles(p)
        if not profs:
            continue
        out.append(PodSummary(ko.name(p), ko.namespace(p), pod_status(p), format_profiles(profs),
                              _ts((p.get("status") or {}).get("startTime")), pod_finish_time(p)))
    out.sort(key=lambda s: (s.namespace, s.name))
    return out


def utilization(inventory: List[GPUInventory], nodes: List[Dict[str, Any]]) -> Dict[str, float]:
    alloc = sum(i.allocated * gpu_fraction(i.gpu) for i in inventory)
    total = sum((i.allocated + i.available) * gpu_fraction(i.gpu) for i in inventory)
    pods = sum(i.allocated for i in inventory)
    n_nodes = max(1, len(nodes))
    return {"gpu_allocated_percent": round(100.0 * alloc / total, 3) if total else 0.0,
            "fractional_pods_per_node": round(pods / n_nodes, 3)}


def probe_summaries(nodes: List[Dict[str, Any]]) -> List[ProbeSummary]:
    from ..api import v1alpha1 as api
    out: List[ProbeSummary] = []
    for n in nodes:
        try:
            doc = json.loads(ko.annotations(n).get(api.ANNOTATION_PROBE_RESULT) or "{}")
        except ValueError:
            continue
        for label, r in sorted((doc.get("slices") or {}).items()):
            if not isinstance(r, dict) or "error" in r:
                continue
            cus = int(r.get("n_cus", 0) or 0)
            bf = r.get("bf16_tflops")
            out.append(ProbeSummary(ko.name(n), label, r.get("gpu"), cus, bf, r.get("fp32_tflops"),
                                    round(bf / cus, 3) if bf is not None and cus else None, r.get("hbm_gbps"),
                                    str(r.get("degraded") or "")))
    return out


def probe_totals(probes: List[ProbeSummary]) -> Dict[str, float]:
    healthy = [p for p in probes if not p.degraded and p.bf16_tflops is not None]
    return {"probed_bf16_tflops": round(sum(p.bf16_tflops for p in healthy), 1),
            "degraded_targets": float(sum(1 for p in probes if p.degraded))}


class Collector:
    def __init__(self, client: Any, clock: Callable[[], float] = time.time):
        self.client = client
        self.clock = clock

    def collect(self) -> Snapshot:
        nodes = self.client.list("Node")
        pods = self.client.list("Pod")
        inv = inventory_from_annotations(nodes) or inventory_from_capacity(nodes, pods)
        probes = probe_summaries(nodes)
        util = utilization(inv, nodes)
        if probes:
            util.update(probe_totals(probes))
        return Snapshot(ko.now_rfc3339(self.clock()), inv, pod_summaries(pods), util, probes)


class Exporter:
    """POST the snapshot every ``interval`` (one immediately at start); status >= 300 is an error."""

    def __init__(self, collector: Collector, endpoint: str, api_token: str = "", http_timeout: float = 10.0,
                 post: Optional[Callable[[str, bytes, Dict[str, str], float], int]] = None):
        self.collector = collector
        self.endpoint = endpoint
        self.api_token = api_token
        self.http_timeout = http_timeout
        self.post = post or _http_post
        self.sent = 0

    def send_snapshot(self) -> int:
        snap = self.collector.collect()
        headers = {"Content-Type": "application/json"}
        if self.api_token:
            headers["Authorization"] = f"Bearer {self.api_token}"
        code = self.post(self.endpoint, snap.to_json().encode(), headers, self.http_timeout)
        if code >= 300:
            raise RuntimeError(f"cluster info endpoint returned status {code}")
        self.sent += 1
        return code


def _http_post(url: str, body: bytes, headers: Dict[str, str], timeout: float) -> int:
    req = urllib.request.Request(url, data=body, headers=headers, method="POST")
    try:
        with urllib.request.urlopen(req, timeout=timeout) as r:  # noqa: S310 - operator-configured endpoint
            return r.status
    except urllib.error.HTTPError as e:
        return e.code
