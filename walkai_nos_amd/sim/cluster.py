"""In-process cluster simulator: the substrate of the integration tests and of the control-plane
benchmark (SURVEY §7.1 "in-memory API server" + §7.3 step 6 "fake kubelet / device plugin /
scheduler").

Per node it runs the *real* partition agent (reporter + actuator + commit barrier) against a
:class:`FakeAmdSmi` and a simulated kubelet/device plugin; the *real* partitioner runs against the
shared in-memory API server; a small scheduler binds pods first-fit by most-allocated GPU and marks
the rest ``PodScheduled=False/Unschedulable`` exactly like kube-scheduler, which is what triggers
the partitioner.  Everything runs on one virtual clock, so minutes of cluster time take
milliseconds and runs are deterministic.
"""
from __future__ import annotations

import itertools
import logging
from collections import defaultdict
from dataclasses import dataclass, field
from typing import Any, Callable, Dict, List, Optional, Tuple

from .. import constant
from ..api import v1alpha1 as api
from ..controllers.agent.setup import setup_partition_agent
from ..controllers.partitioner.setup import setup_partitioner
from ..device.amdsmi import FakeAmdSmi
from ..device.deviceplugin_client import DevicePluginClient
from ..device.partition_client import PartitionClient
from ..device.podresources import StaticResourceClient
from ..kube import objects as ko
from ..kube.errors import Conflict, NotFound
from ..kube.memory import InMemoryAPIServer
from ..kube.runtime import Manager, Request, Result, SimClock, Watch, run_until_idle
from ..models import resource as res
from ..controllers.sliceagent.agent import setup_slice_agent
from ..device.slicing_client import MemorySliceStore, SlicingClient
from ..models.slicing.profile import as_resource_name as slice_resource
from ..models.slicing.profile import extract_profile_name as slice_profile_name
from ..models.slicing.profile import is_slice_resource, parse_profile as parse_slice_profile
from ..models.xcp.profile import COMPUTE_MODES, extract_profile_name, is_xcp_resource


def is_managed(r: str) -> bool:
    return is_xcp_resource(r) or is_slice_resource(r)
from ..parallel.barrier import LocalBarrier
from ..quota.filters import filter_node
from ..utils import pod as podutil

log = logging.getLogger("nos.sim")

DP_NAMESPACE = "kube-system"
DP_LABEL_KEY, DP_LABEL_VALUE = constant.DEFAULT_DEVICE_PLUGIN_LABEL.split("=")


class SimDevicePlugin:
    """xcp: one device per logical partition of each GPU (AMD device plugin, mixed naming);
    cumask: one device per slice of the slice store (the nos device plugin)."""

    def __init__(self, smi: FakeAmdSmi, store: Optional[MemorySliceStore] = None):
        self.smi = smi
        self.store = store
        self.advertised: Dict[str, List[str]] = {}
        self.registrations = 0
        self.reregister()

    def current(self) -> Dict[str, List[str]]:
        out: Dict[str, List[str]] = defaultdict(list)
        if self.store is not None:
            for g, slices in sorted(self.store.load().items()):
                for s in slices:
                    out[slice_resource(s.profile)].append(s.id)
            return dict(out)
        for d in self.smi.logical_devices():
            out[f"amd.com/{d.compute_mode.lower()}_{d.memory_mode.lower()}"].append(d.device_id)
        return dict(out)

    def reregister(self) -> None:
        self.advertised = self.current()
        self.registrations += 1


class SimKubelet:
    """Device accounting for one node: allocatable from the device plugin, allocations per pod."""

    def __init__(self, node_name: str, plugin: SimDevicePlugin, smi: FakeAmdSmi):
        self.node_name = node_name
        self.plugin = plugin
        self.smi = smi
        self.allocations: Dict[Tuple[str, str], List[Tuple[str, str]]] = {}

    def used_ids(self) -> Dict[str, str]:
        return {i: r for devs in self.allocations.values() for r, i in devs}

    def free_devices(self, resource: str, skip_gpus: frozenset = frozenset()) -> List[str]:
        used = self.used_ids()
        return [i for i in self.plugin.advertised.get(resource, []) if i not in used
                and (not skip_gpus or self.smi.gpu_index_of(i) not in skip_gpus)]

    def can_fit(self, req: Dict[str, int], skip_gpus: frozenset = frozenset()) -> bool:
        return all(len(self.free_devices(r, skip_gpus)) >= q for r, q in req.items() if is_managed(r))

    def allocate(self, pod_key: Tuple[str, str], req: Dict[str, int],
                 skip_gpus: frozenset = frozenset()) -> List[Tuple[str, str]]:
        """GetPreferredAllocation semantics: pack onto the GPU that already has the most partitions
        in use, so whole GPUs stay idle for future mode flips (fragmentation control)."""
        out: List[Tuple[str, str]] = []
        for r, q in req.items():
            if not is_managed(r):
                continue
            free = self.free_devices(r, skip_gpus)
            used_per_gpu: Dict[int, int] = defaultdict(int)
            for i in self.used_ids():
                used_per_gpu[self.smi.gpu_index_of(i)] += 1
            free.sort(key=lambda i: (-used_per_gpu[self.smi.gpu_index_of(i)], self.smi.gpu_index_of(i), i))
            if len(free) < q:
                raise RuntimeError(f"not enough {r} on {self.node_name}")
            out.extend((r, i) for i in free[:q])
        self.allocations[pod_key] = out
        return out

    def release(self, pod_key: Tuple[str, str]) -> None:
        self.allocations.pop(pod_key, None)

    def resource_client(self) -> StaticResourceClient:
        return StaticResourceClient(lambda: [(r, i) for devs in self.allocations.values() for r, i in devs],
                                    lambda: [(r, i) for r, ids in self.plugin.advertised.items() for i in ids])

    def allocatable(self) -> Dict[str, str]:
        out = {"cpu": "256", "memory": "2048Gi", "pods": "250"}
        for r, ids in self.plugin.advertised.items():
            out[r] = str(len(ids))
        return out


@dataclass
class SimNode:
    name: str
    smi: FakeAmdSmi
    plugin: SimDevicePlugin
    kubelet: SimKubelet
    manager: Manager
    dp_counter: Any = field(default_factory=lambda: itertools.count(1))


def draining_gpus(node: Optional[Dict[str, Any]]) -> frozenset:
    """GPUs whose spec asks for a different geometry than the one they report while partitions
    are in use: they wait for their pods to leave before the agent flips them, so no new pod may
    land on their free partitions (the pack policy's drain, ``plan_cluster_pack`` step 5)."""
    if node is None:
        return frozenset()
    from ..models import annotation as ann
    status, spec = ann.parse_node_annotations(ko.annotations(node))
    want: Dict[int, Dict[str, int]] = defaultdict(lambda: defaultdict(int))
    have: Dict[int, Dict[str, int]] = defaultdict(lambda: defaultdict(int))
    busy = set()
    for a in spec:
        want[a.index][a.profile] += a.quantity
    for a in status:
        have[a.index][a.profile] += a.quantity
        if a.is_used() and a.quantity > 0:
            busy.add(a.index)
    return frozenset(g for g in busy if g in want and dict(want[g]) != dict(have[g]))


class SimScheduler:
    """Binds pending pods (first-fit over nodes ordered most-allocated first) or marks them
    Unschedulable — the signal the partitioner reacts to."""

    KEY = Request("schedule-all")

    def __init__(self, api_: InMemoryAPIServer, nodes: Dict[str, SimNode], on_bind: Callable[[Dict[str, Any], str], None]):
        self.api = api_
        self.nodes = nodes
        self.on_bind = on_bind
        self.bound = 0

    def reconcile(self, req: Request) -> Result:
        pods = [p for p in self.api.list("Pod", field_selector="status.phase=Pending", copy=False)
                if not podutil.is_scheduled(p)
                and p["spec"].get("schedulerName", "default-scheduler") == "default-scheduler"]
        pods.sort(key=lambda p: (-podutil.priority(p), p["metadata"].get("creationTimestamp", ""), ko.name(p)))
        node_objs = {n.name: self.api.get("Node", n.name) for n in self.nodes.values()}
        draining = {name: draining_gpus(o) for name, o in node_objs.items()}
        # per pass: free-device counts per (node, resource), recomputed only for a node that just
        # took a pod, and filter verdicts per (node, scheduling constraints) — pods of one shape share
        # them (the pass was O(pods x nodes x devices) at 64 nodes)
        free: Dict[Tuple[str, str], int] = {}
        verdict: Dict[Tuple[str, str], bool] = {}

        def fits(n: SimNode, reqs: Dict[str, int]) -> bool:
            for r, q in reqs.items():
                if not is_managed(r):
                    continue
                k = (n.name, r)
                if k not in free:
                    free[k] = len(n.kubelet.free_devices(r, draining[n.name]))
                if free[k] < q:
                    return False
            return True

        def passes(p: Dict[str, Any], shape: str, n: SimNode) -> bool:
            k = (n.name, shape)
            if k not in verdict:
                verdict[k] = filter_node(p, node_objs[n.name])[0]
            return verdict[k]
        unplaceable = set()  # (shape, request) that fit no node in this pass: free devices only shrink
        for p in pods:
            reqs = res.compute_pod_request(p)
            spec = p["spec"]
            shape = repr((spec.get("nodeSelector"), spec.get("tolerations"), spec.get("affinity"),
                          spec.get("nodeName")))
            rkey = (shape, tuple(sorted((r, q) for r, q in reqs.items() if is_managed(r))))
            target = None
            if rkey not in unplaceable:
                order = sorted(self.nodes.values(), key=lambda n: (-len(n.kubelet.allocations), n.name))
                target = next((n for n in order if passes(p, shape, n) and fits(n, reqs)), None)
                if target is None:
                    unplaceable.add(rkey)
            if target is None:
                if not podutil.is_unschedulable(p):
                    st = {"conditions": [{"type": "PodScheduled", "status": "False", "reason": "Unschedulable",
                                          "message": "0/%d nodes are available: insufficient GPU partitions"
                                                     % len(self.nodes)}]}
                    try:
                        self.api.patch("Pod", ko.name(p), {"status": st}, ko.namespace(p))
                    except NotFound:
                        pass
                continue
            try:
                self.api.bind(ko.name(p), ko.namespace(p), target.name)
            except (Conflict, NotFound):
                continue
            self.bound += 1
            self.on_bind(p, target.name, draining[target.name])
            for k in [k for k in free if k[0] == target.name]:
                del free[k]
        return Result()


class SimCluster:
    def __init__(self, n_nodes: int = 1, gpus_per_node: int = 8, model: str = "MI355X",
                 kind: str = api.PARTITIONING_KIND_XCP, refresh_interval: float = 10.0,
                 batch_timeout: float = 0.0, batch_idle: float = 0.0, clock: Optional[SimClock] = None,
                 scoring: str = "fraction", policy: str = "fifo", elastic_quota: bool = False):
        self.clock = clock or SimClock()
        self.api = InMemoryAPIServer(clock=self.clock)
        self.kind = kind
        self.gpus_per_node = gpus_per_node
        self.nodes: Dict[str, SimNode] = {}
        self.pod_seq = itertools.count()
        self.binds: List[Tuple[float, str, str]] = []
        # control plane
        self.partitioner_mgr = Manager(self.api, clock=self.clock)
        self.pod_controllers, _ = setup_partitioner(self.partitioner_mgr, kinds=(kind,), batch_timeout=batch_timeout,
                                                    batch_idle=batch_idle, scoring=scoring, policy=policy)
        self.scheduler_mgr = Manager(self.api, clock=self.clock)
        self.scheduler = SimScheduler(self.api, self.nodes, self._on_bind)
        self.scheduler_mgr.new_controller("sim-scheduler", self.scheduler.reconcile,
                                          [Watch("Pod", mapper=lambda o: [SimScheduler.KEY]),
                                           Watch("Node", mapper=lambda o: [SimScheduler.KEY])])
        self.api.watch("Pod", self._on_pod_event, replay=False)
        self.quota_mgr: Optional[Manager] = None
        self.nos_scheduler = None
        if elastic_quota:
            from ..quota.operator import setup_quota_operator
            from ..quota.scheduler import setup_nos_scheduler
            self.quota_mgr = Manager(self.api, clock=self.clock)
            setup_quota_operator(self.quota_mgr)
            self.nos_scheduler = setup_nos_scheduler(self.quota_mgr, on_bind=self._on_bind)
        for i in range(n_nodes):
            self.add_node(f"node-{i}", gpus_per_node, model, refresh_interval)

    # -- topology -----------------------------------------------------------------------
    def add_node(self, name: str, n_gpus: int, model: str, refresh_interval: float) -> SimNode:
        smi = FakeAmdSmi(n_gpus=n_gpus, model=model)
        store = MemorySliceStore() if self.kind == api.PARTITIONING_KIND_CUMASK else None
        plugin = SimDevicePlugin(smi, store)
        kubelet = SimKubelet(name, plugin, smi)
        labels = {api.LABEL_GPU_PARTITIONING: self.kind, constant.LABEL_AMD_GPU_PRODUCT: f"AMD_Instinct_{model}",
                  constant.LABEL_AMD_GPU_COUNT: str(n_gpus), constant.LABEL_AMD_GPU_VRAM: "288G",
                  constant.LABEL_AMD_GPU_CU_COUNT: "256"}
        self.api.create(ko.new_node(name, labels, allocatable=kubelet.allocatable()))
        mgr = Manager(self.api, clock=self.clock)
        sn = SimNode(name, smi, plugin, kubelet, mgr)
        self.nodes[name] = sn
        self._create_dp_pod(sn)
        dp = DevicePluginClient(self.api, namespace=DP_NAMESPACE, poll_interval=0.5, sleep=lambda s: self.clock.advance(s),
                                clock=self.clock)
        if store is not None:
            sc = SlicingClient(kubelet.resource_client(), smi)
            setup_slice_agent(mgr, name, sc, store, device_plugin=dp, barrier_factory=lambda n: LocalBarrier(n),
                              refresh_interval=refresh_interval)
        else:
            pc = PartitionClient(kubelet.resource_client(), smi)
            setup_partition_agent(mgr, name, pc, device_plugin=dp, barrier_factory=lambda n: LocalBarrier(n),
                                  refresh_interval=refresh_interval)
        return sn

    def _create_dp_pod(self, sn: SimNode) -> None:
        pod = ko.new_pod(f"amdgpu-device-plugin-{sn.name}-{next(sn.dp_counter)}", DP_NAMESPACE,
                         labels_={DP_LABEL_KEY: DP_LABEL_VALUE}, phase="Running", node_name=sn.name)
        self.api.create(pod)

    def _on_pod_event(self, etype: str, pod: Dict[str, Any], old: Optional[Dict[str, Any]]) -> None:
        if etype != "DELETED":
            return
        if ko.labels(pod).get(DP_LABEL_KEY) == DP_LABEL_VALUE:
            # the DaemonSet controller recreates the plugin pod; on start it re-registers its devices
            sn = self.nodes.get(ko.pod_node_name(pod))
            if sn is not None:
                sn.plugin.reregister()
                self._create_dp_pod(sn)
                self._refresh_node_status(sn)
            return
        node = ko.pod_node_name(pod)
        if node in self.nodes:
            self.nodes[node].kubelet.release(ko.key(pod))

    def _refresh_node_status(self, sn: SimNode) -> None:
        alloc = sn.kubelet.allocatable()
        self.api.patch("Node", sn.name, {"status": {"allocatable": alloc, "capacity": alloc}})

    def _on_bind(self, pod: Dict[str, Any], node: str, skip_gpus: frozenset = frozenset()) -> None:
        """kubelet side of a binding: allocate devices (preferred allocation) and start the pod."""
        self.nodes[node].kubelet.allocate(ko.key(pod), res.compute_pod_request(pod), skip_gpus)
        self.api.patch("Pod", ko.name(pod), {"status": {"phase": "Running"}}, ko.namespace(pod))
        self.binds.append((self.clock(), ko.key(pod)[1], node))

    # -- workload -----------------------------------------------------------------------
    def submit(self, requests: Dict[str, int], name: Optional[str] = None, namespace: str = "default",
               labels: Optional[Dict[str, str]] = None, scheduler_name: str = "default-scheduler",
               priority: int = 0) -> Dict[str, Any]:
        name = name or f"pod-{next(self.pod_seq)}"
        return self.api.create(ko.new_pod(name, namespace, requests=requests, labels_=labels,
                                          scheduler_name=scheduler_name, priority=priority))

    def complete(self, name: str, namespace: str = "default", phase: str = "Succeeded") -> None:
        pod = self.api.get("Pod", name, namespace)
        node = ko.pod_node_name(pod)
        self.api.patch("Pod", name, {"status": {"phase": phase}}, namespace)
        if node in self.nodes:
            self.nodes[node].kubelet.release(ko.key(pod))

    def delete_pod(self, name: str, namespace: str = "default") -> None:
        self.api.delete("Pod", name, namespace)

    # -- driving ------------------------------------------------------------------------
    def managers(self) -> List[Manager]:
        extra = [self.quota_mgr] if self.quota_mgr is not None else []
        return [self.scheduler_mgr, self.partitioner_mgr] + extra + [n.manager for n in self.nodes.values()]

    def run(self, horizon: float = 30.0) -> float:
        return run_until_idle(self.managers(), self.clock, horizon=horizon)

    # -- metrics ------------------------------------------------------------------------
    def running_pods(self) -> List[Dict[str, Any]]:
        return [p for p in self.api.list("Pod", field_selector="status.phase=Running", copy=False)
                if ko.namespace(p) != DP_NAMESPACE]

    def pending_pods(self) -> List[Dict[str, Any]]:
        return [p for p in self.api.list("Pod", field_selector="status.phase=Pending", copy=False)
                if ko.namespace(p) != DP_NAMESPACE]

    def gpu_allocated_fraction(self) -> Dict[Tuple[str, int], float]:
        out: Dict[Tuple[str, int], float] = {}
        for sn in self.nodes.values():
            for g in sn.smi.list_gpus():
                out[(sn.name, g.index)] = 0.0
            for r, i in ((r, i) for devs in sn.kubelet.allocations.values() for r, i in devs):
                p = extract_profile_name(r)
                if p is not None:
                    out[(sn.name, sn.smi.gpu_index_of(i))] += 1.0 / COMPUTE_MODES[p.split("_", 1)[0]]
                    continue
                sp = slice_profile_name(r)
                if sp is not None:
                    prof = parse_slice_profile(sp)
                    spec = sn.smi.list_gpus()[0]
                    frac = max(prof.cus / spec.cu_count, prof.memory_gb * 1e9 / spec.vram_bytes)
                    out[(sn.name, sn.smi.gpu_index_of(i))] += frac
        return out

    def utilization(self) -> float:
        f = self.gpu_allocated_fraction()
        return 100.0 * sum(f.values()) / max(1, len(f))

    def pods_per_node(self) -> float:
        return len(self.running_pods()) / max(1, len(self.nodes))
