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
    """The device plugin of one simulated node, as kubelet sees it: ``advertised`` (every device id
    per resource) and ``healthy`` (the ids kubelet may allocate; node allocatable counts these).

    * xcp, ``plugin="nos"`` (default) — the nos partition device plugin's own view
      (:class:`~walkai_nos_amd.deviceplugin.partitions.PartitionState`: device map + node
      annotations + allocated ids): free partitions of a GPU being re-partitioned are Unhealthy,
      which is what enforces the pack policy's drain; updates are pushed (``refresh``);
    * xcp, ``plugin="amd"`` — the AMD k8s-device-plugin: every logical device healthy, re-read only
      when its pod is restarted (``reregister``); no drain enforcement;
    * cumask — one device per slice of the slice store (the nos slice plugin)."""

    def __init__(self, smi: FakeAmdSmi, store: Optional[MemorySliceStore] = None, plugin: str = "nos",
                 annotations: Optional[Callable[[], Dict[str, str]]] = None,
                 used: Optional[Callable[[], set]] = None, xcp_slices: Optional[MemorySliceStore] = None):
        """``store``: a cumask node's slice store; ``xcp_slices``: the CU-mask slices of an xcp
        node's sliced GPUs (served by the nos partition plugin next to its partitions)."""
        self.smi = smi
        self.store = store
        self.plugin = plugin
        self.advertised: Dict[str, List[str]] = {}
        self.healthy: Dict[str, List[str]] = {}
        self.registrations = 0
        self.state = None
        if store is None and plugin == "nos":
            from ..deviceplugin.partitions import PartitionState
            self.state = PartitionState(smi.device_map, annotations or (lambda: {}), used or (lambda: set()),
                                        slices=xcp_slices.load if xcp_slices is not None else None)
        self.reregister()

    def current(self) -> Dict[str, List[Tuple[str, bool]]]:
        out: Dict[str, List[Tuple[str, bool]]] = defaultdict(list)
        if self.store is not None:
            for g, slices in sorted(self.store.load().items()):
                for s in slices:
                    out[slice_resource(s.profile)].append((s.id, True))
            return dict(out)
        if self.state is not None:
            return {r: [(d.id, d.healthy) for d in ds] for r, ds in self.state.view().items()}
        for d in self.smi.logical_devices():
            out[f"amd.com/{d.compute_mode.lower()}_{d.memory_mode.lower()}"].append((d.device_id, True))
        return dict(out)

    def refresh(self) -> bool:
        """Re-read the view (a pushed ListAndWatch update); True if anything kubelet sees changed.
        The AMD plugin only re-reads when it is restarted."""
        if self.store is None and self.state is None:
            return False
        return self._load()

    def _load(self) -> bool:
        cur = self.current()
        adv = {r: [i for i, _ in v] for r, v in cur.items()}
        ok = {r: [i for i, h in v if h] for r, v in cur.items()}
        changed = adv != self.advertised or ok != self.healthy
        self.advertised, self.healthy = adv, ok
        return changed

    def reregister(self) -> None:
        self._load()
        self.registrations += 1

    def withheld_gpus(self) -> frozenset:
        return frozenset(self.smi.gpu_index_of(i) for r, ids in self.advertised.items()
                         for i in set(ids) - set(self.healthy.get(r, ())))


class SimKubelet:
    """Device accounting for one node: allocatable = healthy devices of the plugin, allocations
    per pod (admission picks healthy, unallocated devices through the plugin's preferred
    allocation)."""

    def __init__(self, node_name: str, plugin: SimDevicePlugin, smi: FakeAmdSmi):
        self.node_name = node_name
        self.plugin = plugin
        self.smi = smi
        self.allocations: Dict[Tuple[str, str], List[Tuple[str, str]]] = {}
        self.admission_failures = 0

    def used_ids(self) -> Dict[str, str]:
        return {i: r for devs in self.allocations.values() for r, i in devs}

    def free_devices(self, resource: str) -> List[str]:
        used = self.used_ids()
        return [i for i in self.plugin.healthy.get(resource, []) if i not in used]

    def can_fit(self, req: Dict[str, int]) -> bool:
        return all(len(self.free_devices(r)) >= q for r, q in req.items() if is_managed(r))

    def allocate(self, pod_key: Tuple[str, str], req: Dict[str, int]) -> List[Tuple[str, str]]:
        """Admission: ``GetPreferredAllocation`` semantics — one GPU, the one with the most
        partitions in use (whole GPUs stay idle for future mode flips), withheld GPUs last."""
        from ..deviceplugin.server import preferred_same_gpu
        out: List[Tuple[str, str]] = []
        used = self.used_ids()
        withheld = self.plugin.withheld_gpus()
        for r, q in req.items():
            if not is_managed(r):
                continue
            free = self.free_devices(r)
            if len(free) < q:
                raise RuntimeError(f"not enough {r} on {self.node_name}")
            gpu_of = {i: self.smi.gpu_index_of(i) for i in self.plugin.advertised.get(r, [])}
            total: Dict[int, int] = defaultdict(int)
            for i in self.plugin.advertised.get(r, []):
                total[gpu_of[i]] += 1
            # "in use" per GPU counts every resource's allocations (the busiest GPU of the node)
            in_use: Dict[int, int] = defaultdict(int)
            for i in used:
                in_use[self.smi.gpu_index_of(i)] += 1
            avail_by_gpu: Dict[int, int] = defaultdict(int)
            for i in free:
                avail_by_gpu[gpu_of[i]] += 1
            busy_total = {g: avail_by_gpu[g] + in_use[g] for g in total}
            out.extend((r, i) for i in preferred_same_gpu([], free, q, gpu_of, busy_total, set(withheld)))
        self.allocations[pod_key] = out
        return out

    def release(self, pod_key: Tuple[str, str]) -> None:
        self.allocations.pop(pod_key, None)

    def resource_client(self) -> StaticResourceClient:
        # PodResources GetAllocatableResources lists every registered device, healthy or not
        return StaticResourceClient(lambda: [(r, i) for devs in self.allocations.values() for r, i in devs],
                                    lambda: [(r, i) for r, ids in self.plugin.advertised.items() for i in ids],
                                    lambda: [(ns, p, r, i) for (ns, p), devs in list(self.allocations.items())
                                             for r, i in devs])

    def allocatable(self) -> Dict[str, str]:
        out = {"cpu": "256", "memory": "2048Gi", "pods": "250"}
        for r, ids in self.plugin.healthy.items():
            out[r] = str(len(ids))
        return out

    def capacity(self) -> Dict[str, str]:
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
    xcp_slices: Optional[MemorySliceStore] = None   # CU-mask slices of the node's sliced GPUs


class KubeScheduler:
    """kube-scheduler semantics for ``default-scheduler`` pods: it knows nothing about GPUs,
    partitions or drains — only node **allocatable** (what the device plugins report healthy, via
    kubelet) minus the requests of the non-terminal pods bound to the node (NodeResourcesFit), the
    default filters (``quota/filters.py``: NodeUnschedulable, NodeSelector, NodeAffinity,
    TaintToleration) and MostAllocated scoring.  A pod that fits nowhere gets
    ``PodScheduled=False/Unschedulable`` — the signal the partitioner reacts to.  The device a pod
    gets on its node is kubelet's choice (``SimKubelet.allocate``), not the scheduler's."""

    KEY = Request("schedule-all")

    def __init__(self, api_: InMemoryAPIServer, nodes: Dict[str, SimNode], on_bind: Callable[[Dict[str, Any], str], None],
                 scheduler_name: str = "default-scheduler"):
        self.api = api_
        self.nodes = nodes
        self.on_bind = on_bind
        self.scheduler_name = scheduler_name
        self.bound = 0

    def reconcile(self, req: Request) -> Result:
        pods = self.api.list("Pod", copy=False)
        pending = [p for p in pods if ko.pod_phase(p) == "Pending" and not podutil.is_scheduled(p)
                   and p["spec"].get("schedulerName", "default-scheduler") == self.scheduler_name]
        if not pending:
            return Result()
        pending.sort(key=lambda p: (-podutil.priority(p), p["metadata"].get("creationTimestamp", ""), ko.name(p)))
        node_objs = {n.name: self.api.get("Node", n.name) for n in self.nodes.values()}
        free: Dict[str, Dict[str, int]] = {}
        for name, o in node_objs.items():
            free[name] = {r: v for r, v in res.from_k8s(ko.node_allocatable(o)).items() if is_managed(r)}
        for p in pods:
            nn = ko.pod_node_name(p)
            if nn in free and not podutil.is_terminated(p):
                for r, v in res.compute_pod_request(p).items():
                    if is_managed(r):
                        free[nn][r] = free[nn].get(r, 0) - v
        verdict: Dict[Tuple[str, str], bool] = {}
        unplaceable = set()
        for p in pending:
            reqs = {r: q for r, q in res.compute_pod_request(p).items() if is_managed(r)}
            spec = p["spec"]
            shape = repr((spec.get("nodeSelector"), spec.get("tolerations"), spec.get("affinity"),
                          spec.get("nodeName")))
            rkey = (shape, tuple(sorted(reqs.items())))
            target = None
            if rkey not in unplaceable:
                cands = []
                for name in sorted(free):
                    k = (name, shape)
                    if k not in verdict:
                        verdict[k] = filter_node(p, node_objs[name])[0]
                    if verdict[k] and all(free[name].get(r, 0) >= q for r, q in reqs.items()):
                        cands.append(name)
                if cands:
                    # MostAllocated: the node with the least free GPU capacity left
                    target = min(cands, key=lambda n: (sum(v for v in free[n].values() if v > 0), n))
                else:
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
                self.api.bind(ko.name(p), ko.namespace(p), target)
            except (Conflict, NotFound):
                continue
            self.bound += 1
            for r, q in reqs.items():
                free[target][r] = free[target].get(r, 0) - q
            self.on_bind(p, target)
        return Result()


SimScheduler = KubeScheduler  # the simulator's scheduler is plain kube-scheduler semantics


class _PushedPluginUpdate:
    """The actuator's device-plugin hook with the nos partition plugin: no pod restart, the
    plugin re-reads the device map and pushes the new devices (``PluginManager.restart``)."""

    def __init__(self, cluster: "SimCluster", sn: SimNode):
        self.cluster = cluster
        self.sn = sn
        self.pushes = 0

    def restart(self, node: str, timeout: float = 60.0) -> None:
        self.pushes += 1
        self.sn.plugin.refresh()
        self.cluster._refresh_node_status(self.sn)


class SimCluster:
    def __init__(self, n_nodes: int = 1, gpus_per_node: int = 8, model: str = "MI355X",
                 kind: str = api.PARTITIONING_KIND_XCP, refresh_interval: float = 10.0,
                 batch_timeout: float = 0.0, batch_idle: float = 0.0, clock: Optional[SimClock] = None,
                 scoring: str = "fraction", policy: str = "fifo", elastic_quota: bool = False,
                 device_plugin: str = "nos", pack: Any = None, xcp_layout: str = "partitions"):
        """``device_plugin``: ``nos`` (the nos partition plugin: drains enforced through device
        health) or ``amd`` (the AMD k8s-device-plugin, restarted after flips: no drain enforcement).
        ``xcp_layout``: the nodes' ``nos.nebuly.com/xcp-layout`` (``partitions`` | ``slices`` |
        ``auto``; slices need the nos plugin)."""
        if device_plugin not in ("nos", "amd"):
            raise ValueError(f"unknown device plugin {device_plugin!r}")
        if xcp_layout != "partitions" and device_plugin != "nos":
            raise ValueError("CU-mask slices of xcp nodes are served by the nos partition plugin")
        self.xcp_layout = xcp_layout
        self.clock = clock or SimClock()
        self.api = InMemoryAPIServer(clock=self.clock)
        self.kind = kind
        self.device_plugin = device_plugin
        self.gpus_per_node = gpus_per_node
        self.nodes: Dict[str, SimNode] = {}
        self.pod_seq = itertools.count()
        self.binds: List[Tuple[float, str, str]] = []
        # control plane
        self.partitioner_mgr = Manager(self.api, clock=self.clock)
        self.pod_controllers, _ = setup_partitioner(self.partitioner_mgr, kinds=(kind,), batch_timeout=batch_timeout,
                                                    batch_idle=batch_idle, scoring=scoring, policy=policy, pack=pack)
        # kubelet (one controller for every simulated node): device plugin updates -> node status
        self.kubelet_mgr = Manager(self.api, clock=self.clock)
        self.kubelet_mgr.new_controller("sim-kubelet", self._kubelet_sync,
                                        [Watch("Node", mapper=lambda o: [Request(ko.name(o))]),
                                         Watch("Pod", mapper=lambda o: [Request(ko.pod_node_name(o))]
                                               if ko.pod_node_name(o) else [])])
        self.scheduler_mgr = Manager(self.api, clock=self.clock)
        self.scheduler = SimScheduler(self.api, self.nodes, self._on_bind)
        self.scheduler_mgr.new_controller("sim-scheduler", self.scheduler.reconcile,
                                          [Watch("Pod", mapper=lambda o: [SimScheduler.KEY]),
                                           Watch("Node", mapper=lambda o: [SimScheduler.KEY])])
        self.admission_failures = 0
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
        xcp_slices = MemorySliceStore() if store is None and self.device_plugin == "nos" else None
        holder: Dict[str, SimKubelet] = {}

        def node_annotations() -> Dict[str, str]:
            try:
                return ko.annotations(self.api.get("Node", name))
            except NotFound:
                return {}
        plugin = SimDevicePlugin(smi, store, plugin=self.device_plugin, annotations=node_annotations,
                                 used=lambda: set(holder["k"].used_ids()) if "k" in holder else set(),
                                 xcp_slices=xcp_slices)
        kubelet = SimKubelet(name, plugin, smi)
        holder["k"] = kubelet
        labels = {api.LABEL_GPU_PARTITIONING: self.kind, constant.LABEL_AMD_GPU_PRODUCT: f"AMD_Instinct_{model}",
                  constant.LABEL_AMD_GPU_COUNT: str(n_gpus), constant.LABEL_AMD_GPU_VRAM: "288G",
                  constant.LABEL_AMD_GPU_CU_COUNT: "256"}
        if self.kind == api.PARTITIONING_KIND_XCP and self.xcp_layout != "partitions":
            labels[api.LABEL_XCP_LAYOUT] = self.xcp_layout
        self.api.create(ko.new_node(name, labels, allocatable=kubelet.allocatable()))
        mgr = Manager(self.api, clock=self.clock)
        sn = SimNode(name, smi, plugin, kubelet, mgr, xcp_slices=xcp_slices)
        self.nodes[name] = sn
        self._create_dp_pod(sn)
        if store is None and self.device_plugin == "nos":
            dp: Any = _PushedPluginUpdate(self, sn)  # the agent's PluginManager.restart(): a pushed update
        else:
            dp = DevicePluginClient(self.api, namespace=DP_NAMESPACE, poll_interval=0.5,
                                    sleep=lambda s: self.clock.advance(s), clock=self.clock)
        if store is not None:
            sc = SlicingClient(kubelet.resource_client(), smi)
            setup_slice_agent(mgr, name, sc, store, device_plugin=dp, barrier_factory=lambda n: LocalBarrier(n),
                              refresh_interval=refresh_interval)
        else:
            pc = PartitionClient(kubelet.resource_client(), smi)
            setup_partition_agent(mgr, name, pc, device_plugin=dp, barrier_factory=lambda n: LocalBarrier(n),
                                  refresh_interval=refresh_interval, slice_store=xcp_slices)
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
        """Publish the node's allocatable (healthy devices) and capacity (all devices) when they
        changed (the partition agent's eager allocatable patch; kubelet's node status sync)."""
        alloc, cap = sn.kubelet.allocatable(), sn.kubelet.capacity()
        try:
            cur = self.api.get("Node", sn.name).get("status", {})
        except NotFound:
            return
        if cur.get("allocatable") == alloc and cur.get("capacity") == cap:
            return
        # a merge patch keeps keys it does not mention: resources that disappeared are nulled
        gone = lambda old, new: {k: None for k in (old or {}) if k not in new}  # noqa: E731
        self.api.patch("Node", sn.name, {"status": {"allocatable": {**gone(cur.get("allocatable"), alloc), **alloc},
                                                    "capacity": {**gone(cur.get("capacity"), cap), **cap}}})

    def _kubelet_sync(self, req: Request) -> Result:
        sn = self.nodes.get(req.name)
        if sn is not None:
            sn.plugin.refresh()
            self._refresh_node_status(sn)
        return Result()

    def _on_bind(self, pod: Dict[str, Any], node: str, skip_gpus: frozenset = frozenset()) -> None:
        """kubelet side of a binding: admission allocates healthy devices (the plugin's preferred
        allocation) and starts the pod; a pod whose devices are not available is rejected
        (``UnexpectedAdmissionError``, phase Failed), as kubelet does."""
        sn = self.nodes[node]
        sn.plugin.refresh()
        try:
            sn.kubelet.allocate(ko.key(pod), res.compute_pod_request(pod))
        except RuntimeError as e:
            self.admission_failures += 1
            log.warning("admission of %s on %s failed: %s", ko.name(pod), node, e)
            self.api.patch("Pod", ko.name(pod), {"status": {"phase": "Failed", "reason": "UnexpectedAdmissionError",
                                                            "message": str(e)}}, ko.namespace(pod))
            return
        self.api.patch("Pod", ko.name(pod), {"status": {"phase": "Running",
                                                        "startTime": ko.now_rfc3339(self.clock())}},
                       ko.namespace(pod))
        self.binds.append((self.clock(), ko.key(pod)[1], node))

    # -- workload -----------------------------------------------------------------------
    def submit(self, requests: Dict[str, int], name: Optional[str] = None, namespace: str = "default",
               labels: Optional[Dict[str, str]] = None, scheduler_name: str = "default-scheduler",
               priority: int = 0, deadline_s: Optional[float] = None) -> Dict[str, Any]:
        """``deadline_s``: the pod's declared bound, ``spec.activeDeadlineSeconds`` (the workload
        ends it no later; the simulation does not kill pods that outrun it)."""
        name = name or f"pod-{next(self.pod_seq)}"
        pod = ko.new_pod(name, namespace, requests=requests, labels_=labels, scheduler_name=scheduler_name,
                         priority=priority)
        if deadline_s:
            pod["spec"]["activeDeadlineSeconds"] = int(deadline_s)
        return self.api.create(pod)

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
        return [self.kubelet_mgr, self.scheduler_mgr, self.partitioner_mgr] + extra + \
            [n.manager for n in self.nodes.values()]

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
