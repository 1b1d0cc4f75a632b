"""nos partition device plugin: MI355X compute partitions as ``amd.com/<mode>_<nps>`` devices,
with the drain enforced where kubelet and kube-scheduler can see it.

Why nos serves partitions itself.  On MIG the reference never needs a drain: a geometry can change
around used devices (ref ``pkg/gpu/mig/gpu.go:99-112``) and the agent deletes only free devices
(ref ``internal/controllers/migagent/actuator.go:225``).  An MI355X mode flip destroys every
partition of the GPU, so it needs the GPU empty: the partitioner's ``pack`` policy writes the new
spec for a busy GPU (its *drain target*) and expects that no new pod lands there.  kube-scheduler
only counts node allocatable, and with the AMD device plugin every free partition of that GPU stays
allocatable — new pods keep landing on it and the drain never ends.

So the devices of this plugin carry the drain: **every partition of a GPU that is being
re-partitioned is advertised ``Unhealthy``** — the node's spec annotations ask this GPU for a
different geometry than its status reports (draining while partitions are in use, or about to
flip) — and so is every partition of a GPU that left the device map.  kubelet never hands an
unhealthy partition to a new container, and node allocatable counts healthy partitions only.

Why *used* partitions too, not just the free ones.  kube-scheduler sees free = allocatable minus
the requests of the pods bound to the node.  Withholding only the free partitions looks exact, but
it races: when a pod on the draining GPU finishes, its request leaves the scheduler's sum at once
while the plugin withholds the freed partition only on its next sync — with pods of that profile
queued, the scheduler binds one immediately, kubelet admits it onto the freed (still healthy)
partition, and under a standing queue the GPU never drains.  With every partition of the GPU
unhealthy there is nothing to race for: a finished pod frees a request and an unhealthy device, so
the next pod can only be admitted onto another GPU.  The price: while a GPU drains, the scheduler
undercounts the node's free partitions *of that GPU's mode* by the partitions still in use there
(none on a single-GPU node; the planner drains the least-used GPU).  Running containers are not
affected by the health of their devices.

The partition agent also patches the node's ``status.allocatable`` with the healthy counts right
after each sync (kubelet's own node status sync runs every 10 s): between the partitioner writing a
drain spec and the agent's sync a pod bound to the GPU's last free partitions would be rejected at
admission; the agent reacts to the spec annotation within one watch event.

When the agent flips the GPU and reports the new status, the spec matches again and the new
partitions are advertised healthy — pushed through ``ListAndWatch`` (a new resource name registers
one more plugin), no plugin restart.  The same pure function (:func:`partition_view`) drives the
gRPC plugin on a node and the simulator's kubelet, so the drain the benchmark relies on is this
production rule, not a simulator shortcut.

``GetPreferredAllocation`` packs a request onto the GPU with the most partitions in use (idle GPUs
stay idle for future flips); ``Allocate`` returns ``/dev/kfd`` and the partition's own render node
(from the device map) — a CPX container sees exactly its partition.
"""
from __future__ import annotations

import logging
from collections import defaultdict
from dataclasses import dataclass
from typing import Any, Callable, Dict, Iterable, List, Mapping, Optional, Set, Tuple

from .. import constant
from ..api import v1alpha1 as api
from ..device.protos import dp
from ..models import annotation as ann
from ..models.slicing.cumask import hsa_cu_mask
from ..models.xcp.slices import SLICED_MODE, parse_gpu_set, recarve, serial_of, spec_by_gpu
from .server import DEVICE_PLUGIN_DIR, KUBELET_SOCKET, DeviceState, PluginManager, PluginServer, \
    preferred_same_gpu

log = logging.getLogger("nos.deviceplugin.partitions")

LOST = "gpu left the device map"


def reconfiguring_gpus(annotations: Mapping[str, str]) -> frozenset:
    """GPUs whose spec annotations ask for a different geometry than their status reports (a GPU
    without spec annotations is not being changed), or for the other layout (hardware partitions
    vs CU-mask slices, ``models/xcp/slices.py``)."""
    anns = dict(annotations or {})
    status, spec = ann.parse_node_annotations(anns)
    want: Dict[int, Dict[str, int]] = defaultdict(dict)
    have: Dict[int, Dict[str, int]] = defaultdict(dict)
    for a in spec:
        want[a.index][a.profile] = want[a.index].get(a.profile, 0) + a.quantity
    for a in status:
        if a.quantity > 0:
            have[a.index][a.profile] = have[a.index].get(a.profile, 0) + a.quantity
    sliced_want = parse_gpu_set(anns.get(api.ANNOTATION_SLICED_GPUS_SPEC))
    sliced_have = parse_gpu_set(anns.get(api.ANNOTATION_SLICED_GPUS_STATUS))
    return frozenset(g for g, w in want.items() if {p: q for p, q in w.items() if q > 0} != have.get(g, {})
                     or (g in sliced_want) != (g in sliced_have))


def slice_withholding(annotations: Mapping[str, str], slices: Mapping[int, List[Any]],
                      used_ids: Set[str]) -> Tuple[frozenset, frozenset]:
    """(GPUs whose every device is withheld, slice ids withheld) for a node with sliced GPUs.

    A sliced GPU the spec keeps sliced is re-carved, not flipped: while the change is pending only
    the free slices the agent is about to delete are withheld (the same :func:`recarve` decides),
    so its other slices keep serving.  A spec its slices in use leave no room for is a drain: every
    slice of the GPU is withheld, like a partitioned GPU being re-partitioned.  Any other GPU
    follows :func:`reconfiguring_gpus`."""
    anns = dict(annotations or {})
    recon = set(reconfiguring_gpus(anns))
    _, spec = ann.parse_node_annotations(anns)
    want = spec_by_gpu(spec)
    sliced_want = parse_gpu_set(anns.get(api.ANNOTATION_SLICED_GPUS_SPEC))
    ids: Set[str] = set()
    for g, ss in slices.items():
        if not ss or g not in sliced_want or g not in recon:
            continue
        rc = recarve(ss, used_ids, want.get(g, {}))
        if rc.achievable:
            recon.discard(g)
            ids.update(s.id for s in rc.delete)
    return frozenset(recon), frozenset(ids)


def draining_gpus(annotations: Mapping[str, str]) -> frozenset:
    """Re-partitioning GPUs that still have partitions in use (they flip once their pods leave)."""
    status, _ = ann.parse_node_annotations(dict(annotations or {}))
    busy = {a.index for a in status if a.is_used() and a.quantity > 0}
    return frozenset(g for g in reconfiguring_gpus(annotations) if g in busy)


def resource_of(device: Any) -> str:
    return f"{constant.AMD_RESOURCE_PREFIX}{device.compute_mode.lower()}_{device.memory_mode.lower()}"


@dataclass(frozen=True)
class PartitionDevice:
    id: str
    resource: str
    gpu_index: int
    partition_index: int
    render_minor: int
    healthy: bool
    reason: str = ""
    bdf: str = ""
    #: a CU-mask slice of an SPX GPU (``models/xcp/slices.py``): its CU bits and HBM budget
    cus: Tuple[int, ...] = ()
    hbm_bytes: int = 0

    @property
    def sliced(self) -> bool:
        return bool(self.cus)


def partition_view(device_map: Any, withheld_gpus: Iterable[int], used_ids: Set[str],
                   lost: Iterable[PartitionDevice] = (), slices: Optional[Mapping[int, List[Any]]] = None,
                   withheld_slices: Iterable[str] = (), degraded: Optional[Mapping[str, str]] = None
                   ) -> Dict[str, List[PartitionDevice]]:
    """resource name -> the partitions to advertise, with their health (see the module docstring).
    ``lost``: devices of GPUs that left the map since the last view, kept listed as unhealthy.
    ``slices``: GPU index -> CU-mask slices of the GPUs served sliced (their SPX device is
    advertised as its slices instead); ``withheld_slices``: slice ids being re-carved away;
    ``degraded``: probe label (``gpu<i>.p<k>`` or a slice id) -> reason, for targets whose last
    probe fell below their model's expected rate (``controllers/agent/probe.py``)."""
    withheld = frozenset(withheld_gpus)
    held_slices = frozenset(withheld_slices)
    bad = dict(degraded or {})
    out: Dict[str, List[PartitionDevice]] = defaultdict(list)
    for d in device_map.devices:
        held = d.gpu_index in withheld
        ss = (slices or {}).get(d.gpu_index) if d.compute_mode.lower() == SLICED_MODE else None
        if ss:
            for s in ss:
                r = constant.AMD_RESOURCE_PREFIX + s.profile
                why = ("gpu re-partitioning (in use, draining)" if s.id in used_ids else "gpu re-partitioning") \
                    if held else ("slice being re-carved" if s.id in held_slices else bad.get(s.id, ""))
                out[r].append(PartitionDevice(s.id, r, d.gpu_index, serial_of(s.id), d.render_minor, not why, why,
                                              d.bdf.lower(), tuple(s.cus), s.hbm_bytes))
            continue
        r = resource_of(d)
        why = ("gpu re-partitioning (in use, draining)" if d.device_id in used_ids else "gpu re-partitioning") \
            if held else bad.get(f"gpu{d.gpu_index}.p{d.partition_index}", "")
        out[r].append(PartitionDevice(d.device_id, r, d.gpu_index, d.partition_index, d.render_minor,
                                      not why, why, d.bdf.lower()))
    present = {d.id for ds in out.values() for d in ds}
    for d in lost:
        if d.id not in present:
            out[d.resource].append(PartitionDevice(d.id, d.resource, d.gpu_index, d.partition_index, d.render_minor,
                                                   False, LOST, d.bdf, d.cus, d.hbm_bytes))
    return {r: sorted(v, key=lambda x: (x.gpu_index, x.partition_index, x.id)) for r, v in out.items()}


def preferred_partitions(view: List[PartitionDevice], must: List[str], available: List[str], size: int,
                         withheld: Iterable[int] = ()) -> List[str]:
    """GetPreferredAllocation for one container: one GPU, the most-used one first (GPUs being
    re-partitioned are unhealthy, so kubelet never offers them)."""
    gpu_of = {d.id: d.gpu_index for d in view}
    total: Dict[int, int] = {}
    for d in view:
        total[d.gpu_index] = total.get(d.gpu_index, 0) + 1
    return preferred_same_gpu(must, available, size, gpu_of, total, set(withheld))


class PartitionState:
    """The node-side inputs of the view: device map (amd-smi), node annotations (the partitioner's
    spec, the reporter's status) and the partitions kubelet has allocated."""

    def __init__(self, device_map: Callable[[], Any], annotations: Callable[[], Mapping[str, str]],
                 used_ids: Callable[[], Set[str]], slices: Optional[Callable[[], Mapping[int, List[Any]]]] = None,
                 degraded: Optional[Callable[[], Mapping[str, str]]] = None):
        self._map = device_map
        self._annotations = annotations
        self._used = used_ids
        self._slices = slices
        self._degraded = degraded
        self._last: Dict[str, PartitionDevice] = {}   # devices of the previous view, by id
        self._lost: Dict[str, PartitionDevice] = {}   # devices of GPUs that left the map

    def view(self) -> Dict[str, List[PartitionDevice]]:
        try:
            anns = self._annotations()
        except Exception as e:  # noqa: BLE001 - without the spec nothing is known to be draining
            log.warning("node annotations unavailable: %s", e)
            anns = {}
        try:
            used = set(self._used())
        except Exception as e:  # noqa: BLE001 - usage only labels the reason
            log.warning("kubelet allocations unavailable: %s", e)
            used = set()
        slices: Mapping[int, List[Any]] = {}
        if self._slices is not None:
            try:
                slices = self._slices()
            except Exception as e:  # noqa: BLE001 - the slice store unreadable: its GPUs are withheld
                log.warning("slice layout unavailable: %s", e)
                slices = {}
                anns = dict(anns)
                anns[api.ANNOTATION_SLICED_GPUS_STATUS] = ""
        withheld, held_slices = slice_withholding(anns, slices, used) if slices else (reconfiguring_gpus(anns), ())
        try:
            m = self._map()
        except Exception as e:  # noqa: BLE001 - a ListAndWatch stream must not end on a map error
            # amd-smi failing (driver reload, a GPU falling off the bus): keep listing the last
            # known devices, all Unhealthy, until the map is readable again
            log.warning("device map unavailable (%s): last known devices reported unhealthy", e)
            out: Dict[str, List[PartitionDevice]] = defaultdict(list)
            for d in list(self._last.values()) + [d for i, d in self._lost.items() if i not in self._last]:
                out[d.resource].append(PartitionDevice(d.id, d.resource, d.gpu_index, d.partition_index,
                                                       d.render_minor, False, f"device map unavailable: {e}"[:120],
                                                       d.bdf, d.cus, d.hbm_bytes))
            return {r: sorted(v, key=lambda x: (x.gpu_index, x.partition_index, x.id)) for r, v in out.items()}
        bdfs = {g.bdf.lower() for g in m.gpus}
        for d in self._last.values():
            if d.bdf not in bdfs:
                self._lost[d.id] = d
        self._lost = {i: d for i, d in self._lost.items() if d.bdf not in bdfs}  # back on the bus
        bad: Mapping[str, str] = {}
        if self._degraded is not None:
            try:
                bad = self._degraded()
            except Exception as e:  # noqa: BLE001 - no probe verdict: nothing is withheld for it
                log.warning("probe results unavailable: %s", e)
        v = partition_view(m, withheld, used, self._lost.values(), slices, held_slices, bad)
        self._last = {d.id: d for ds in v.values() for d in ds if d.bdf in bdfs}
        return v


class PartitionDevicePlugin(PluginServer):
    """One ``amd.com/<mode>_<nps>`` resource of the node's compute partitions."""

    def __init__(self, resource_name: str, state: PartitionState, socket_dir: str = DEVICE_PLUGIN_DIR,
                 poll_interval: float = 1.0, shim_path: str = "/usr/lib/nos/libnos_hbmlimit.so", cu_count: int = 256,
                 shim_present: Optional[Callable[[], bool]] = None):
        super().__init__(resource_name, socket_dir, poll_interval, prefix="nos-xcp-")
        self.state = state
        self.shim_path = shim_path
        #: whether the shim exists on the host (None: assume it does); the agent mounts the host's
        #: shim directory at the same path, so it checks its own view
        self.shim_present = shim_present
        self.cu_count = cu_count

    def _devices(self) -> List[PartitionDevice]:
        return self.state.view().get(self.resource_name, [])

    def device_states(self) -> List[DeviceState]:
        return [(d.id, d.healthy) for d in self._devices()]

    def GetPreferredAllocation(self, req, ctx):
        view = self._devices()
        withheld = {d.gpu_index for d in view if not d.healthy}
        resp = dp.PreferredAllocationResponse()
        for cr in req.container_requests:
            ids = preferred_partitions(view, list(cr.must_include_deviceIDs), list(cr.available_deviceIDs),
                                       int(cr.allocation_size), withheld)
            resp.container_responses.add(deviceIDs=ids)
        return resp

    def Allocate(self, req, ctx):
        """A partition: ``/dev/kfd`` + its own render node.  A CU-mask slice of an SPX GPU: its
        GPU's render node + ``HSA_CU_MASK`` (the slice's CU set, every queue of the container) +
        the HBM budget (``NOS_HBM_LIMIT_BYTES`` and the ``LD_PRELOAD`` limiter), as the CU-mask
        slice plugin serves ``amd.com/gpu-<c>cu.<m>gb``; a whole-GPU slice needs no mask."""
        import grpc
        by_id = {d.id: d for d in self._devices()}
        resp = dp.AllocateResponse()
        for cr in req.container_requests:
            car = resp.container_responses.add()
            nodes = []
            cus: List[int] = []
            hbm = 0
            gpus = set()
            for did in cr.devicesIDs:
                d = by_id.get(did)
                if d is None or not d.healthy:
                    msg = f"partition {did} is not allocatable ({'unknown' if d is None else d.reason})"
                    if ctx is not None:
                        ctx.abort(grpc.StatusCode.FAILED_PRECONDITION, msg)
                    raise KeyError(msg)
                if d.render_minor >= 0:
                    nodes.append(f"/dev/dri/renderD{d.render_minor}")
                if d.sliced:
                    cus.extend(d.cus)
                    hbm += d.hbm_bytes
                    gpus.add(d.gpu_index)
            if len(gpus) > 1:
                msg = f"slices {list(cr.devicesIDs)} span GPUs {sorted(gpus)}: one CU mask covers one GPU"
                if ctx is not None:
                    ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, msg)
                raise ValueError(msg)
            car.envs["NOS_PARTITION_IDS"] = ",".join(cr.devicesIDs)
            if cus and len(set(cus)) < self.cu_count:
                car.envs[constant.ENV_HSA_CU_MASK] = hsa_cu_mask(cus, 0)
            if cus:
                car.envs[constant.ENV_HBM_LIMIT] = str(hbm)
                car.envs["NOS_SLICE_IDS"] = ",".join(cr.devicesIDs)
                if self.shim_present is None or self.shim_present():
                    car.envs["LD_PRELOAD"] = self.shim_path
                    car.mounts.add(container_path=self.shim_path, host_path=self.shim_path, read_only=True)
                else:
                    # a bind mount of a missing host file fails the container's creation: start the
                    # pod without the in-process limiter (the HBM guard still polices its budget)
                    log.warning("HBM-limit shim %s is missing on this node: slices %s start without it",
                                self.shim_path, list(cr.devicesIDs))
            car.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
            for n in sorted(set(nodes)):
                car.devices.add(container_path=n, host_path=n, permissions="rw")
        return resp


def partition_plugin_manager(state: PartitionState, socket_dir: str = DEVICE_PLUGIN_DIR,
                             kubelet_socket: str = KUBELET_SOCKET, shim_path: str = "/usr/lib/nos/libnos_hbmlimit.so",
                             shim_present: Optional[Callable[[], bool]] = None, **kw: Any) -> PluginManager:
    """A :class:`PluginManager` over the partition view: one plugin per resource name present (a
    flip to a mode never served before registers its resource on the next sync)."""
    return PluginManager(None, socket_dir=socket_dir, kubelet_socket=kubelet_socket,
                         resources=lambda: sorted(state.view()),
                         factory=lambda r: PartitionDevicePlugin(r, state, socket_dir, shim_path=shim_path,
                                                                 shim_present=shim_present), **kw)


class AllocatablePublisher:
    """Patches the node's ``status.allocatable`` when the healthy partition counts of a view DROP
    (a drain starting, a flip taking partitions away, a GPU lost): kubelet's own node-status sync
    runs every 10 s, and a scheduler reading the stale, higher count would bind pods that kubelet
    then rejects at admission. Increases are left to kubelet, which publishes a resource only once
    its device manager holds the devices: published first by the agent, a partition kubelet has
    not yet received through ListAndWatch would be bound and then fail admission
    (``UnexpectedAdmissionError``; found by ``tests/test_e2e_processes.py::test_churn_soak_over_processes``)."""

    def __init__(self, client: Any, node: str):
        self.client = client
        self.node = node
        self.patches = 0

    def publish(self, view: Mapping[str, List[PartitionDevice]]) -> bool:
        healthy = {r: sum(1 for d in ds if d.healthy) for r, ds in view.items()}
        try:
            cur = (self.client.get("Node", self.node).get("status") or {}).get("allocatable") or {}
        except Exception as e:  # noqa: BLE001 - kubelet's own sync still gets there
            log.warning("node %s unavailable for the allocatable update: %s", self.node, e)
            return False
        want: Dict[str, str] = {}
        for r, v in cur.items():
            if not (r.startswith(constant.AMD_RESOURCE_PREFIX) and _is_partition_resource(r)):
                continue
            # only decreases: a resource no longer served drops to 0 (kubelet keeps a registered
            # resource at 0), fewer healthy partitions lower it; more are kubelet's to publish
            n = healthy.get(r, 0)
            try:
                if n < int(v):
                    want[r] = str(n)
            except ValueError:
                want[r] = str(n)
        if not want:
            return False
        self.client.patch("Node", self.node, {"status": {"allocatable": want}})
        self.patches += 1
        return True


def _is_partition_resource(r: str) -> bool:
    from ..models.xcp.profile import is_xcp_resource
    return is_xcp_resource(r)


class PartitionPluginHook:
    """The partition agent's device-plugin hook (``Actuator._reregister`` calls ``restart``): sync
    the plugins — a pushed ListAndWatch update, no pod restart — and publish the allocatable."""

    def __init__(self, manager: PluginManager, state: PartitionState,
                 publisher: Optional[AllocatablePublisher] = None):
        self.manager = manager
        self.state = state
        self.publisher = publisher

    def restart(self, node: str = "", timeout: float = 60.0) -> None:
        """Never raises: it runs after a flip has committed, and a kubelet that is restarting (its
        registration failing) must not keep the actuator from clearing its journal; one
        registration attempt here, the periodic sync (``run_forever``) retries."""
        try:
            self.manager.sync(attempts=1)
        except Exception as e:  # noqa: BLE001 - retried by the periodic sync
            log.warning("device plugin sync after the change failed (retried by the periodic sync): %s", e)
        finally:
            if self.publisher is not None:
                self.publisher.publish(self.state.view())

    def reconcile(self, req: Any) -> Any:
        """Controller entry point: the node's annotations changed (a new spec = a drain starts, a new
        status = a flip committed)."""
        from ..kube.runtime import Result
        self.restart()
        return Result()
