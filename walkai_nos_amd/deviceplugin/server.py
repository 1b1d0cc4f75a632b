"""nos device plugins for MI355X slices and partitions (kubelet device-plugin API v1beta1).

The reference relies on the NVIDIA device plugin and restarts its pod after every MIG change
(``pkg/gpu/client.go``).  BASELINE.json asks for "no nvidia-device-plugin": both kinds of MI355X
capacity are served by nos's own plugins, which push changes instead of being restarted:

* :class:`SliceDevicePlugin` — CU-mask slices (``amd.com/gpu-<profile>``) of the slice store;
* :class:`~walkai_nos_amd.deviceplugin.partitions.PartitionDevicePlugin` — compute partitions
  (``amd.com/<mode>_<nps>``) of the device map, withholding the free partitions of a GPU that is
  being re-partitioned (the drain), see that module.

Common to both (:class:`PluginServer`):

* one gRPC ``DevicePlugin`` server per resource name on a unix socket in
  ``/var/lib/kubelet/device-plugins/``, registered with kubelet's ``Registration`` service —
  with retries and exponential back-off (kubelet may be restarting);
* ``ListAndWatch`` streams ``(id, health)`` and re-sends whenever the view changes (``notify``,
  or the poll interval);
* **kubelet restarts**: kubelet deletes every socket in the plugin directory and recreates
  ``kubelet.sock`` when it starts; :class:`PluginManager` notices (its socket file gone, or
  ``kubelet.sock`` with a new inode) and serves + registers the plugin again.

Slices: ``Allocate`` returns ``HSA_CU_MASK`` (the slice's XCD-symmetric CU rows, or the shared
pool for memory-only slices), ``NOS_HBM_LIMIT_BYTES`` + ``LD_PRELOAD`` of the HBM-budget shim and
the ``/dev/kfd`` + render-node device specs of its GPU, the render node taken from the device map
(the GPU's BDF is the slice id's prefix) rather than from ``/dev/dri`` listing order;
``GetPreferredAllocation`` keeps a request on one GPU, the most-used one; a slice whose GPU left the
device map is reported ``Unhealthy``.
"""
from __future__ import annotations

import logging
import os
import threading
import time
from concurrent import futures
from typing import Any, Callable, Dict, List, Optional, Tuple

import grpc

from .. import constant
from ..device.protos import dp
from ..device.slicing_client import SliceStore
from ..models.slicing.cumask import Slice, cus_of, hsa_cu_mask
from ..models.slicing.profile import as_resource_name, extract_gpu_id
from .startgate import StartGate

log = logging.getLogger("nos.deviceplugin")

DEVICE_PLUGIN_DIR = "/var/lib/kubelet/device-plugins"
KUBELET_SOCKET = os.path.join(DEVICE_PLUGIN_DIR, "kubelet.sock")

DeviceState = Tuple[str, bool]  # (device id, healthy)


def preferred_same_gpu(must: List[str], available: List[str], size: int, gpu_of: Dict[str, int],
                       total: Dict[int, int], avoid: Optional[set] = None) -> List[str]:
    """``size`` ids including ``must``, all on one GPU when any GPU can serve the request: the GPU
    of the must-include ids if there are any, else the GPU with the most devices in use (``total``
    advertised minus available), ties to the lower index, GPUs in ``avoid`` last; within it, ids in
    sorted order.  When no single GPU has enough, fall back to sorted first-fit (``Allocate`` will
    then refuse)."""
    avoid = avoid or set()
    avail_by_gpu: Dict[int, List[str]] = {}
    for i in sorted(available):
        avail_by_gpu.setdefault(gpu_of.get(i, -1), []).append(i)
    must_gpus = {gpu_of.get(i, -1) for i in must}
    cands = sorted(avail_by_gpu, key=lambda g: (g in avoid, -(total.get(g, 0) - len(avail_by_gpu[g])), g))
    if must_gpus:
        cands = [g for g in cands if g in must_gpus] if len(must_gpus) == 1 else []
    for g in cands:
        pick = list(must) + [i for i in avail_by_gpu[g] if i not in must]
        if len(pick) >= size:
            return pick[:size]
    ids = list(must)
    for i in sorted(available):
        if len(ids) >= size:
            break
        if i not in ids:
            ids.append(i)
    return ids


class PluginServer:
    """gRPC plumbing of one device plugin (one resource name); subclasses provide the view."""

    def __init__(self, resource_name: str, socket_dir: str = DEVICE_PLUGIN_DIR, poll_interval: float = 1.0,
                 prefix: str = "nos-"):
        self.resource_name = resource_name
        self.socket = os.path.join(socket_dir, prefix + resource_name.replace("/", "_") + ".sock")
        self.poll_interval = poll_interval
        self._server: Optional[grpc.Server] = None
        self._stop = threading.Event()
        self._changed = threading.Condition()
        self._version = 0
        self.registered_inode: Optional[int] = None   # kubelet.sock inode at our last registration
        self.registrations = 0

    # -- view (subclasses) -------------------------------------------------------------------
    def device_states(self) -> List[DeviceState]:
        raise NotImplementedError

    def devices(self) -> List[str]:
        return [i for i, _ in self.device_states()]

    def healthy_devices(self) -> List[str]:
        return [i for i, ok in self.device_states() if ok]

    def notify(self) -> None:
        with self._changed:
            self._version += 1
            self._changed.notify_all()

    #: kubelet calls PreStartContainer before each container of this resource starts
    pre_start_required = False

    def options(self) -> Any:
        return dp.DevicePluginOptions(pre_start_required=self.pre_start_required,
                                      get_preferred_allocation_available=True)

    # -- gRPC handlers -------------------------------------------------------------------------
    def GetDevicePluginOptions(self, req, ctx):
        return self.options()

    def ListAndWatch(self, req, ctx):
        last: Optional[List[DeviceState]] = None
        while not self._stop.is_set() and (ctx is None or ctx.is_active()):
            cur = self.device_states()
            if cur != last:
                yield dp.ListAndWatchResponse(devices=[dp.Device(ID=i, health=dp.HEALTHY if ok else dp.UNHEALTHY)
                                                       for i, ok in cur])
                last = cur
            with self._changed:
                self._changed.wait(self.poll_interval)

    def PreStartContainer(self, req, ctx):
        return dp.PreStartContainerResponse()

    def GetPreferredAllocation(self, req, ctx):  # pragma: no cover - overridden
        raise NotImplementedError

    def Allocate(self, req, ctx):  # pragma: no cover - overridden
        raise NotImplementedError

    # -- lifecycle -----------------------------------------------------------------------------
    def serving(self) -> bool:
        return self._server is not None and os.path.exists(self.socket)

    def serve(self) -> "PluginServer":
        if self._server is not None:
            self._server.stop(grace=None)
            self._server = None
        h = grpc.method_handlers_generic_handler(dp.SERVICE, {
            "GetDevicePluginOptions": grpc.unary_unary_rpc_method_handler(
                self.GetDevicePluginOptions, dp.Empty.FromString, dp.DevicePluginOptions.SerializeToString),
            "ListAndWatch": grpc.unary_stream_rpc_method_handler(
                self.ListAndWatch, dp.Empty.FromString, dp.ListAndWatchResponse.SerializeToString),
            "GetPreferredAllocation": grpc.unary_unary_rpc_method_handler(
                self.GetPreferredAllocation, dp.PreferredAllocationRequest.FromString,
                dp.PreferredAllocationResponse.SerializeToString),
            "Allocate": grpc.unary_unary_rpc_method_handler(
                self.Allocate, dp.AllocateRequest.FromString, dp.AllocateResponse.SerializeToString),
            "PreStartContainer": grpc.unary_unary_rpc_method_handler(
                self.PreStartContainer, dp.PreStartContainerRequest.FromString,
                dp.PreStartContainerResponse.SerializeToString),
        })
        srv = grpc.server(futures.ThreadPoolExecutor(max_workers=8))
        srv.add_generic_rpc_handlers((h,))
        if os.path.exists(self.socket):
            os.unlink(self.socket)
        srv.add_insecure_port("unix://" + self.socket)
        srv.start()
        self._server = srv
        self._stop.clear()
        return self

    def register(self, kubelet_socket: str = KUBELET_SOCKET, timeout: float = 10.0, attempts: int = 5,
                 backoff: float = 0.5, sleep: Callable[[float], None] = time.sleep) -> None:
        """Register with kubelet, retrying with exponential back-off (kubelet may be restarting);
        raises the last error when every attempt failed."""
        last: Optional[Exception] = None
        for k in range(max(1, attempts)):
            try:
                with grpc.insecure_channel("unix://" + kubelet_socket) as ch:
                    stub = ch.unary_unary(f"/{dp.REGISTRATION_SERVICE}/Register",
                                          request_serializer=dp.RegisterRequest.SerializeToString,
                                          response_deserializer=dp.Empty.FromString)
                    stub(dp.RegisterRequest(version=dp.VERSION, endpoint=os.path.basename(self.socket),
                                            resource_name=self.resource_name, options=self.options()),
                         timeout=timeout)
                self.registered_inode = _inode(kubelet_socket)
                self.registrations += 1
                return
            except grpc.RpcError as e:
                last = e
                log.warning("registering %s with kubelet failed (attempt %d/%d): %s", self.resource_name, k + 1,
                            attempts, getattr(e, "details", lambda: e)())
                if k + 1 < attempts:
                    sleep(backoff * (2 ** k))
        raise RuntimeError(f"unable to register {self.resource_name} with kubelet: {last}")

    def stop(self) -> None:
        self._stop.set()
        self.notify()
        if self._server is not None:
            self._server.stop(grace=None)
            self._server = None


def _inode(path: str) -> Optional[int]:
    try:
        return os.stat(path).st_ino
    except OSError:
        return None


class SliceDevicePlugin(PluginServer):
    """Serves one CU-mask slice resource name backed by the node's slice store.

    ``gpu_render_nodes``: GPU index -> render node, the fallback when no ``device_map`` is given;
    ``device_map``: callable returning the node's :class:`~walkai_nos_amd.device.topology.DeviceMap`
    — the render node of a slice is its GPU's (looked up by the BDF in the slice id), and a slice
    whose GPU is not in the map is ``Unhealthy``."""

    def __init__(self, resource_name: str, store: SliceStore, gpu_render_nodes: Dict[int, str],
                 cu_count: int = 256, shim_path: str = "/usr/lib/nos/libnos_hbmlimit.so",
                 socket_dir: str = DEVICE_PLUGIN_DIR, poll_interval: float = 1.0,
                 device_map: Optional[Callable[[], Any]] = None, shared_hw_queues: int = -1,
                 start_gate: Optional[StartGate] = None):
        super().__init__(resource_name, socket_dir, poll_interval)
        self.store = store
        self.render = gpu_render_nodes
        self.cu_count = cu_count
        self.shim_path = shim_path
        self.device_map = device_map
        self.shared_hw_queues = shared_hw_queues
        #: memory-only containers of one GPU start one after another (deviceplugin/startgate.py)
        self.start_gate = start_gate
        self.pre_start_required = start_gate is not None

    # -- device view ------------------------------------------------------------------------
    def _map(self) -> Any:
        if self.device_map is None:
            return None
        try:
            return self.device_map()
        except Exception as e:  # noqa: BLE001 - an unreadable map marks nothing healthy by mistake
            log.warning("device map unavailable: %s", e)
            return None

    def device_states(self) -> List[DeviceState]:
        m = self._map()
        out = []
        for _, ss in sorted(self.store.load().items()):
            for s in ss:
                if as_resource_name(s.profile) != self.resource_name:
                    continue
                ok = True
                if self.device_map is not None:
                    ok = m is not None and m.lookup(extract_gpu_id(s.id)) is not None
                out.append((s.id, ok))
        return out

    def render_node(self, gpu: int, slice_id: str, m: Any = None) -> Optional[str]:
        if self.device_map is not None:
            m = m if m is not None else self._map()
            d = m.lookup(extract_gpu_id(slice_id)) if m is not None else None
            if d is not None and d.render_minor >= 0:
                return f"/dev/dri/renderD{d.render_minor}"
        return self.render.get(gpu)

    def shared_queues(self, mine: List[Slice], slices: Dict[int, List[Slice]]) -> int:
        """``GPU_MAX_HW_QUEUES`` for a memory-only slice (0 = leave HIP's default). Memory-only pods
        share every CU and dispatch is arbitrated per hardware pipe, so the queue count decides the
        split (measured, ``profiles/fairness_r4_repeat.json``: per-pod max/min at 3 / 5 / 7 pods —
        one queue 1.8 / 1.2-1.5 / 1.1-1.2, two queues 1.0-1.05 / 2.0-2.4 / 2.0, HIP's four 1.1 /
        1.7-2.0 / 1.9-2.2). Auto (-1): two queues while at most 3 memory-only slices share the GPU,
        one beyond."""
        if self.shared_hw_queues >= 0:
            return self.shared_hw_queues
        gpu = next((g for g, ss in slices.items() if any(s.id == mine[0].id for s in ss)), None) if mine else None
        n = sum(1 for s in slices.get(gpu, []) if not s.rows)
        return 2 if n <= 3 else 1

    def PreStartContainer(self, req, ctx):
        """Memory-only slices pass the start gate of their GPU: the container starts once the
        previous memory-only container of that GPU has its compute queues (or the gate's timeout);
        dedicated-CU slices start at once."""
        if self.start_gate is not None:
            slices = self.store.load()
            by_id = {s.id: (g, s) for g, ss in slices.items() for s in ss}
            mine = [by_id[d] for d in req.devicesIDs if d in by_id]
            if mine and all(not s.rows for _, s in mine):
                self.start_gate.enter(mine[0][0], [s.id for _, s in mine], bdf=extract_gpu_id(mine[0][1].id))
        return dp.PreStartContainerResponse()

    def GetPreferredAllocation(self, req, ctx):
        gpu_of = {s.id: g for g, ss in self.store.load().items() for s in ss}
        total: Dict[int, int] = {}
        for i in self.devices():
            total[gpu_of.get(i, -1)] = total.get(gpu_of.get(i, -1), 0) + 1
        resp = dp.PreferredAllocationResponse()
        for cr in req.container_requests:
            ids = preferred_same_gpu(list(cr.must_include_deviceIDs), list(cr.available_deviceIDs),
                                     int(cr.allocation_size), gpu_of, total)
            resp.container_responses.add(deviceIDs=ids)
        return resp

    def Allocate(self, req, ctx):
        slices = self.store.load()
        by_id = {s.id: (g, s) for g, ss in slices.items() for s in ss}
        m = self._map()
        resp = dp.AllocateResponse()
        for cr in req.container_requests:
            car = resp.container_responses.add()
            cus: List[int] = []
            hbm = 0
            gpus: Dict[int, str] = {}
            shared = True
            for did in cr.devicesIDs:
                if did not in by_id:
                    if ctx is not None:
                        ctx.abort(grpc.StatusCode.NOT_FOUND, f"unknown slice {did}")
                    raise KeyError(did)
                g, s = by_id[did]
                gpus.setdefault(g, did)
                if len(gpus) > 1:
                    msg = f"slices {list(cr.devicesIDs)} span GPUs {sorted(gpus)}: one container's CU mask and HBM budget cover one GPU"
                    if ctx is not None:
                        ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, msg)
                    raise ValueError(msg)
                cus.extend(cus_of(s, slices[g], self.cu_count))
                hbm += s.hbm_bytes
                shared = shared and not s.rows
            car.envs[constant.ENV_HSA_CU_MASK] = hsa_cu_mask(cus, 0)
            q = self.shared_queues([s for _, s in (by_id[d] for d in cr.devicesIDs)], slices) if shared else 0
            if q:
                car.envs[constant.ENV_GPU_MAX_HW_QUEUES] = str(q)
            car.envs[constant.ENV_HBM_LIMIT] = str(hbm)
            car.envs["LD_PRELOAD"] = self.shim_path
            car.envs["NOS_SLICE_IDS"] = ",".join(cr.devicesIDs)
            car.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
            for g, did in sorted(gpus.items()):
                node = self.render_node(g, did, m)
                if node:
                    car.devices.add(container_path=node, host_path=node, permissions="rw")
            car.mounts.add(container_path=self.shim_path, host_path=self.shim_path, read_only=True)
        return resp


class RegistrationServer:
    """kubelet's Registration endpoint (used by tests and the simulator)."""

    def __init__(self, socket: str):
        self.socket = socket
        self.registered: List[dp.RegisterRequest] = []
        self._server: Optional[grpc.Server] = None

    def _register(self, req, ctx):
        self.registered.append(req)
        return dp.Empty()

    def start(self) -> "RegistrationServer":
        h = grpc.method_handlers_generic_handler(dp.REGISTRATION_SERVICE, {
            "Register": grpc.unary_unary_rpc_method_handler(self._register, dp.RegisterRequest.FromString,
                                                            dp.Empty.SerializeToString)})
        srv = grpc.server(futures.ThreadPoolExecutor(max_workers=2))
        srv.add_generic_rpc_handlers((h,))
        if os.path.exists(self.socket):
            os.unlink(self.socket)
        srv.add_insecure_port("unix://" + self.socket)
        srv.start()
        self._server = srv
        return self

    def stop(self) -> None:
        if self._server is not None:
            self._server.stop(grace=None)
            self._server = None


class PluginManager:
    """Keeps one plugin server per resource name of a view, served and registered with kubelet.

    ``sync()`` (called periodically by :func:`run_forever`, and right after every change by the
    agents): starts a plugin for every new resource name, re-serves and re-registers a plugin whose
    socket disappeared or that registered with a previous kubelet (``kubelet.sock`` recreated =
    kubelet restarted), retries a failed registration on the next sync, and notifies every plugin
    so ``ListAndWatch`` streams the current view.  Resource names that disappear keep their
    (now empty) plugin: kubelet then reports zero capacity instead of a stale count.

    The default factory serves CU-mask slices of ``store``; the partition agent passes its own
    ``resources`` + ``factory`` (:mod:`walkai_nos_amd.deviceplugin.partitions`)."""

    def __init__(self, store: Optional[SliceStore], gpu_render_nodes: Optional[Dict[int, str]] = None,
                 socket_dir: str = DEVICE_PLUGIN_DIR, kubelet_socket: str = KUBELET_SOCKET, cu_count: int = 256,
                 shim_path: str = "/usr/lib/nos/libnos_hbmlimit.so", device_map: Optional[Callable[[], Any]] = None,
                 resources: Optional[Callable[[], List[str]]] = None,
                 factory: Optional[Callable[[str], PluginServer]] = None,
                 register_attempts: int = 5, register_backoff: float = 0.5, shared_hw_queues: int = -1,
                 start_gate: Optional[StartGate] = None):
        self.store = store
        self.shared_hw_queues = shared_hw_queues
        self.start_gate = start_gate   # one gate for every slice resource of the node
        self.render = gpu_render_nodes or {}
        self.socket_dir = socket_dir
        self.kubelet_socket = kubelet_socket
        self.cu_count = cu_count
        self.shim_path = shim_path
        self.device_map = device_map
        self.register_attempts = register_attempts
        self.register_backoff = register_backoff
        self._resources = resources or self._slice_resources
        self._factory = factory or self._slice_plugin
        self.plugins: Dict[str, PluginServer] = {}
        self._lock = threading.RLock()

    def _slice_resources(self) -> List[str]:
        return sorted({as_resource_name(s.profile) for ss in self.store.load().values() for s in ss})

    def _slice_plugin(self, r: str) -> PluginServer:
        return SliceDevicePlugin(r, self.store, self.render, self.cu_count, self.shim_path, self.socket_dir,
                                 device_map=self.device_map, shared_hw_queues=self.shared_hw_queues,
                                 start_gate=self.start_gate)

    def sync(self, attempts: Optional[int] = None) -> None:
        """``attempts``: registration attempts per plugin this call (default: the manager's); the
        agents' flip path passes 1 and leaves further retries to the periodic sync."""
        with self._lock:
            for r in self._resources():
                if r not in self.plugins:
                    self.plugins[r] = self._factory(r)
            kubelet = _inode(self.kubelet_socket)
            errors = []
            for r, p in sorted(self.plugins.items()):
                fresh = not p.serving()
                if fresh:
                    p.serve()
                if fresh or p.registered_inode is None or p.registered_inode != kubelet:
                    if p.registered_inode is not None and kubelet is not None and p.registered_inode != kubelet:
                        log.info("kubelet restarted (new %s): re-registering %s", self.kubelet_socket, r)
                    try:
                        p.register(self.kubelet_socket,
                                   attempts=self.register_attempts if attempts is None else attempts,
                                   backoff=self.register_backoff)
                    except RuntimeError as e:
                        p.registered_inode = None  # retried on the next sync
                        errors.append(str(e))
            for p in self.plugins.values():
                p.notify()
            if errors:
                raise RuntimeError("; ".join(errors))

    def restart(self, node_name: str = "", timeout: float = 60.0) -> None:
        """The agents' device-plugin hook after a change: no pod restart, just a pushed update (one
        registration attempt; a kubelet that is restarting is retried by :func:`run_forever`)."""
        self.sync(attempts=1)

    def stop(self) -> None:
        with self._lock:
            for p in self.plugins.values():
                p.stop()
            self.plugins.clear()


def render_nodes_from_sysfs() -> Dict[int, str]:
    """GPU index -> /dev/dri/renderD<N> by render minor order: only the fallback when no device map
    is available (the plugins map render nodes through ``DeviceMap``)."""
    d = "/dev/dri"
    if not os.path.isdir(d):
        return {}
    nodes = sorted((n for n in os.listdir(d) if n.startswith("renderD")), key=lambda n: int(n[7:]))
    return {i: os.path.join(d, n) for i, n in enumerate(nodes)}


def run_forever(manager: PluginManager, interval: float = 2.0, stop: Optional[threading.Event] = None) -> None:
    stop = stop or threading.Event()
    while not stop.is_set():
        try:
            manager.sync()
        except Exception as e:  # noqa: BLE001 - retried on the next tick
            log.warning("device plugin sync failed: %s", e)
        stop.wait(interval)
    manager.stop()
