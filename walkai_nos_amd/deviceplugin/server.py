"""nos device plugin for MI355X slices and partitions (kubelet device-plugin API v1beta1).

The reference relies on the NVIDIA device plugin and restarts its pod after every MIG change
(``pkg/gpu/client.go``).  BASELINE.json asks for "no nvidia-device-plugin": compute partitions are
served by the AMD k8s-device-plugin (restarted the same way), and CU-mask slices — which no
upstream plugin knows — are served by this plugin:

* one gRPC ``DevicePlugin`` server per resource name (``amd.com/gpu-<profile>``) on a unix socket
  in ``/var/lib/kubelet/device-plugins/``, registered with kubelet's ``Registration`` service;
* ``ListAndWatch`` streams the slices of the :class:`SliceStore` and re-sends whenever the slice
  agent changes it (no plugin restart needed: the change is pushed);
* ``Allocate`` returns, for the allocated slice, ``HSA_CU_MASK`` (its XCD-symmetric CU rows, or the
  shared pool for memory-only slices), ``NOS_HBM_LIMIT_BYTES`` + ``LD_PRELOAD`` of the HBM-budget
  shim, and the ``/dev/kfd`` + render-node device specs of its GPU;
* ``GetPreferredAllocation`` keeps a request on **one GPU** (a container's ``HSA_CU_MASK`` and HBM
  budget describe one device), choosing, among the GPUs that can serve all of it, the one with
  the most slices already in use (packing keeps other GPUs idle so they can be re-sliced);
* ``Allocate`` rejects a request whose slices span GPUs instead of merging CU ids of different
  GPUs into one mask.
"""
from __future__ import annotations

import logging
import os
import threading

from concurrent import futures
from typing import Dict, List, Optional

import grpc

from .. import constant
from ..device.protos import dp
from ..device.slicing_client import SliceStore
from ..models.slicing.cumask import cus_of, hsa_cu_mask
from ..models.slicing.profile import as_resource_name

log = logging.getLogger("nos.deviceplugin")

DEVICE_PLUGIN_DIR = "/var/lib/kubelet/device-plugins"
KUBELET_SOCKET = os.path.join(DEVICE_PLUGIN_DIR, "kubelet.sock")


def preferred_same_gpu(must: List[str], available: List[str], size: int, gpu_of: Dict[str, int],
                       total: Dict[int, int]) -> List[str]:
    """``size`` ids including ``must``, all on one GPU when any GPU can serve the request: the GPU
    of the must-include ids if there are any, else the GPU with the most slices in use (``total``
    advertised minus available), ties to the lower index; within it, ids in sorted order.  When no
    single GPU has enough, fall back to sorted first-fit (``Allocate`` will then refuse)."""
    avail_by_gpu: Dict[int, List[str]] = {}
    for i in sorted(available):
        avail_by_gpu.setdefault(gpu_of.get(i, -1), []).append(i)
    must_gpus = {gpu_of.get(i, -1) for i in must}
    cands = sorted(avail_by_gpu, key=lambda g: (-(total.get(g, 0) - len(avail_by_gpu[g])), g))
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


class SliceDevicePlugin:
    """Serves one resource name backed by the node's slice store."""

    def __init__(self, resource_name: str, store: SliceStore, gpu_render_nodes: Dict[int, str],
                 cu_count: int = 256, shim_path: str = "/usr/lib/nos/libnos_hbmlimit.so",
                 socket_dir: str = DEVICE_PLUGIN_DIR, poll_interval: float = 1.0):
        self.resource_name = resource_name
        self.store = store
        self.render = gpu_render_nodes
        self.cu_count = cu_count
        self.shim_path = shim_path
        self.socket = os.path.join(socket_dir, "nos-" + resource_name.replace("/", "_") + ".sock")
        self.poll_interval = poll_interval
        self._server: Optional[grpc.Server] = None
        self._stop = threading.Event()
        self._changed = threading.Condition()
        self._version = 0

    # -- device view ------------------------------------------------------------------------
    def devices(self) -> List[str]:
        return [s.id for _, ss in sorted(self.store.load().items()) for s in ss
                if as_resource_name(s.profile) == self.resource_name]

    def notify(self) -> None:
        with self._changed:
            self._version += 1
            self._changed.notify_all()

    # -- gRPC handlers ------------------------------------------------------------------------
    def GetDevicePluginOptions(self, req, ctx):
        return dp.DevicePluginOptions(pre_start_required=False, get_preferred_allocation_available=True)

    def ListAndWatch(self, req, ctx):
        last: Optional[List[str]] = None
        while not self._stop.is_set() and (ctx is None or ctx.is_active()):
            cur = self.devices()
            if cur != last:
                yield dp.ListAndWatchResponse(devices=[dp.Device(ID=i, health=dp.HEALTHY) for i in cur])
                last = cur
            with self._changed:
                self._changed.wait(self.poll_interval)

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
        resp = dp.AllocateResponse()
        for cr in req.container_requests:
            car = resp.container_responses.add()
            cus: List[int] = []
            hbm = 0
            gpus = set()
            for did in cr.devicesIDs:
                if did not in by_id:
                    if ctx is not None:
                        ctx.abort(grpc.StatusCode.NOT_FOUND, f"unknown slice {did}")
                    raise KeyError(did)
                g, s = by_id[did]
                gpus.add(g)
                if len(gpus) > 1:
                    msg = f"slices {list(cr.devicesIDs)} span GPUs {sorted(gpus)}: one container's CU mask and HBM budget cover one GPU"
                    if ctx is not None:
                        ctx.abort(grpc.StatusCode.INVALID_ARGUMENT, msg)
                    raise ValueError(msg)
                cus.extend(cus_of(s, slices[g], self.cu_count))
                hbm += s.hbm_bytes
            car.envs[constant.ENV_HSA_CU_MASK] = hsa_cu_mask(cus, 0)
            car.envs[constant.ENV_HBM_LIMIT] = str(hbm)
            car.envs["LD_PRELOAD"] = self.shim_path
            car.envs["NOS_SLICE_IDS"] = ",".join(cr.devicesIDs)
            car.devices.add(container_path="/dev/kfd", host_path="/dev/kfd", permissions="rw")
            for g in sorted(gpus):
                node = self.render.get(g)
                if node:
                    car.devices.add(container_path=node, host_path=node, permissions="rw")
            car.mounts.add(container_path=self.shim_path, host_path=self.shim_path, read_only=True)
        return resp

    def PreStartContainer(self, req, ctx):
        return dp.PreStartContainerResponse()

    # -- lifecycle -----------------------------------------------------------------------------
    def serve(self) -> "SliceDevicePlugin":
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
        return self

    def register(self, kubelet_socket: str = KUBELET_SOCKET, timeout: float = 10.0) -> None:
        with grpc.insecure_channel("unix://" + kubelet_socket) as ch:
            stub = ch.unary_unary(f"/{dp.REGISTRATION_SERVICE}/Register",
                                  request_serializer=dp.RegisterRequest.SerializeToString,
                                  response_deserializer=dp.Empty.FromString)
            stub(dp.RegisterRequest(version=dp.VERSION, endpoint=os.path.basename(self.socket),
                                    resource_name=self.resource_name,
                                    options=dp.DevicePluginOptions(get_preferred_allocation_available=True)),
                 timeout=timeout)

    def stop(self) -> None:
        self._stop.set()
        self.notify()
        if self._server is not None:
            self._server.stop(grace=None)
            self._server = None


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


class PluginManager:
    """Keeps one :class:`SliceDevicePlugin` per resource name present in the store."""

    def __init__(self, store: SliceStore, gpu_render_nodes: Dict[int, str], socket_dir: str = DEVICE_PLUGIN_DIR,
                 kubelet_socket: str = KUBELET_SOCKET, cu_count: int = 256,
                 shim_path: str = "/usr/lib/nos/libnos_hbmlimit.so"):
        self.store = store
        self.render = gpu_render_nodes
        self.socket_dir = socket_dir
        self.kubelet_socket = kubelet_socket
        self.cu_count = cu_count
        self.shim_path = shim_path
        self.plugins: Dict[str, SliceDevicePlugin] = {}

    def sync(self) -> None:
        wanted = {as_resource_name(s.profile) for ss in self.store.load().values() for s in ss}
        for r in sorted(wanted - set(self.plugins)):
            p = SliceDevicePlugin(r, self.store, self.render, self.cu_count, self.shim_path, self.socket_dir).serve()
            p.register(self.kubelet_socket)
            self.plugins[r] = p
        for p in self.plugins.values():
            p.notify()

    def stop(self) -> None:
        for p in self.plugins.values():
            p.stop()
        self.plugins.clear()


def render_nodes_from_sysfs() -> Dict[int, str]:
    """GPU index -> /dev/dri/renderD<N> (best effort, ordered by render minor)."""
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
        except Exception as e:  # noqa: BLE001
            log.warning("device plugin sync failed: %s", e)
        stop.wait(interval)
    manager.stop()



