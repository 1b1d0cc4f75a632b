"""Kubelet PodResources client (reference ``pkg/resource/client.go:26-87``, ``lister.go:26-38``).

``get_used_devices`` = devices of running containers (``List``) with status ``used``;
``get_allocatable_devices`` = ``GetAllocatableResources`` with status ``unknown``.
gRPC over the kubelet unix socket with the reference defaults (10 s timeout, 16 MiB max message,
``pkg/constant/constants.go:87-90``).

Also provides :class:`PodResourcesServer`, a gRPC server speaking the same protocol, backed by a
callable — the fake kubelet of the simulator and of the integration tests, so the agent's real
client code path (socket, framing, protobuf) is exercised end to end.
"""
from __future__ import annotations

import os
import threading
from concurrent import futures
from typing import Callable, Iterable, List, Optional, Tuple

import grpc

from .. import constant
from ..models.device import STATUS_UNKNOWN, STATUS_USED, Device
from .protos import podres

# (resource_name, [device ids]) per container, per pod
UsedFn = Callable[[], List[Tuple[str, str, List[Tuple[str, List[str]]]]]]   # [(pod, ns, [(res, ids)])]
AllocFn = Callable[[], List[Tuple[str, List[str]]]]                          # [(res, ids)]


class ResourceClient:
    """Interface used by the partition / slicing clients."""

    def get_used_devices(self) -> List[Device]:
        raise NotImplementedError

    def get_allocatable_devices(self) -> List[Device]:
        raise NotImplementedError

    def get_used_devices_by_pod(self) -> List[Tuple[str, str, Device]]:
        """[(namespace, pod, device)] of running containers; empty when the source cannot tell."""
        return []


class PodResourcesClient(ResourceClient):
    def __init__(self, socket_path: str = constant.DEFAULT_POD_RESOURCES_SOCKET,
                 timeout: float = constant.DEFAULT_POD_RESOURCES_TIMEOUT_S,
                 max_msg_size: int = constant.DEFAULT_POD_RESOURCES_MAX_MSG_SIZE):
        self.timeout = timeout
        target = socket_path if socket_path.startswith("unix:") else "unix://" + os.path.abspath(socket_path)
        self._channel = grpc.insecure_channel(target, options=[("grpc.max_receive_message_length", max_msg_size)])
        self._list = self._channel.unary_unary(f"/{podres.SERVICE}/List",
                                               request_serializer=podres.ListPodResourcesRequest.SerializeToString,
                                               response_deserializer=podres.ListPodResourcesResponse.FromString)
        self._alloc = self._channel.unary_unary(f"/{podres.SERVICE}/GetAllocatableResources",
                                                request_serializer=podres.AllocatableResourcesRequest.SerializeToString,
                                                response_deserializer=podres.AllocatableResourcesResponse.FromString)

    def get_used_devices(self) -> List[Device]:
        resp = self._list(podres.ListPodResourcesRequest(), timeout=self.timeout)
        out: List[Device] = []
        for p in resp.pod_resources:
            for c in p.containers:
                for d in c.devices:
                    for i in d.device_ids:
                        out.append(Device(d.resource_name, i, STATUS_USED))
        return out

    def get_used_devices_by_pod(self) -> List[Tuple[str, str, Device]]:
        resp = self._list(podres.ListPodResourcesRequest(), timeout=self.timeout)
        return [(p.namespace, p.name, Device(d.resource_name, i, STATUS_USED))
                for p in resp.pod_resources for c in p.containers for d in c.devices for i in d.device_ids]

    def get_allocatable_devices(self) -> List[Device]:
        resp = self._alloc(podres.AllocatableResourcesRequest(), timeout=self.timeout)
        return [Device(d.resource_name, i, STATUS_UNKNOWN) for d in resp.devices for i in d.device_ids]

    def close(self) -> None:
        self._channel.close()


class StaticResourceClient(ResourceClient):
    """In-process client over callables (simulator / unit tests)."""

    def __init__(self, used: Callable[[], Iterable[Tuple[str, str]]], allocatable: Callable[[], Iterable[Tuple[str, str]]],
                 used_by_pod: Optional[Callable[[], Iterable[Tuple[str, str, str, str]]]] = None):
        self._used = used
        self._alloc = allocatable
        self._by_pod = used_by_pod    # -> [(namespace, pod, resource, id)]

    def get_used_devices(self) -> List[Device]:
        return [Device(r, i, STATUS_USED) for r, i in self._used()]

    def get_allocatable_devices(self) -> List[Device]:
        return [Device(r, i, STATUS_UNKNOWN) for r, i in self._alloc()]

    def get_used_devices_by_pod(self) -> List[Tuple[str, str, Device]]:
        if self._by_pod is None:
            return []
        return [(ns, p, Device(r, i, STATUS_USED)) for ns, p, r, i in self._by_pod()]


class PodResourcesServer:
    """A kubelet PodResources v1 endpoint on a unix socket."""

    def __init__(self, socket_path: str, used: UsedFn, allocatable: AllocFn):
        self.socket_path = socket_path
        self._used = used
        self._alloc = allocatable
        self._server: Optional[grpc.Server] = None
        self._lock = threading.Lock()

    def _list(self, req, ctx):
        resp = podres.ListPodResourcesResponse()
        for name, ns, devs in self._used():
            p = resp.pod_resources.add(name=name, namespace=ns)
            c = p.containers.add(name="main")
            for r, ids in devs:
                d = c.devices.add(resource_name=r)
                d.device_ids.extend(ids)
        return resp

    def _allocatable(self, req, ctx):
        resp = podres.AllocatableResourcesResponse()
        for r, ids in self._alloc():
            d = resp.devices.add(resource_name=r)
            d.device_ids.extend(ids)
        return resp

    def start(self) -> "PodResourcesServer":
        handlers = {
            "List": grpc.unary_unary_rpc_method_handler(
                self._list, request_deserializer=podres.ListPodResourcesRequest.FromString,
                response_serializer=podres.ListPodResourcesResponse.SerializeToString),
            "GetAllocatableResources": grpc.unary_unary_rpc_method_handler(
                self._allocatable, request_deserializer=podres.AllocatableResourcesRequest.FromString,
                response_serializer=podres.AllocatableResourcesResponse.SerializeToString),
        }
        srv = grpc.server(futures.ThreadPoolExecutor(max_workers=4))
        srv.add_generic_rpc_handlers((grpc.method_handlers_generic_handler(podres.SERVICE, handlers),))
        if os.path.exists(self.socket_path):
            os.unlink(self.socket_path)
        srv.add_insecure_port("unix://" + os.path.abspath(self.socket_path))
        srv.start()
        self._server = srv
        return self

    def stop(self) -> None:
        if self._server is not None:
            self._server.stop(grace=None)
            self._server = None
