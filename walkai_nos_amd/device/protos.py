"""Kubelet gRPC protocol messages built at runtime (no ``protoc`` in this environment).

* ``v1.PodResourcesLister`` (k8s.io/kubelet/pkg/apis/podresources/v1/api.proto) — ``List`` and
  ``GetAllocatableResources``, the two RPCs the reference agents call (``pkg/resource/client.go``,
  SURVEY Appendix A.7).  Only the fields nos reads are declared; unknown fields on the wire are
  skipped by protobuf, so a real kubelet's richer messages parse fine.
* ``v1beta1`` device-plugin API (k8s.io/kubelet/pkg/apis/deviceplugin/v1beta1/api.proto) —
  ``Registration.Register`` and the ``DevicePlugin`` service, used by the nos device plugin that
  advertises compute partitions and CU-mask slices.

Field numbers match the upstream .proto files.
"""
from __future__ import annotations

from typing import Dict, List, Tuple

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto
_T = {"string": F.TYPE_STRING, "int64": F.TYPE_INT64, "bool": F.TYPE_BOOL, "uint64": F.TYPE_UINT64,
      "int32": F.TYPE_INT32, "msg": F.TYPE_MESSAGE}

FieldSpec = Tuple[str, int, str, bool, str]  # name, number, type, repeated, message type name


def _file(name: str, package: str, messages: Dict[str, List[FieldSpec]], map_entries: Dict[str, Tuple[str, str]] | None = None):
    fd = descriptor_pb2.FileDescriptorProto(name=name, package=package, syntax="proto3")
    for mname, fields in messages.items():
        m = fd.message_type.add(name=mname)
        for fname, num, ftype, rep, tname in fields:
            f = m.field.add(name=fname, number=num, type=_T[ftype],
                            label=F.LABEL_REPEATED if rep else F.LABEL_OPTIONAL)
            if ftype == "msg":
                f.type_name = f".{package}.{tname}"
        for entry_field, (kt, vt) in (map_entries or {}).items():
            if not entry_field.startswith(mname + "."):
                continue
            fname = entry_field.split(".", 1)[1]
            entry_name = "".join(p.capitalize() for p in fname.split("_")) + "Entry"
            e = m.nested_type.add(name=entry_name)
            e.options.map_entry = True
            e.field.add(name="key", number=1, type=_T[kt], label=F.LABEL_OPTIONAL)
            e.field.add(name="value", number=2, type=_T[vt], label=F.LABEL_OPTIONAL)
    return fd


_pool = descriptor_pool.DescriptorPool()

_PODRES = _file("nos_podresources_v1.proto", "v1", {
    "NUMANode": [("ID", 1, "int64", False, "")],
    "TopologyInfo": [("nodes", 1, "msg", True, "NUMANode")],
    "ContainerDevices": [("resource_name", 1, "string", False, ""), ("device_ids", 2, "string", True, ""),
                         ("topology", 3, "msg", False, "TopologyInfo")],
    "ContainerResources": [("name", 1, "string", False, ""), ("devices", 2, "msg", True, "ContainerDevices"),
                           ("cpu_ids", 3, "int64", True, "")],
    "PodResources": [("name", 1, "string", False, ""), ("namespace", 2, "string", False, ""),
                     ("containers", 3, "msg", True, "ContainerResources")],
    "ListPodResourcesRequest": [],
    "ListPodResourcesResponse": [("pod_resources", 1, "msg", True, "PodResources")],
    "AllocatableResourcesRequest": [],
    "AllocatableResourcesResponse": [("devices", 1, "msg", True, "ContainerDevices"),
                                     ("cpu_ids", 2, "int64", True, "")],
})

_DP = _file("nos_deviceplugin_v1beta1.proto", "v1beta1", {
    "DevicePluginOptions": [("pre_start_required", 1, "bool", False, ""),
                            ("get_preferred_allocation_available", 2, "bool", False, "")],
    "RegisterRequest": [("version", 1, "string", False, ""), ("endpoint", 2, "string", False, ""),
                        ("resource_name", 3, "string", False, ""), ("options", 4, "msg", False, "DevicePluginOptions")],
    "Empty": [],
    "NUMANode": [("ID", 1, "int64", False, "")],
    "TopologyInfo": [("nodes", 1, "msg", True, "NUMANode")],
    "Device": [("ID", 1, "string", False, ""), ("health", 2, "string", False, ""),
               ("topology", 3, "msg", False, "TopologyInfo")],
    "ListAndWatchResponse": [("devices", 1, "msg", True, "Device")],
    "PreStartContainerRequest": [("devicesIDs", 1, "string", True, "")],
    "PreStartContainerResponse": [],
    "ContainerPreferredAllocationRequest": [("available_deviceIDs", 1, "string", True, ""),
                                            ("must_include_deviceIDs", 2, "string", True, ""),
                                            ("allocation_size", 3, "int32", False, "")],
    "PreferredAllocationRequest": [("container_requests", 1, "msg", True, "ContainerPreferredAllocationRequest")],
    "ContainerPreferredAllocationResponse": [("deviceIDs", 1, "string", True, "")],
    "PreferredAllocationResponse": [("container_responses", 1, "msg", True, "ContainerPreferredAllocationResponse")],
    "ContainerAllocateRequest": [("devicesIDs", 1, "string", True, "")],
    "AllocateRequest": [("container_requests", 1, "msg", True, "ContainerAllocateRequest")],
    "Mount": [("container_path", 1, "string", False, ""), ("host_path", 2, "string", False, ""),
              ("read_only", 3, "bool", False, "")],
    "DeviceSpec": [("container_path", 1, "string", False, ""), ("host_path", 2, "string", False, ""),
                   ("permissions", 3, "string", False, "")],
    "ContainerAllocateResponse": [("mounts", 2, "msg", True, "Mount"), ("devices", 3, "msg", True, "DeviceSpec")],
    "AllocateResponse": [("container_responses", 1, "msg", True, "ContainerAllocateResponse")],
}, map_entries={"ContainerAllocateResponse.envs": ("string", "string"),
                "ContainerAllocateResponse.annotations": ("string", "string")})

# map fields (envs = 1, annotations = 4) reference the nested entry types
_car = [m for m in _DP.message_type if m.name == "ContainerAllocateResponse"][0]
_car.field.add(name="envs", number=1, type=F.TYPE_MESSAGE, label=F.LABEL_REPEATED,
               type_name=".v1beta1.ContainerAllocateResponse.EnvsEntry")
_car.field.add(name="annotations", number=4, type=F.TYPE_MESSAGE, label=F.LABEL_REPEATED,
               type_name=".v1beta1.ContainerAllocateResponse.AnnotationsEntry")

_pool.Add(_PODRES)
_pool.Add(_DP)


def _cls(full: str):
    return message_factory.GetMessageClass(_pool.FindMessageTypeByName(full))


class podres:  # namespace for PodResources v1 messages
    ListPodResourcesRequest = _cls("v1.ListPodResourcesRequest")
    ListPodResourcesResponse = _cls("v1.ListPodResourcesResponse")
    AllocatableResourcesRequest = _cls("v1.AllocatableResourcesRequest")
    AllocatableResourcesResponse = _cls("v1.AllocatableResourcesResponse")
    PodResources = _cls("v1.PodResources")
    ContainerResources = _cls("v1.ContainerResources")
    ContainerDevices = _cls("v1.ContainerDevices")
    SERVICE = "v1.PodResourcesLister"


class dp:  # namespace for device-plugin v1beta1 messages
    VERSION = "v1beta1"
    DevicePluginOptions = _cls("v1beta1.DevicePluginOptions")
    RegisterRequest = _cls("v1beta1.RegisterRequest")
    Empty = _cls("v1beta1.Empty")
    Device = _cls("v1beta1.Device")
    ListAndWatchResponse = _cls("v1beta1.ListAndWatchResponse")
    PreStartContainerRequest = _cls("v1beta1.PreStartContainerRequest")
    PreStartContainerResponse = _cls("v1beta1.PreStartContainerResponse")
    PreferredAllocationRequest = _cls("v1beta1.PreferredAllocationRequest")
    PreferredAllocationResponse = _cls("v1beta1.PreferredAllocationResponse")
    ContainerPreferredAllocationResponse = _cls("v1beta1.ContainerPreferredAllocationResponse")
    AllocateRequest = _cls("v1beta1.AllocateRequest")
    AllocateResponse = _cls("v1beta1.AllocateResponse")
    ContainerAllocateResponse = _cls("v1beta1.ContainerAllocateResponse")
    DeviceSpec = _cls("v1beta1.DeviceSpec")
    Mount = _cls("v1beta1.Mount")
    REGISTRATION_SERVICE = "v1beta1.Registration"
    SERVICE = "v1beta1.DevicePlugin"
    HEALTHY = "Healthy"
    UNHEALTHY = "Unhealthy"
