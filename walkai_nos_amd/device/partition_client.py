"""Compute-partition client (the MIG client analogue, reference ``pkg/gpu/mig/client.go:28-174``).

``get_partition_devices`` = used devices (kubelet ``List``) ∪ (allocatable − used, marked free)
restricted to ``amd.com/<mode>_<nps>`` resources, each resolved to its physical GPU index through
the node's device map (``device/topology.py``: partition UUID, HIP UUID, render node or BDF ->
logical partition -> physical GPU).  A device the current map does not know — typically a
partition of the layout before a flip, still advertised until the device plugin re-registers — is
skipped, like the reference's NotFound path (``pkg/gpu/mig/client.go:141-174``).

Applying a geometry is a *mode flip* per physical GPU (``set_compute_partition``) — there are no
per-instance create/delete calls and no placement-order search on MI355X.
"""
from __future__ import annotations

import logging
import time
from typing import Dict, List, Optional

from ..models.device import STATUS_FREE, DeviceList, GpuDevice
from ..models.errors import GpuError
from ..models.xcp.profile import COMPUTE_MODES, extract_profile_name, is_xcp_resource, parse_profile
from ..utils.metrics import REGISTRY
from .amdsmi import AmdSmi
from .podresources import ResourceClient

log = logging.getLogger("nos.partition_client")


class PartitionClient:
    def __init__(self, resources: ResourceClient, smi: AmdSmi):
        self.resources = resources
        self.smi = smi

    def get_partition_devices(self) -> DeviceList:
        used = [d for d in self.resources.get_used_devices() if is_xcp_resource(d.resource_name)]
        alloc = [d for d in self.resources.get_allocatable_devices() if is_xcp_resource(d.resource_name)]
        used_ids = {d.device_id for d in used}
        out = DeviceList()
        for d in used:
            g = self._gpu_index(d.device_id)
            if g is not None:
                out.append(GpuDevice(d.resource_name, d.device_id, d.status, g))
        for d in alloc:
            if d.device_id in used_ids:
                continue
            g = self._gpu_index(d.device_id)
            if g is not None:
                out.append(GpuDevice(d.resource_name, d.device_id, STATUS_FREE, g))
        return out

    def _gpu_index(self, device_id: str) -> Optional[int]:
        try:
            return self.smi.gpu_index_of(device_id)
        except GpuError as e:
            if e.is_not_found():
                log.debug("device %s: GPU not found, skipping", device_id)
                return None
            raise

    def used_ids(self) -> set:
        """Device ids (partitions and slices) kubelet has allocated to running containers."""
        return {d.device_id for d in self.resources.get_used_devices() if is_xcp_resource(d.resource_name)}

    def pods_by_gpu(self) -> Dict[int, List[str]]:
        """Physical GPU index -> ``<ns>/<pod>`` of the pods using one of its partitions."""
        out: Dict[int, set] = {}
        for ns, pod, d in self.resources.get_used_devices_by_pod():
            if not is_xcp_resource(d.resource_name):
                continue
            g = self._gpu_index(d.device_id)
            if g is not None:
                out.setdefault(g, set()).add(f"{ns}/{pod}")
        return {g: sorted(v) for g, v in sorted(out.items())}

    def current_profiles(self) -> Dict[int, str]:
        """Physical GPU index -> current profile name (``<mode>_<nps>``) from the device map."""
        return self.smi.device_map().modes()

    def device_map(self):
        """The node's current physical <-> logical map (rebuilt by the backend after every flip)."""
        return self.smi.device_map()

    def set_profile(self, gpu_index: int, profile: str) -> None:
        """Flip one physical GPU to ``profile``'s compute mode (its NPS must already match)."""
        p = parse_profile(profile)
        cur_nps = self.smi.get_memory_partition(gpu_index).lower()
        if cur_nps != p.nps:
            raise GpuError(f"GPU {gpu_index} is in {cur_nps.upper()}, profile {profile} needs {p.nps.upper()}")
        if self.smi.get_compute_partition(gpu_index).lower() == p.mode:
            return
        t0 = time.perf_counter()
        self.smi.set_compute_partition(gpu_index, p.mode.upper())
        REGISTRY.phase_seconds.labels(phase="amdsmi_apply").observe(time.perf_counter() - t0)

    def set_memory_partition(self, nps: str) -> None:
        t0 = time.perf_counter()
        self.smi.set_memory_partition(nps.upper())
        REGISTRY.phase_seconds.labels(phase="amdsmi_apply").observe(time.perf_counter() - t0)

    def gpu_busy(self, gpu_index: int) -> bool:
        """Any process on any partition of the GPU (amd-smi process list)."""
        return self.smi.process_count(gpu_index) > 0


def profile_partitions(profile: str) -> int:
    return COMPUTE_MODES[parse_profile(profile).mode]


def extract_profile(resource_name: str) -> Optional[str]:
    return extract_profile_name(resource_name)
