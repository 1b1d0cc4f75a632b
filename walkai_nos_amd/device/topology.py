"""Physical-GPU <-> logical-partition map of one node.

The reference never caches device state: NVML is initialised and shut down around every call
(ref ``pkg/gpu/nvml/client.go:46-57``) and devices are re-visited each time (``:449-511``).  On
MI355X that matters more than on MIG, because a compute-partition flip changes *what the devices
are*: in SPX amd-smi exposes one processor per GPU, in CPX eight, each with its own UUID, KFD
node, render node and HIP ordinal, while the PCI BDF stays the physical GPU's (the partition id
lives in bits [31:28] of the KFD ``location_id``, ``amdsmi.h`` ``amdsmi_get_gpu_bdf_id``).

:class:`DeviceMap` is one enumeration of that state:

* every processor amd-smi reports becomes a :class:`LogicalDevice`;
* processors are grouped into physical GPUs by BDF (sorted, so GPU indexes are stable across
  flips — a flip never moves a GPU on the PCI bus);
* the partition index is the KFD ``current_partition_id`` when the driver reports one, else the
  location-id partition bits, else the order inside the group;
* every id a kubelet device plugin may advertise for a partition resolves to it: the partition
  UUID (the canonical id), the HIP UUID, ``renderD<minor>``, and for partition 0 the bare BDF
  (what device plugins use in SPX, and the prefix of CU-mask slice ids ``<bdf>::s<n>``).

Maps are immutable snapshots with a ``generation``; backends build a new one after every
partition change (see :class:`~walkai_nos_amd.device.amdsmi.AmdSmi`), so nothing downstream can
resolve an id against a layout that no longer exists.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, Iterable, List, Optional

from ..models.errors import GpuError

NO_PARTITION = 0xFFFFFFFF


@dataclass(frozen=True)
class ProcInfo:
    """One amd-smi processor (a whole GPU in SPX, one compute partition otherwise)."""
    ordinal: int                 # position in amd-smi's processor list
    uuid: str
    bdf: str                     # PCI address of the physical GPU, "dddd:bb:dd.f"
    bdf_id: int = 0              # KFD location id incl. partition bits [31:28]
    partition_id: int = NO_PARTITION
    kfd_node: int = -1
    hip_id: int = -1             # HIP ordinal in a process that sees every device of the node
    hip_uuid: str = ""
    render_minor: int = -1       # /dev/dri/renderD<minor>
    market_name: str = ""
    vram_bytes: int = 0
    cu_count: int = 0
    xcds: int = 0


@dataclass(frozen=True)
class GpuInfo:
    """One physical GPU of the node."""
    index: int
    uuid: str
    bdf: str
    model: str
    vram_bytes: int
    cu_count: int
    xcds: int = 8


@dataclass(frozen=True)
class LogicalDevice:
    """One logical GPU (a compute partition, or the whole GPU in SPX)."""
    gpu_index: int
    partition_index: int
    uuid: str
    bdf: str
    compute_mode: str
    memory_mode: str
    hip_id: int = -1
    render_minor: int = -1
    kfd_node: int = -1
    hip_uuid: str = ""
    cu_count: int = 0
    vram_bytes: int = 0
    proc_ordinal: int = -1

    @property
    def device_id(self) -> str:
        """Canonical kubelet device id of the partition (its amd-smi UUID)."""
        return self.uuid

    def aliases(self) -> List[str]:
        out = [self.uuid]
        if self.hip_uuid:
            out.append(self.hip_uuid)
        if self.render_minor >= 0:
            out.append(f"renderD{self.render_minor}")
        if self.partition_index == 0:
            out.append(self.bdf)
        return out


@dataclass
class DeviceMap:
    gpus: List[GpuInfo]
    devices: List[LogicalDevice]
    generation: int = 0
    _ids: Dict[str, LogicalDevice] = field(default_factory=dict, repr=False)

    def __post_init__(self) -> None:
        for d in self.devices:
            for a in d.aliases():
                self._ids.setdefault(a, d)

    # -- queries ---------------------------------------------------------------------------
    def lookup(self, device_id: str) -> Optional[LogicalDevice]:
        base = device_id.split("::", 1)[0]  # CU-mask slice / replica suffix (ref slicing/util.go:51-57)
        return self._ids.get(base)

    def resolve(self, device_id: str) -> LogicalDevice:
        d = self.lookup(device_id)
        if d is None:
            raise GpuError(f"device {device_id!r} not found on this node (layout generation {self.generation})",
                           GpuError.NOT_FOUND)
        return d

    def partitions_of(self, gpu_index: int) -> List[LogicalDevice]:
        return [d for d in self.devices if d.gpu_index == gpu_index]

    def primary(self, gpu_index: int) -> LogicalDevice:
        parts = self.partitions_of(gpu_index)
        if not parts:
            raise GpuError(f"GPU {gpu_index} not found", GpuError.NOT_FOUND)
        return parts[0]

    def hip_ids(self) -> List[int]:
        """HIP ordinals of every logical device (what a fresh process sees), ascending."""
        return sorted(d.hip_id for d in self.devices if d.hip_id >= 0)

    def modes(self) -> Dict[int, str]:
        out: Dict[int, str] = {}
        for d in self.devices:
            out.setdefault(d.gpu_index, f"{d.compute_mode.lower()}_{d.memory_mode.lower()}")
        return out

    def describe(self) -> List[Dict[str, object]]:
        return [{"gpu": d.gpu_index, "partition": d.partition_index, "uuid": d.uuid, "bdf": d.bdf,
                 "hip_id": d.hip_id, "render": d.render_minor, "kfd_node": d.kfd_node,
                 "mode": f"{d.compute_mode}/{d.memory_mode}", "cus": d.cu_count} for d in self.devices]


def build_device_map(procs: Iterable[ProcInfo], compute_mode_of, memory_mode_of, nps_of=None,
                     generation: int = 0) -> DeviceMap:
    """Group raw processors into physical GPUs.

    ``compute_mode_of(proc)`` / ``memory_mode_of(proc)`` read the (GPU-wide) modes through one
    processor of the group; ``nps_of(mode)`` gives the number of memory partitions of a memory
    mode (physical VRAM = partition-0 VRAM x NPS, since in NPS<n> a partition sees 1/n of HBM and
    in NPS1 every partition sees all of it)."""
    groups: Dict[str, List[ProcInfo]] = {}
    for p in procs:
        groups.setdefault(p.bdf.lower(), []).append(p)
    gpus: List[GpuInfo] = []
    devices: List[LogicalDevice] = []
    for gi, bdf in enumerate(sorted(groups)):
        members = groups[bdf]

        def part_key(p: ProcInfo):
            if p.partition_id != NO_PARTITION:
                return (0, p.partition_id, p.ordinal)
            return (1, (p.bdf_id >> 28) & 0xF, p.ordinal)
        members.sort(key=part_key)
        head = members[0]
        cm = compute_mode_of(head).upper()
        mm = memory_mode_of(head).upper()
        nps = nps_of(mm) if nps_of is not None else 1
        cus = sum(m.cu_count for m in members)
        xcds = sum(m.xcds for m in members) or 8
        gpus.append(GpuInfo(gi, head.uuid, head.bdf, head.market_name, head.vram_bytes * max(1, nps), cus, xcds))
        for k, m in enumerate(members):
            devices.append(LogicalDevice(gi, k, m.uuid, m.bdf, cm, mm, m.hip_id, m.render_minor, m.kfd_node,
                                         m.hip_uuid, m.cu_count, m.vram_bytes, m.ordinal))
    return DeviceMap(gpus, devices, generation)
