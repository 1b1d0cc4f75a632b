"""Devices as seen by kubelet + the amd-smi backend.

Reference: ``pkg/resource/device.go:26-68`` (``Device{ResourceName, DeviceId, Status}`` with
status ``used|free|unknown``) and ``pkg/gpu/device.go:26-137`` (``gpu.Device`` adds the physical
GPU index; ``AsStatusAnnotation`` groups by GPU, resource and status — Appendix B.6).
"""
from __future__ import annotations

from collections import defaultdict
from dataclasses import dataclass
from typing import Callable, Dict, Iterable, Optional, Tuple

STATUS_USED = "used"
STATUS_FREE = "free"
STATUS_UNKNOWN = "unknown"
_STATUSES = (STATUS_USED, STATUS_FREE, STATUS_UNKNOWN)


def parse_status(s: str) -> str:
    v = s.lower()
    if v not in _STATUSES:
        raise ValueError(f"invalid device status {s!r}")
    return v


@dataclass(frozen=True)
class Device:
    resource_name: str
    device_id: str
    status: str = STATUS_UNKNOWN

    def is_used(self) -> bool:
        return self.status == STATUS_USED

    def is_free(self) -> bool:
        return self.status == STATUS_FREE


@dataclass(frozen=True)
class GpuDevice:
    resource_name: str
    device_id: str
    status: str
    gpu_index: int

    def is_used(self) -> bool:
        return self.status == STATUS_USED

    def is_free(self) -> bool:
        return self.status == STATUS_FREE

    def full_resource_name(self) -> str:
        return self.resource_name


class DeviceList(list):
    """``List[GpuDevice]`` with the grouping helpers of ``gpu.DeviceList``."""

    def get_used(self) -> "DeviceList":
        return DeviceList(d for d in self if d.is_used())

    def get_free(self) -> "DeviceList":
        return DeviceList(d for d in self if d.is_free())

    def group_by_gpu_index(self) -> Dict[int, "DeviceList"]:
        out: Dict[int, DeviceList] = defaultdict(DeviceList)
        for d in self:
            out[d.gpu_index].append(d)
        return dict(out)

    def group_by_resource_name(self) -> Dict[str, "DeviceList"]:
        out: Dict[str, DeviceList] = defaultdict(DeviceList)
        for d in self:
            out[d.resource_name].append(d)
        return dict(out)

    def sort_by_device_id(self) -> "DeviceList":
        return DeviceList(sorted(self, key=lambda d: d.device_id))

    def as_status_annotation(self, profile_extractor: Callable[[str], Optional[str]]):
        """Appendix B.6: group by GPU, resource, status; quantity = count; keep only resources
        the extractor accepts (returns a profile name)."""
        from .annotation import StatusAnnotation

        counts: Dict[Tuple[int, str, str], int] = defaultdict(int)
        for d in self:
            profile = profile_extractor(d.resource_name)
            if profile is None:
                continue
            counts[(d.gpu_index, profile, d.status)] += 1
        return [StatusAnnotation(profile=p, index=i, status=s, quantity=q)
                for (i, p, s), q in sorted(counts.items())]


def devices(items: Iterable[GpuDevice]) -> DeviceList:
    return DeviceList(items)
