"""Recording fakes of the device-side clients (reference ``pkg/test/mocks``: the hand-written MIG
client with call counters and canned returns, and the mockery-generated interfaces).

Each fake records every call in ``calls`` (name, args) and exposes per-method counters, and can be
told to fail the next N calls of a method, so controller tests assert on interactions instead of
on hardware state.
"""
from __future__ import annotations

from collections import Counter
from typing import Any, Dict, List, Optional, Tuple

from ..models.device import DeviceList
from ..models.errors import GpuError
from ..parallel.barrier import CommitBarrier


class _Recorder:
    def __init__(self) -> None:
        self.calls: List[Tuple[str, tuple]] = []
        self.counts: Counter = Counter()
        self._fail: Dict[str, int] = {}

    def fail_next(self, method: str, n: int = 1) -> None:
        self._fail[method] = self._fail.get(method, 0) + n

    def _record(self, method: str, *args: Any) -> None:
        self.calls.append((method, args))
        self.counts[method] += 1
        if self._fail.get(method, 0) > 0:
            self._fail[method] -= 1
            raise GpuError(f"injected failure in {method}", GpuError.GENERIC)


class MockPartitionClient(_Recorder):
    """Canned partition-client: ``devices`` is returned by ``get_partition_devices``; ``profiles``
    maps GPU index -> current profile and is updated by ``set_profile``."""

    def __init__(self, devices: Optional[DeviceList] = None, profiles: Optional[Dict[int, str]] = None,
                 busy: Optional[set] = None):
        super().__init__()
        self.devices = devices if devices is not None else DeviceList()
        self.profiles = dict(profiles or {})
        self.busy = set(busy or ())
        self.nps: Optional[str] = None

    def get_partition_devices(self) -> DeviceList:
        self._record("get_partition_devices")
        return self.devices

    def current_profiles(self) -> Dict[int, str]:
        self._record("current_profiles")
        return dict(self.profiles)

    def set_profile(self, gpu_index: int, profile: str) -> None:
        self._record("set_profile", gpu_index, profile)
        self.profiles[gpu_index] = profile

    def set_memory_partition(self, nps: str) -> None:
        self._record("set_memory_partition", nps)
        self.nps = nps

    def gpu_busy(self, gpu_index: int) -> bool:
        self._record("gpu_busy", gpu_index)
        return gpu_index in self.busy


class MockDevicePluginClient(_Recorder):
    def restart(self, node_name: str, timeout: float = 60.0) -> None:
        self._record("restart", node_name, timeout)


class MockNodeInitializer(_Recorder):
    def init_node_partitioning(self, node: Dict[str, Any]) -> bool:
        self._record("init_node_partitioning", node["metadata"]["name"])
        return True


class RecordingBarrier(CommitBarrier):
    """Commit barrier that records votes; ``veto`` makes it reject every commit."""

    def __init__(self, veto: bool = False):
        self.veto = veto
        self.votes: List[bool] = []

    def vote(self, ok: bool) -> bool:
        self.votes.append(ok)
        return ok and not self.veto
