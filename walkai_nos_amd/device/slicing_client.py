"""CU-mask slice client and slice configuration store.

* :class:`SlicingClient` (reference ``pkg/gpu/slicing/client.go:27-105``): used ∪ free slice
  devices from kubelet for ``amd.com/gpu-<profile>`` resources, device id ``<gpu>::s<n>`` mapped to
  the physical GPU index (replica suffix stripped, reference ``ExtractGpuId``).
* :class:`SliceStore` — the per-node slice configuration (which slices exist, their CU rows and
  HBM budgets).  The slice agent writes it, the nos device plugin serves it: devices are
  advertised from it and ``Allocate`` injects ``HSA_CU_MASK`` / ``NOS_HBM_LIMIT_BYTES`` /
  ``LD_PRELOAD`` for the allocated slice.  Backed by a ConfigMap in a cluster, by memory in tests.
"""
from __future__ import annotations

import json
import threading
from typing import Any, Dict, List, Optional

from ..kube.errors import NotFound
from ..models.device import STATUS_FREE, DeviceList, GpuDevice
from ..models.errors import GpuError
from ..models.slicing.cumask import Slice
from ..models.slicing.profile import extract_profile_name, is_slice_resource
from .amdsmi import AmdSmi
from .podresources import ResourceClient

SliceMap = Dict[int, List[Slice]]


class SliceStore:
    def load(self) -> SliceMap:
        raise NotImplementedError

    def save(self, slices: SliceMap) -> None:
        raise NotImplementedError

    @staticmethod
    def encode(slices: SliceMap) -> str:
        return json.dumps({str(g): [s.to_dict() for s in ss] for g, ss in sorted(slices.items())}, sort_keys=True)

    @staticmethod
    def decode(text: str) -> SliceMap:
        doc = json.loads(text or "{}")
        return {int(g): [Slice.from_dict(d) for d in ss] for g, ss in doc.items()}


class MemorySliceStore(SliceStore):
    def __init__(self) -> None:
        self._text = "{}"
        self._lock = threading.Lock()
        self.saves = 0

    def load(self) -> SliceMap:
        with self._lock:
            return self.decode(self._text)

    def save(self, slices: SliceMap) -> None:
        with self._lock:
            self._text = self.encode(slices)
            self.saves += 1


class FileSliceStore(SliceStore):
    """A node-local JSON file: the partition agent's sliced-GPU layout (``models/xcp/slices.py``),
    which its own device plugin serves in the same process; it survives an agent restart (a host
    path), is replaced atomically, and is re-read only when it changed (the plugin reads it on every
    ListAndWatch poll)."""

    def __init__(self, path: str):
        self.path = path
        self._lock = threading.Lock()
        self._cache: Optional[tuple] = None   # (mtime_ns, size, text)

    def load(self) -> SliceMap:
        import os
        with self._lock:
            try:
                st = os.stat(self.path)
            except FileNotFoundError:
                return {}
            key = (st.st_mtime_ns, st.st_size)
            if self._cache is None or self._cache[:2] != key:
                with open(self.path) as f:
                    self._cache = (*key, f.read())
            return self.decode(self._cache[2])

    def save(self, slices: SliceMap) -> None:
        import os
        text = self.encode(slices)
        with self._lock:
            os.makedirs(os.path.dirname(os.path.abspath(self.path)), exist_ok=True)
            tmp = f"{self.path}.tmp.{os.getpid()}"
            with open(tmp, "w") as f:
                f.write(text)
                f.flush()
                os.fsync(f.fileno())
            os.replace(tmp, self.path)
            self._cache = None


class ConfigMapSliceStore(SliceStore):
    """``ConfigMap <namespace>/nos-slices-<node>``, key ``slices.json``."""

    KEY = "slices.json"

    def __init__(self, client: Any, node: str, namespace: str = "nos-system"):
        self.client = client
        self.name = f"nos-slices-{node}"
        self.namespace = namespace

    def load(self) -> SliceMap:
        try:
            cm = self.client.get("ConfigMap", self.name, self.namespace)
        except NotFound:
            return {}
        return self.decode((cm.get("data") or {}).get(self.KEY, "{}"))

    def save(self, slices: SliceMap) -> None:
        data = {self.KEY: self.encode(slices)}
        try:
            self.client.patch("ConfigMap", self.name, {"data": data}, self.namespace)
        except NotFound:
            self.client.create({"apiVersion": "v1", "kind": "ConfigMap",
                                "metadata": {"name": self.name, "namespace": self.namespace,
                                             "labels": {"app.kubernetes.io/part-of": "nos"}},
                                "data": data})


class SlicingClient:
    def __init__(self, resources: ResourceClient, smi: AmdSmi):
        self.resources = resources
        self.smi = smi

    def get_slice_devices(self) -> DeviceList:
        used = [d for d in self.resources.get_used_devices() if is_slice_resource(d.resource_name)]
        alloc = [d for d in self.resources.get_allocatable_devices() if is_slice_resource(d.resource_name)]
        used_ids = {d.device_id for d in used}
        out = DeviceList()
        for d in used:
            g = self._gpu(d.device_id)
            if g is not None:
                out.append(GpuDevice(d.resource_name, d.device_id, d.status, g))
        for d in alloc:
            if d.device_id not in used_ids:
                g = self._gpu(d.device_id)
                if g is not None:
                    out.append(GpuDevice(d.resource_name, d.device_id, STATUS_FREE, g))
        return out

    # the reporter calls this name on every client
    get_partition_devices = get_slice_devices

    def used_ids(self) -> set:
        return {d.device_id for d in self.resources.get_used_devices() if is_slice_resource(d.resource_name)}

    def _gpu(self, device_id: str) -> Optional[int]:
        try:
            return self.smi.gpu_index_of(device_id)
        except GpuError as e:
            if e.is_not_found():
                return None
            raise


def slice_profile(resource_name: str) -> Optional[str]:
    return extract_profile_name(resource_name)
