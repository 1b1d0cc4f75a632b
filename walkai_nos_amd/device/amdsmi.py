"""amd-smi partition backend (the NVML client replacement).

Two implementations of one interface:

* :class:`NativeAmdSmi` — ctypes over ``libnos_amdsmi.so`` (``csrc/amdsmi_backend.cpp``), a thin C
  ABI over ``libamd_smi``: inventory (UUID, BDF, VRAM, CU count), compute-partition get/set
  (``amdsmi.h:5768,5799``), memory-partition get/set (``:5844,5876``), activity, VRAM usage and the
  process list used for the "GPU busy" check.  Setters need root (``AMDSMI_STATUS_PERMISSION``,
  ``amdsmi.h:5790``) and surface as :class:`GpuError` with code ``permission``.
* :class:`FakeAmdSmi` — same API, in memory, with fault injection (permission denied, device
  busy, per-GPU failures, partial success) and re-enumeration; the test and simulator backend
  (and the only one that can flip modes on the non-root ``gpurun`` box).

Unlike the reference NVML client, which does ``Init``/``Shutdown`` around every call,
one session is kept per agent process.
"""
from __future__ import annotations

import ctypes
import os
import threading
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Set

from ..models.errors import GpuError
from ..models.xcp.known_configs import get_model_spec
from ..models.xcp.profile import COMPUTE_MODES, MEMORY_MODES

COMPUTE_MODE_NAMES = ("SPX", "DPX", "QPX", "CPX")
MEMORY_MODE_NAMES = ("NPS1", "NPS2", "NPS4", "NPS8")


@dataclass
class GpuInfo:
    index: int
    uuid: str
    bdf: str
    model: str
    vram_bytes: int
    cu_count: int
    xcds: int = 8


@dataclass
class LogicalDevice:
    """One logical GPU (compute partition) as enumerated after a mode switch."""
    gpu_index: int
    partition_index: int
    device_id: str
    compute_mode: str
    memory_mode: str


class AmdSmi:
    """Backend interface."""

    def list_gpus(self) -> List[GpuInfo]:
        raise NotImplementedError

    def get_compute_partition(self, index: int) -> str:
        raise NotImplementedError

    def set_compute_partition(self, index: int, mode: str) -> None:
        raise NotImplementedError

    def get_memory_partition(self, index: int) -> str:
        raise NotImplementedError

    def set_memory_partition(self, mode: str) -> None:
        """Node-wide: reloads the driver for every GPU (``amdsmi.h:6600-6615``)."""
        raise NotImplementedError

    def process_count(self, index: int) -> int:
        raise NotImplementedError

    def activity(self, index: int) -> Dict[str, float]:
        raise NotImplementedError

    def vram_usage(self, index: int) -> Dict[str, int]:
        raise NotImplementedError

    def logical_devices(self) -> List[LogicalDevice]:
        out: List[LogicalDevice] = []
        for g in self.list_gpus():
            cm = self.get_compute_partition(g.index)
            mm = self.get_memory_partition(g.index)
            for p in range(COMPUTE_MODES[cm.lower()]):
                out.append(LogicalDevice(g.index, p, f"{g.bdf}/xcp{p}", cm, mm))
        return out

    def gpu_index_of(self, device_id: str) -> int:
        """Map a device id (GPU UUID, BDF or ``<bdf>/xcp<k>``) to the physical GPU index."""
        base = device_id.split("/xcp", 1)[0].split("::", 1)[0]
        # the GPU set of a node is fixed for the process: index the ids once (re-scanned on a miss),
        # the device plugin and the reporters resolve every allocated device on each pass
        ids = getattr(self, "_gpu_ids", None)
        if ids is None or base not in ids:
            ids = {}
            for g in self.list_gpus():
                for k in (g.uuid, g.bdf, str(g.index)):
                    ids.setdefault(k, g.index)
            self._gpu_ids = ids
        if base in ids:
            return ids[base]
        raise GpuError(f"device {device_id!r} not found", GpuError.NOT_FOUND)

    def close(self) -> None:
        return


# ------------------------------------------------------------------------------------------
@dataclass
class _FakeGpu:
    info: GpuInfo
    compute: str = "SPX"
    memory: str = "NPS1"
    processes: int = 0


@dataclass
class FakeAmdSmi(AmdSmi):
    """In-memory amd-smi with fault injection."""
    n_gpus: int = 8
    model: str = "MI355X"
    is_root: bool = True
    fail_set: Set[int] = field(default_factory=set)          # GPU indexes whose set fails
    busy: Set[int] = field(default_factory=set)              # GPU indexes reported busy
    fail_next: int = 0                                       # fail the next N set calls
    memory_mode_requires_idle: bool = True

    def __post_init__(self) -> None:
        spec = get_model_spec(self.model)
        mem = (spec.memory_gb if spec else 288) * 10**9
        cus = spec.compute_units if spec else 256
        xcds = spec.xcds if spec else 8
        self._lock = threading.Lock()
        self._gpus = [_FakeGpu(GpuInfo(i, f"GPU-fake-{i:04x}", f"0000:{0x05 + i * 0x10:02x}:00.0", self.model,
                                       mem, cus, xcds)) for i in range(self.n_gpus)]
        self.set_calls: List[tuple] = []
        self.reenumerations = 0

    def list_gpus(self) -> List[GpuInfo]:
        return [g.info for g in self._gpus]

    def _gpu(self, index: int) -> _FakeGpu:
        if not 0 <= index < len(self._gpus):
            raise GpuError(f"GPU {index} not found", GpuError.NOT_FOUND)
        return self._gpus[index]

    def get_compute_partition(self, index: int) -> str:
        return self._gpu(index).compute

    def _check_set(self, index: Optional[int]) -> None:
        if not self.is_root:
            raise GpuError("amdsmi: AMDSMI_STATUS_PERMISSION (setting partitions requires root)", GpuError.PERMISSION)
        if self.fail_next > 0:
            self.fail_next -= 1
            raise GpuError(f"amdsmi: injected failure on GPU {index}", GpuError.GENERIC)
        if index is not None and index in self.fail_set:
            raise GpuError(f"amdsmi: injected failure on GPU {index}", GpuError.GENERIC)
        if index is not None and (index in self.busy or self._gpu(index).processes > 0):
            raise GpuError(f"amdsmi: GPU {index} is busy", GpuError.BUSY)

    def set_compute_partition(self, index: int, mode: str) -> None:
        mode = mode.upper()
        if mode not in COMPUTE_MODE_NAMES:
            raise GpuError(f"invalid compute partition {mode!r}")
        with self._lock:
            self._check_set(index)
            g = self._gpu(index)
            nps = MEMORY_MODES[g.memory.lower()]
            if COMPUTE_MODES[mode.lower()] < nps:
                raise GpuError(f"compute partition {mode} is incompatible with memory partition {g.memory}")
            g.compute = mode
            self.set_calls.append(("compute", index, mode))
            self.reenumerations += 1

    def get_memory_partition(self, index: int) -> str:
        return self._gpu(index).memory

    def set_memory_partition(self, mode: str) -> None:
        mode = mode.upper()
        if mode not in MEMORY_MODE_NAMES:
            raise GpuError(f"invalid memory partition {mode!r}")
        with self._lock:
            self._check_set(None)
            if self.memory_mode_requires_idle and any(g.processes > 0 or g.info.index in self.busy for g in self._gpus):
                raise GpuError("amdsmi: memory partition change needs every GPU of the node idle", GpuError.BUSY)
            nps = MEMORY_MODES[mode.lower()]
            for g in self._gpus:
                g.memory = mode
                if COMPUTE_MODES[g.compute.lower()] < nps:
                    g.compute = {1: "SPX", 2: "DPX", 4: "QPX", 8: "CPX"}[nps]
            self.set_calls.append(("memory", None, mode))
            self.reenumerations += 1

    def process_count(self, index: int) -> int:
        return self._gpu(index).processes

    def set_processes(self, index: int, n: int) -> None:
        self._gpu(index).processes = n

    def activity(self, index: int) -> Dict[str, float]:
        g = self._gpu(index)
        return {"gfx": 100.0 if g.processes else 0.0, "umc": 0.0, "mm": 0.0}

    def vram_usage(self, index: int) -> Dict[str, int]:
        g = self._gpu(index)
        return {"total": g.info.vram_bytes, "used": 0}


# ------------------------------------------------------------------------------------------
class _CInfo(ctypes.Structure):
    _fields_ = [("index", ctypes.c_uint32), ("uuid", ctypes.c_char * 64), ("bdf", ctypes.c_char * 32),
                ("market_name", ctypes.c_char * 64), ("vram_bytes", ctypes.c_uint64), ("cu_count", ctypes.c_uint32),
                ("xcds", ctypes.c_uint32)]


def native_library_path() -> str:
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return os.path.join(here, "_native", "libnos_amdsmi.so")


class NativeAmdSmi(AmdSmi):
    """ctypes binding to ``libnos_amdsmi.so`` (one amd-smi session per process)."""

    def __init__(self, lib_path: Optional[str] = None):
        path = lib_path or native_library_path()
        if not os.path.exists(path):
            raise GpuError(f"native amd-smi backend not built: {path} (run __graft_entry__.build())")
        self._lib = ctypes.CDLL(path)
        L = self._lib
        L.nos_smi_init.restype = ctypes.c_int
        L.nos_smi_last_error.restype = ctypes.c_char_p
        L.nos_smi_gpu_count.restype = ctypes.c_int
        L.nos_smi_gpu_info.argtypes = [ctypes.c_uint32, ctypes.POINTER(_CInfo)]
        L.nos_smi_get_compute_partition.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]
        L.nos_smi_set_compute_partition.argtypes = [ctypes.c_uint32, ctypes.c_char_p]
        L.nos_smi_get_memory_partition.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]
        L.nos_smi_set_memory_partition.argtypes = [ctypes.c_uint32, ctypes.c_char_p]
        L.nos_smi_process_count.argtypes = [ctypes.c_uint32]
        L.nos_smi_activity.argtypes = [ctypes.c_uint32] + [ctypes.POINTER(ctypes.c_uint32)] * 3
        L.nos_smi_vram.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        rc = L.nos_smi_init()
        if rc != 0:
            raise GpuError(f"amdsmi init failed: {self._err()}")
        self._lock = threading.Lock()

    def _err(self) -> str:
        e = self._lib.nos_smi_last_error()
        return e.decode() if e else "unknown error"

    def _check(self, rc: int, what: str) -> None:
        if rc == 0:
            return
        code = GpuError.GENERIC
        if rc == 2:
            code = GpuError.PERMISSION
        elif rc == 3:
            code = GpuError.NOT_FOUND
        elif rc == 4:
            code = GpuError.BUSY
        raise GpuError(f"{what}: {self._err()}", code)

    def list_gpus(self) -> List[GpuInfo]:
        out = []
        with self._lock:
            n = self._lib.nos_smi_gpu_count()
            for i in range(max(0, n)):
                c = _CInfo()
                self._check(self._lib.nos_smi_gpu_info(i, ctypes.byref(c)), "gpu info")
                out.append(GpuInfo(c.index, c.uuid.decode(), c.bdf.decode(), c.market_name.decode(),
                                   c.vram_bytes, c.cu_count, c.xcds or 8))
        return out

    def _get_str(self, fn, index: int) -> str:
        buf = ctypes.create_string_buffer(64)
        with self._lock:
            self._check(fn(index, buf, 64), "partition query")
        return buf.value.decode().upper()

    def get_compute_partition(self, index: int) -> str:
        return self._get_str(self._lib.nos_smi_get_compute_partition, index)

    def get_memory_partition(self, index: int) -> str:
        return self._get_str(self._lib.nos_smi_get_memory_partition, index)

    def set_compute_partition(self, index: int, mode: str) -> None:
        with self._lock:
            self._check(self._lib.nos_smi_set_compute_partition(index, mode.upper().encode()), "set compute partition")

    def set_memory_partition(self, mode: str) -> None:
        with self._lock:
            self._check(self._lib.nos_smi_set_memory_partition(0, mode.upper().encode()), "set memory partition")

    def process_count(self, index: int) -> int:
        with self._lock:
            n = self._lib.nos_smi_process_count(index)
        if n < 0:
            raise GpuError(f"process list: {self._err()}")
        return n

    def activity(self, index: int) -> Dict[str, float]:
        a, b, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        with self._lock:
            self._check(self._lib.nos_smi_activity(index, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), "activity")
        return {"gfx": float(a.value), "umc": float(b.value), "mm": float(c.value)}

    def vram_usage(self, index: int) -> Dict[str, int]:
        t, u = ctypes.c_uint64(), ctypes.c_uint64()
        with self._lock:
            self._check(self._lib.nos_smi_vram(index, ctypes.byref(t), ctypes.byref(u)), "vram")
        return {"total": t.value, "used": u.value}

    def close(self) -> None:
        self._lib.nos_smi_shutdown()


def new_backend(kind: str = "auto", **fake_kwargs) -> AmdSmi:
    """``native`` | ``fake`` | ``auto`` (native when the library loads and sees a GPU)."""
    if kind == "fake":
        return FakeAmdSmi(**fake_kwargs)
    if kind == "native":
        return NativeAmdSmi()
    try:
        b = NativeAmdSmi()
        if b.list_gpus():
            return b
    except (GpuError, OSError):
        pass
    return FakeAmdSmi(**fake_kwargs)
