"""amd-smi partition backend (the NVML client replacement).

Two implementations of one interface:

* :class:`NativeAmdSmi` — ctypes over ``libnos_amdsmi.so`` (``csrc/amdsmi_backend.cpp``), a thin C
  ABI over ``libamd_smi``: processor enumeration (UUID, BDF + KFD location id, partition id, KFD
  node, HIP ordinal, render node, VRAM, CU and XCD counts), compute-partition get/set
  (``amdsmi.h:5768,5799``), memory-partition get/set (``:5844,5876``), activity, VRAM usage and
  the process list used for the "GPU busy" check.  Setters need root (``AMDSMI_STATUS_PERMISSION``,
  ``amdsmi.h:5790``) and surface as :class:`GpuError` with code ``permission``.
* :class:`FakeAmdSmi` — same API, in memory, with fault injection (permission denied, device
  busy, per-GPU failures, partial success) and **faithful re-enumeration**: after a flip to CPX it
  reports eight processors per GPU with new UUIDs, HIP ordinals and render nodes, as the real
  library does, so stale ids stop resolving.

Both keep a :class:`~walkai_nos_amd.device.topology.DeviceMap` (physical GPU <-> logical
partition) that is rebuilt after every ``set_*`` call — the native backend re-initialises its
amd-smi session for that, because processor handles do not survive a partition change.  All
public per-GPU methods take the *physical* GPU index; the partition agent never sees a stale
handle (ref ``pkg/gpu/nvml/client.go:46-57`` gets the same effect by re-initialising NVML around
every call).

Nothing here initialises HIP: the agent process must not hold a KFD context while it flips modes
(a held context is exactly what makes a compute-partition switch fail with "busy").
"""
from __future__ import annotations

import ctypes
import os
import threading
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Set, Tuple

from ..models.errors import GpuError
from ..models.xcp.known_configs import get_model_spec
from ..models.xcp.profile import COMPUTE_MODES, MEMORY_MODES
from .topology import NO_PARTITION, DeviceMap, GpuInfo, LogicalDevice, ProcInfo, build_device_map

__all__ = ["AmdSmi", "FakeAmdSmi", "NativeAmdSmi", "ProcessStats", "GpuInfo", "LogicalDevice", "DeviceMap", "new_backend",
           "COMPUTE_MODE_NAMES", "MEMORY_MODE_NAMES"]

COMPUTE_MODE_NAMES = ("SPX", "DPX", "QPX", "CPX")
MEMORY_MODE_NAMES = ("NPS1", "NPS2", "NPS4", "NPS8")


def _nps(mode: str) -> int:
    return MEMORY_MODES.get(mode.lower(), 1)


@dataclass
class ProcessStats:
    """One process on one GPU as amd-smi reports it (``amdsmi_proc_info_t``): VRAM bytes; CU
    occupancy — the KFD's CU-equivalents of the process's waves in flight when sampled (waves over
    waves-per-CU), so a process confined to n CUs never reads more than n; None when the backend
    has no such field — and the milliseconds its queues spent evicted (time-sliced out)."""
    vram: int = 0
    cu_occupancy: Optional[int] = None
    evicted_ms: int = 0

    def merge(self, o: "ProcessStats") -> "ProcessStats":
        cu = None if self.cu_occupancy is None and o.cu_occupancy is None else \
            (self.cu_occupancy or 0) + (o.cu_occupancy or 0)
        return ProcessStats(self.vram + o.vram, cu, self.evicted_ms + o.evicted_ms)


class AmdSmi:
    """Backend interface.  Subclasses implement the per-processor hooks (``_processors`` …); the
    base class owns the node's device map and re-enumerates it after every partition change."""

    #: minimum seconds between re-enumerations triggered by unknown device ids (kubelet keeps
    #: advertising the old partitions until the device plugin re-registers)
    miss_rescan_interval = 5.0

    def __init__(self) -> None:
        self._map_lock = threading.RLock()
        self._map: Optional[DeviceMap] = None
        self._procs: Dict[int, ProcInfo] = {}
        self._generation = 0
        self._last_miss_scan = -1e9
        self.enumerations = 0

    # -- backend hooks ------------------------------------------------------------------------
    def _processors(self, reinit: bool) -> List[ProcInfo]:
        raise NotImplementedError

    def _compute_partition(self, proc: ProcInfo) -> str:
        raise NotImplementedError

    def _memory_partition(self, proc: ProcInfo) -> str:
        raise NotImplementedError

    def _set_compute_partition(self, proc: ProcInfo, mode: str) -> None:
        raise NotImplementedError

    def _set_memory_partition(self, proc: ProcInfo, mode: str) -> None:
        raise NotImplementedError

    def _process_count(self, proc: ProcInfo) -> int:
        raise NotImplementedError

    def _process_memory(self, proc: ProcInfo) -> Dict[int, int]:
        raise NotImplementedError

    def _process_info(self, proc: ProcInfo) -> Dict[int, ProcessStats]:
        """pid -> stats; backends without CU occupancy report VRAM only (``cu_occupancy`` None)."""
        return {pid: ProcessStats(b) for pid, b in self._process_memory(proc).items()}

    def _activity(self, proc: ProcInfo) -> Dict[str, float]:
        raise NotImplementedError

    def _vram_usage(self, proc: ProcInfo) -> Dict[str, int]:
        raise NotImplementedError

    def _power_clock(self, proc: ProcInfo) -> Dict[str, float]:
        return {}

    # -- device map -------------------------------------------------------------------------------
    def enumerate(self, reinit: bool = True) -> DeviceMap:
        """Re-read every processor and rebuild the physical <-> logical map."""
        with self._map_lock:
            procs = self._processors(reinit)
            self._procs = {p.ordinal: p for p in procs}
            old = self._map
            m = build_device_map(procs, self._compute_partition, self._memory_partition, _nps, self._generation)
            if old is None or [d.uuid for d in old.devices] != [d.uuid for d in m.devices] or \
                    old.modes() != m.modes():
                self._generation += 1
                m.generation = self._generation
            else:
                m.generation = old.generation
            self._map = m
            self.enumerations += 1
            return m

    def device_map(self) -> DeviceMap:
        with self._map_lock:
            if self._map is None:
                return self.enumerate(reinit=False)
            return self._map

    def list_gpus(self) -> List[GpuInfo]:
        return list(self.device_map().gpus)

    def logical_devices(self) -> List[LogicalDevice]:
        return list(self.device_map().devices)

    def resolve(self, device_id: str) -> LogicalDevice:
        """Device id (partition UUID, HIP UUID, ``renderD<n>``, BDF, ``<bdf>::s<n>``) -> partition.
        An unknown id triggers one rate-limited re-enumeration before NOT_FOUND."""
        m = self.device_map()
        d = m.lookup(device_id)
        if d is not None:
            return d
        with self._map_lock:
            now = time.monotonic()
            if now - self._last_miss_scan >= self.miss_rescan_interval:
                self._last_miss_scan = now
                m = self.enumerate(reinit=True)
        return m.resolve(device_id)

    def gpu_index_of(self, device_id: str) -> int:
        return self.resolve(device_id).gpu_index

    def _primary(self, gpu_index: int) -> ProcInfo:
        d = self.device_map().primary(gpu_index)
        return self._procs[d.proc_ordinal]

    def _members(self, gpu_index: int) -> List[ProcInfo]:
        m = self.device_map()
        parts = m.partitions_of(gpu_index)
        if not parts:
            raise GpuError(f"GPU {gpu_index} not found", GpuError.NOT_FOUND)
        return [self._procs[d.proc_ordinal] for d in parts]

    # -- per physical GPU -------------------------------------------------------------------------
    def get_compute_partition(self, index: int) -> str:
        return self.device_map().primary(index).compute_mode

    def get_memory_partition(self, index: int) -> str:
        return self.device_map().primary(index).memory_mode

    def set_compute_partition(self, index: int, mode: str) -> None:
        mode = mode.upper()
        if mode not in COMPUTE_MODE_NAMES:
            raise GpuError(f"invalid compute partition {mode!r}")
        with self._map_lock:
            proc = self._primary(index)
            try:
                self._set_compute_partition(proc, mode)
            finally:
                # the old handles are gone whether or not the switch completed
                self.enumerate(reinit=True)

    def set_memory_partition(self, mode: str) -> None:
        """Node-wide: reloads the driver for every GPU (``amdsmi.h:6600-6615``)."""
        mode = mode.upper()
        if mode not in MEMORY_MODE_NAMES:
            raise GpuError(f"invalid memory partition {mode!r}")
        with self._map_lock:
            proc = self._primary(0)
            try:
                self._set_memory_partition(proc, mode)
            finally:
                self.enumerate(reinit=True)

    def process_count(self, index: int) -> int:
        """Processes holding any partition of physical GPU ``index`` (a flip destroys them all)."""
        return sum(self._process_count(p) for p in self._members(index))

    def process_memory(self, index: int) -> Dict[int, int]:
        """pid -> VRAM bytes of every process holding a context on physical GPU ``index`` (the
        input of :class:`~walkai_nos_amd.controllers.hbmguard.HbmGuard`)."""
        out: Dict[int, int] = {}
        for p in self._members(index):
            for pid, b in self._process_memory(p).items():
                out[pid] = out.get(pid, 0) + b
        return out

    def process_info(self, index: int) -> Dict[int, ProcessStats]:
        """pid -> :class:`ProcessStats` (VRAM bytes, CU occupancy, queue-eviction ms) of every process
        holding a context on physical GPU ``index``, summed over its logical devices (the input of
        the slice guards, ``controllers/hbmguard.py``)."""
        out: Dict[int, ProcessStats] = {}
        for p in self._members(index):
            for pid, st in self._process_info(p).items():
                out[pid] = out[pid].merge(st) if pid in out else st
        return out

    def activity(self, index: int) -> Dict[str, float]:
        acts = [self._activity(p) for p in self._members(index)]
        return {k: sum(a[k] for a in acts) / len(acts) for k in ("gfx", "umc", "mm")}

    def vram_usage(self, index: int) -> Dict[str, int]:
        members = self._members(index)
        used = sum(self._vram_usage(p)["used"] for p in members)
        return {"total": self.device_map().gpus[index].vram_bytes, "used": used}

    def power_clock(self, index: int) -> Dict[str, float]:
        """Socket power / limit (W) and GFX clock / max (MHz) of physical GPU ``index``."""
        return self._power_clock(self._primary(index))

    def close(self) -> None:
        return


# ------------------------------------------------------------------------------------------
@dataclass
class _FakeGpu:
    index: int
    uuid: str
    bdf: str
    compute: str = "SPX"
    memory: str = "NPS1"
    processes: Dict[int, int] = field(default_factory=dict)  # partition -> process count
    vram: Dict[int, Dict[int, int]] = field(default_factory=dict)  # partition -> {pid: VRAM bytes}
    cu: Dict[int, Tuple[int, int]] = field(default_factory=dict)     # pid -> (CU occupancy, evicted ms)


class FakeAmdSmi(AmdSmi):
    """In-memory amd-smi with fault injection and MI300-style re-enumeration."""

    def __init__(self, n_gpus: int = 8, model: str = "MI355X", is_root: bool = True,
                 fail_set: Optional[Set[int]] = None, busy: Optional[Set[int]] = None, fail_next: int = 0,
                 memory_mode_requires_idle: bool = True, state_file: str = ""):
        """``state_file``: keep the modes in a JSON file, so a restarted process finds the GPUs in
        the modes it left them (as the real devices stay) — the agent-restart scenarios of the
        development cluster."""
        super().__init__()
        self.state_file = state_file
        self.n_gpus, self.model, self.is_root = n_gpus, model, is_root
        self.fail_set: Set[int] = set(fail_set or ())      # GPU indexes whose set fails
        self.busy: Set[int] = set(busy or ())              # GPU indexes reported busy
        self.fail_next = fail_next                         # fail the next N set calls
        self.memory_mode_requires_idle = memory_mode_requires_idle
        spec = get_model_spec(model)
        self._mem = (spec.memory_gb if spec else 288) * 10**9
        self._cus = spec.compute_units if spec else 256
        self._xcds = spec.xcds if spec else 8
        self._lock = threading.Lock()
        self._gpus = [_FakeGpu(i, f"GPU-fake-{i:04x}", f"0000:{0x05 + i * 0x10:02x}:00.0") for i in range(n_gpus)]
        self.set_calls: List[tuple] = []
        self.reenumerations = 0
        if state_file and os.path.exists(state_file):
            import json
            with open(state_file) as f:
                modes = json.load(f)
            for g, m in zip(self._gpus, modes):
                g.compute, g.memory = m["compute"], m["memory"]

    def _save(self) -> None:
        if self.state_file:
            import json
            tmp = self.state_file + ".tmp"
            with open(tmp, "w") as f:
                json.dump([{"compute": g.compute, "memory": g.memory} for g in self._gpus], f)
            os.replace(tmp, self.state_file)

    # -- hooks ---------------------------------------------------------------------------------
    def _processors(self, reinit: bool) -> List[ProcInfo]:
        out: List[ProcInfo] = []
        with self._lock:
            for g in self._gpus:
                n = COMPUTE_MODES[g.compute.lower()]
                nps = _nps(g.memory)
                for k in range(n):
                    o = len(out)
                    uuid = g.uuid if k == 0 else f"{g.uuid}-{g.compute.lower()}{k}"
                    bus = int(g.bdf.split(":")[1], 16)
                    out.append(ProcInfo(o, uuid, g.bdf, bdf_id=(k << 28) | (bus << 8), partition_id=k,
                                        kfd_node=o + 1, hip_id=o, hip_uuid=f"GPU-{g.index:02x}{k:02x}{o:012x}",
                                        render_minor=128 + o, market_name=self.model,
                                        vram_bytes=self._mem // nps, cu_count=self._cus // n,
                                        xcds=self._xcds // n))
        return out

    def _gpu(self, index: int) -> _FakeGpu:
        if not 0 <= index < len(self._gpus):
            raise GpuError(f"GPU {index} not found", GpuError.NOT_FOUND)
        return self._gpus[index]

    def _gpu_of(self, proc: ProcInfo) -> _FakeGpu:
        for g in self._gpus:
            if g.bdf == proc.bdf:
                return g
        raise GpuError(f"processor {proc.uuid} not found", GpuError.NOT_FOUND)

    def _compute_partition(self, proc: ProcInfo) -> str:
        return self._gpu_of(proc).compute

    def _memory_partition(self, proc: ProcInfo) -> str:
        return self._gpu_of(proc).memory

    def _check_set(self, index: Optional[int]) -> None:
        if not self.is_root:
            raise GpuError("amdsmi: AMDSMI_STATUS_PERMISSION (setting partitions requires root)", GpuError.PERMISSION)
        if self.fail_next > 0:
            self.fail_next -= 1
            raise GpuError(f"amdsmi: injected failure on GPU {index}", GpuError.GENERIC)
        if index is not None and index in self.fail_set:
            raise GpuError(f"amdsmi: injected failure on GPU {index}", GpuError.GENERIC)
        if index is not None and (index in self.busy or sum(self._gpu(index).processes.values()) > 0):
            raise GpuError(f"amdsmi: GPU {index} is busy", GpuError.BUSY)

    def _set_compute_partition(self, proc: ProcInfo, mode: str) -> None:
        with self._lock:
            g = self._gpu_of(proc)
            self._check_set(g.index)
            if COMPUTE_MODES[mode.lower()] < _nps(g.memory):
                raise GpuError(f"compute partition {mode} is incompatible with memory partition {g.memory}")
            g.compute = mode
            g.processes.clear()
            self.set_calls.append(("compute", g.index, mode))
            self.reenumerations += 1
            self._save()

    def _set_memory_partition(self, proc: ProcInfo, mode: str) -> None:
        with self._lock:
            self._check_set(None)
            if self.memory_mode_requires_idle and any(sum(g.processes.values()) > 0 or g.index in self.busy
                                                      for g in self._gpus):
                raise GpuError("amdsmi: memory partition change needs every GPU of the node idle", GpuError.BUSY)
            nps = _nps(mode)
            for g in self._gpus:
                g.memory = mode
                if COMPUTE_MODES[g.compute.lower()] < nps:
                    g.compute = {1: "SPX", 2: "DPX", 4: "QPX", 8: "CPX"}[nps]
            self.set_calls.append(("memory", None, mode))
            self.reenumerations += 1
            self._save()

    def _process_count(self, proc: ProcInfo) -> int:
        g = self._gpu_of(proc)
        return g.processes.get(proc.partition_id if proc.partition_id != NO_PARTITION else 0, 0)

    def _process_memory(self, proc: ProcInfo) -> Dict[int, int]:
        g = self._gpu_of(proc)
        return dict(g.vram.get(proc.partition_id if proc.partition_id != NO_PARTITION else 0, {}))

    def _process_info(self, proc: ProcInfo) -> Dict[int, ProcessStats]:
        g = self._gpu_of(proc)
        out = {}
        for pid, b in self._process_memory(proc).items():
            cu, ev = g.cu.get(pid, (0, 0))
            out[pid] = ProcessStats(b, cu, ev)
        return out

    def _activity(self, proc: ProcInfo) -> Dict[str, float]:
        return {"gfx": 100.0 if self._process_count(proc) else 0.0, "umc": 0.0, "mm": 0.0}

    def _vram_usage(self, proc: ProcInfo) -> Dict[str, int]:
        return {"total": proc.vram_bytes, "used": 0}

    def _power_clock(self, proc: ProcInfo) -> Dict[str, float]:
        busy = self._process_count(proc) > 0
        return {"power_w": 1000.0 if busy else 150.0, "power_limit_w": 1400.0, "gfx_mhz": 2000.0 if busy else 100.0,
                "gfx_max_mhz": 2400.0}

    # -- test helpers -----------------------------------------------------------------------------
    def set_processes(self, index: int, n: int, partition: int = 0) -> None:
        """Pretend ``n`` processes hold partition ``partition`` of GPU ``index``."""
        with self._lock:
            g = self._gpu(index)
            if n:
                g.processes[partition] = n
            else:
                g.processes.pop(partition, None)

    def set_process_memory(self, index: int, pid: int, nbytes: int, partition: int = 0) -> None:
        """Pretend process ``pid`` holds ``nbytes`` of VRAM on partition ``partition`` of GPU
        ``index`` (0 bytes: the process exits)."""
        with self._lock:
            per = self._gpu(index).vram.setdefault(partition, {})
            if nbytes:
                per[pid] = nbytes
            else:
                per.pop(pid, None)

    def set_process_cus(self, index: int, pid: int, cu_occupancy: int, evicted_ms: int = 0) -> None:
        """Pretend process ``pid`` on GPU ``index`` has ``cu_occupancy`` CUs' worth of waves in
        flight and ``evicted_ms`` of queue eviction (it must hold VRAM to be listed)."""
        with self._lock:
            self._gpu(index).cu[pid] = (cu_occupancy, evicted_ms)

    def attach(self, device_id: str, n: int = 1) -> None:
        """Pretend ``n`` more processes opened the partition behind ``device_id``."""
        d = self.resolve(device_id)
        with self._lock:
            g = self._gpus[d.gpu_index]
            g.processes[d.partition_index] = g.processes.get(d.partition_index, 0) + n


# ------------------------------------------------------------------------------------------
class _CProc(ctypes.Structure):
    _fields_ = [("ordinal", ctypes.c_uint32), ("uuid", ctypes.c_char * 64), ("bdf", ctypes.c_char * 32),
                ("market_name", ctypes.c_char * 64), ("hip_uuid", ctypes.c_char * 64),
                ("bdf_id", ctypes.c_uint64), ("kfd_id", ctypes.c_uint64), ("vram_bytes", ctypes.c_uint64),
                ("partition_id", ctypes.c_uint32), ("kfd_node", ctypes.c_int32), ("hip_id", ctypes.c_int32),
                ("hsa_id", ctypes.c_int32), ("render_minor", ctypes.c_int32), ("cu_count", ctypes.c_uint32),
                ("xcds", ctypes.c_uint32)]


def native_library_path() -> str:
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return os.path.join(here, "_native", "libnos_amdsmi.so")


class NativeAmdSmi(AmdSmi):
    """ctypes binding to ``libnos_amdsmi.so``.  One session per process, re-initialised by every
    re-enumeration (processor handles are invalid after a compute/memory partition change)."""

    def __init__(self, lib_path: Optional[str] = None):
        super().__init__()
        path = lib_path or native_library_path()
        if not os.path.exists(path):
            raise GpuError(f"native amd-smi backend not built: {path} (run __graft_entry__.build())")
        if lib_path is None and os.environ.get("NOS_ALLOW_STALE_NATIVE") != "1":
            from ..ops.build import verify
            try:
                verify("libnos_amdsmi.so")
            except RuntimeError as e:
                raise GpuError(str(e)) from None
        self._lib = ctypes.CDLL(path)
        L = self._lib
        L.nos_smi_init.restype = ctypes.c_int
        L.nos_smi_last_error.restype = ctypes.c_char_p
        L.nos_smi_enumerate.argtypes = [ctypes.c_int]
        L.nos_smi_proc_info.argtypes = [ctypes.c_uint32, ctypes.POINTER(_CProc)]
        L.nos_smi_get_compute_partition.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]
        L.nos_smi_set_compute_partition.argtypes = [ctypes.c_uint32, ctypes.c_char_p]
        L.nos_smi_get_memory_partition.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint32]
        L.nos_smi_set_memory_partition.argtypes = [ctypes.c_uint32, ctypes.c_char_p]
        L.nos_smi_process_count.argtypes = [ctypes.c_uint32]
        L.nos_smi_process_memory.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                             ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint32]
        self._has_info = hasattr(L, "nos_smi_process_info")
        if self._has_info:
            L.nos_smi_process_info.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                               ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint32),
                                               ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32]
        L.nos_smi_activity.argtypes = [ctypes.c_uint32] + [ctypes.POINTER(ctypes.c_uint32)] * 3
        L.nos_smi_vram.argtypes = [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(ctypes.c_uint64)]
        L.nos_smi_power_clock.argtypes = [ctypes.c_uint32] + [ctypes.POINTER(ctypes.c_uint32)] * 4
        self._lock = threading.Lock()
        rc = L.nos_smi_init()
        if rc != 0:
            raise GpuError(f"amdsmi init failed: {self._err()}")

    def _err(self) -> str:
        e = self._lib.nos_smi_last_error()
        return e.decode() if e else "unknown error"

    def _check(self, rc: int, what: str) -> None:
        if rc == 0:
            return
        code = {2: GpuError.PERMISSION, 3: GpuError.NOT_FOUND, 4: GpuError.BUSY}.get(rc, GpuError.GENERIC)
        raise GpuError(f"{what}: {self._err()}", code)

    def _processors(self, reinit: bool) -> List[ProcInfo]:
        out = []
        with self._lock:
            n = self._lib.nos_smi_enumerate(1 if reinit else 0)
            if n < 0:
                raise GpuError(f"amdsmi enumerate: {self._err()}")
            for i in range(n):
                c = _CProc()
                self._check(self._lib.nos_smi_proc_info(i, ctypes.byref(c)), "processor info")
                out.append(ProcInfo(i, c.uuid.decode(), c.bdf.decode(), c.bdf_id, c.partition_id, c.kfd_node,
                                    c.hip_id, c.hip_uuid.decode(), c.render_minor, c.market_name.decode(),
                                    c.vram_bytes, c.cu_count, c.xcds))
        return out

    def _get_str(self, fn, proc: ProcInfo) -> str:
        buf = ctypes.create_string_buffer(64)
        with self._lock:
            self._check(fn(proc.ordinal, buf, 64), "partition query")
        return buf.value.decode().upper()

    def _compute_partition(self, proc: ProcInfo) -> str:
        return self._get_str(self._lib.nos_smi_get_compute_partition, proc)

    def _memory_partition(self, proc: ProcInfo) -> str:
        return self._get_str(self._lib.nos_smi_get_memory_partition, proc)

    def _set_compute_partition(self, proc: ProcInfo, mode: str) -> None:
        with self._lock:
            self._check(self._lib.nos_smi_set_compute_partition(proc.ordinal, mode.encode()), "set compute partition")

    def _set_memory_partition(self, proc: ProcInfo, mode: str) -> None:
        with self._lock:
            self._check(self._lib.nos_smi_set_memory_partition(proc.ordinal, mode.encode()), "set memory partition")

    def _process_count(self, proc: ProcInfo) -> int:
        with self._lock:
            n = self._lib.nos_smi_process_count(proc.ordinal)
        if n < 0:
            raise GpuError(f"process list: {self._err()}")
        return n

    def _process_memory(self, proc: ProcInfo) -> Dict[int, int]:
        cap = 64
        while True:
            pids, vram = (ctypes.c_uint32 * cap)(), (ctypes.c_uint64 * cap)()
            with self._lock:
                n = self._lib.nos_smi_process_memory(proc.ordinal, pids, vram, cap)
            if n < 0:
                raise GpuError(f"process list: {self._err()}")
            if n <= cap:
                return {int(pids[i]): int(vram[i]) for i in range(n)}
            cap = n + 16

    def _process_info(self, proc: ProcInfo) -> Dict[int, ProcessStats]:
        if not self._has_info:
            return super()._process_info(proc)
        cap = 64
        while True:
            pids, vram = (ctypes.c_uint32 * cap)(), (ctypes.c_uint64 * cap)()
            cu, ev = (ctypes.c_uint32 * cap)(), (ctypes.c_uint32 * cap)()
            with self._lock:
                n = self._lib.nos_smi_process_info(proc.ordinal, pids, vram, cu, ev, cap)
            if n < 0:
                raise GpuError(f"process list: {self._err()}")
            if n <= cap:
                return {int(pids[i]): ProcessStats(int(vram[i]), int(cu[i]), int(ev[i])) for i in range(n)}
            cap = n + 16

    def _activity(self, proc: ProcInfo) -> Dict[str, float]:
        a, b, c = ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        with self._lock:
            self._check(self._lib.nos_smi_activity(proc.ordinal, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)),
                        "activity")
        return {"gfx": float(a.value), "umc": float(b.value), "mm": float(c.value)}

    def _vram_usage(self, proc: ProcInfo) -> Dict[str, int]:
        t, u = ctypes.c_uint64(), ctypes.c_uint64()
        with self._lock:
            self._check(self._lib.nos_smi_vram(proc.ordinal, ctypes.byref(t), ctypes.byref(u)), "vram")
        return {"total": t.value, "used": u.value}

    def _power_clock(self, proc: ProcInfo) -> Dict[str, float]:
        v = [ctypes.c_uint32() for _ in range(4)]
        with self._lock:
            self._check(self._lib.nos_smi_power_clock(proc.ordinal, *[ctypes.byref(x) for x in v]), "power/clock")
        limit = float(v[1].value)
        if limit > 1e5:  # some drivers report the limit in microwatts
            limit /= 1e6
        return {"power_w": float(v[0].value), "power_limit_w": limit, "gfx_mhz": float(v[2].value),
                "gfx_max_mhz": float(v[3].value)}

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
