"""Start gate: memory-only slice pods of one GPU start one after another (``PreStartContainer``).

The reference promises that memory-sliced ("MPS") pods share the GPU's compute equally
(ref ``docs/en/docs/dynamic-gpu-partitioning/getting-started-mps.md:22``). On an MI355X the
memory-only slices share every CU, and the command processor arbitrates dispatch per hardware pipe:
a process's compute queues are dealt over the pipes in the order the queues are created, so a pod's
share follows where its queues land. Measured (``profiles/fair_probe_r5.json``,
``tests/test_gpu_native.py``): pods that start one after another — each one's queues created before
the next process starts — share within 1.25x at 4, 6 and 8 pods; pods started at one instant race
their queue creation, and one run of eight dealt one pod a pipe of its own, 115 inf/s against 37.

kubelet starts the pods of a Deployment concurrently, so the order has to be imposed by the node:
the slice device plugin asks kubelet for ``PreStartContainer`` (``pre_start_required``) and its
handler passes every memory-only container through this gate. Per GPU, a container is let through
once the previous memory-only container let through on that GPU is *ready* — it has its compute
queues in the KFD (``/sys/class/kfd/kfd/proc/<pid>/queues/*/type`` = 0, on that GPU's KFD
``gpuid``) — or ``timeout`` seconds after it was let through (a container that never opens the GPU,
or one that failed, does not hold the others back for longer; kubelet gives the call 30 s).
Dedicated-CU slices pass at once: their CUs are their own.

Which KFD process is the previous container's: with hostPID (the agent's DaemonSet) the process
whose environment carries the slice in ``NOS_SLICE_IDS``; where the agent's PIDs are not the KFD's
(a PID namespace of its own), the first process on that GPU to reach its queues that was not there
when the container was let through (:class:`KfdProbe`).

Churn needs no extra rule: a departure removes its process's queues, and the next start through the
gate is created after every running pod's queues, as at first start (``tests/test_gpu_native.py``
measures 8 running, 3 of one start parity stopping, 3 new starting). Every wait is counted
(``nos_start_gate_waits_total`` / ``..._timeouts_total``, ``nos_start_gate_wait_seconds``).
"""
from __future__ import annotations

import glob
import logging
import os
import threading
import time
from typing import Any, Callable, Dict, Iterable, List, Optional, Tuple

log = logging.getLogger("nos.startgate")

KFD_PROC = "/sys/class/kfd/kfd/proc"
#: KFD queue type of a compute (AQL) queue; 1 is SDMA
KFD_COMPUTE = "0"


def kfd_compute_queues(pid: int, root: str = KFD_PROC) -> int:
    """Compute queues the KFD holds for ``pid`` (0 when the process has none or is gone)."""
    n = 0
    for q in glob.glob(os.path.join(root, str(pid), "queues", "*")):
        try:
            with open(os.path.join(q, "type")) as f:
                if f.read().strip() == KFD_COMPUTE:
                    n += 1
        except OSError:
            continue
    return n


def slice_ids_of(pid: int, proc: str = "/proc") -> frozenset:
    """The slice ids in a process's ``NOS_SLICE_IDS`` (empty when it has none or is gone)."""
    try:
        with open(os.path.join(proc, str(pid), "environ"), "rb") as f:
            env = f.read()
    except OSError:
        return frozenset()
    for kv in env.split(b"\0"):
        if kv.startswith(b"NOS_SLICE_IDS="):
            return frozenset(x.decode(errors="replace") for x in kv[len(b"NOS_SLICE_IDS="):].split(b",") if x)
    return frozenset()


def pids_with_slice(slice_id: str, proc: str = "/proc") -> List[int]:
    """Processes whose environment carries ``slice_id`` in ``NOS_SLICE_IDS`` (the env ``Allocate``
    gives a slice's container; the agent runs with hostPID, so it sees every container's processes)."""
    return [int(d) for d in os.listdir(proc) if d.isdigit() and slice_id in slice_ids_of(int(d), proc)]


def kfd_slice_ready(slice_id: str, min_queues: int = 2, proc: str = "/proc", kfd: str = KFD_PROC) -> bool:
    """A process of the slice's container has created its compute queues (HIP's utility queue and
    at least one user queue: two)."""
    return any(kfd_compute_queues(pid, kfd) >= min_queues for pid in pids_with_slice(slice_id, proc))


def kfd_gpu_id(bdf: str, topology: str = "/sys/class/kfd/kfd/topology/nodes") -> Optional[str]:
    """The KFD ``gpu_id`` of the GPU at PCI ``bdf`` (``dddd:bb:dd.f``), from the topology nodes'
    ``location_id`` (bus << 8 | device << 3 | function) and ``domain``; None when not found."""
    try:
        dom, bus, df = bdf.split(":")
        dev, fn = df.split(".")
        loc, domain = (int(bus, 16) << 8) | (int(dev, 16) << 3) | int(fn, 16), int(dom, 16)
    except ValueError:
        return None
    for n in glob.glob(os.path.join(topology, "*")):
        try:
            with open(os.path.join(n, "gpu_id")) as f:
                gid = f.read().strip()
            with open(os.path.join(n, "properties")) as f:
                props = dict(ln.split()[:2] for ln in f if len(ln.split()) >= 2)
        except OSError:
            continue
        if gid and gid != "0" and int(props.get("location_id", -1)) == loc and int(props.get("domain", 0)) == domain:
            return gid
    return None


class KfdProbe:
    """Readiness of a container's GPU process from the KFD (module docstring)."""

    def __init__(self, min_queues: int = 2, proc: str = "/proc", kfd: str = KFD_PROC,
                 topology: str = "/sys/class/kfd/kfd/topology/nodes"):
        self.min_queues = min_queues
        self.proc, self.kfd, self.topology = proc, kfd, topology
        self._gpu_ids: Dict[str, Optional[str]] = {}

    def _gpu_id(self, bdf: Optional[str]) -> Optional[str]:
        if not bdf:
            return None
        if bdf not in self._gpu_ids:
            self._gpu_ids[bdf] = kfd_gpu_id(bdf, self.topology)
        return self._gpu_ids[bdf]

    def ready_pids(self, bdf: Optional[str] = None) -> frozenset:
        """KFD processes with their compute queues (on the GPU at ``bdf`` when its gpu_id is known)."""
        gid = self._gpu_id(bdf)
        out = set()
        for d in glob.glob(os.path.join(self.kfd, "*")):
            pid = os.path.basename(d)
            if not pid.isdigit():
                continue
            n = 0
            for q in glob.glob(os.path.join(d, "queues", "*")):
                try:
                    with open(os.path.join(q, "type")) as f:
                        if f.read().strip() != KFD_COMPUTE:
                            continue
                    if gid is not None:
                        with open(os.path.join(q, "gpuid")) as f:
                            if f.read().strip() != gid:
                                continue
                except OSError:
                    continue
                n += 1
            if n >= self.min_queues:
                out.add(int(pid))
        return frozenset(out)

    def snapshot(self, bdf: Optional[str]) -> frozenset:
        return self.ready_pids(bdf)

    def ready(self, slice_id: str, bdf: Optional[str], snap: frozenset) -> bool:
        # only the few KFD processes with their queues are candidates: their environments are read
        # (not every process of the node, every poll)
        now = self.ready_pids(bdf)
        envs = {pid: slice_ids_of(pid, self.proc) for pid in now}
        if any(slice_id in ids for ids in envs.values()):
            return True
        # a PID namespace of our own (the KFD's PIDs are not ours, their environments unreadable):
        # the container's process is a ready one that appeared since it was let through and carries
        # no other slice
        return any(pid not in snap and not ids for pid, ids in envs.items())


class _CallableProbe:
    def __init__(self, fn: Callable[[str], bool]):
        self.fn = fn

    def snapshot(self, bdf: Optional[str]) -> frozenset:
        return frozenset()

    def ready(self, slice_id: str, bdf: Optional[str], snap: frozenset) -> bool:
        return self.fn(slice_id)


class StartGate:
    """Per-GPU FIFO of memory-only container starts (module docstring).

    ``probe``: readiness of a let-through container (default :class:`KfdProbe`); ``ready``: a plain
    ``slice_id -> bool`` instead (tests); ``timeout``: longest hold, seconds after the previous
    container was let through."""

    def __init__(self, ready: Optional[Callable[[str], bool]] = None, timeout: float = 20.0, poll: float = 0.05,
                 clock: Callable[[], float] = time.monotonic, sleep: Callable[[float], None] = time.sleep,
                 probe: Any = None):
        self.probe = probe or (_CallableProbe(ready) if ready is not None else KfdProbe())
        self.timeout = timeout
        self.poll = poll
        self.clock = clock
        self.sleep = sleep
        self._locks: Dict[int, threading.Lock] = {}
        self._guard = threading.Lock()
        # GPU -> (slice of the last container let through, when, its GPU's BDF, KFD snapshot then)
        self._last: Dict[int, Tuple[str, float, Optional[str], frozenset]] = {}
        self.order: List[Tuple[int, str]] = []  # (GPU, slice) in the order they were let through
        self.waits = 0
        self.timeouts = 0
        self.waited_s = 0.0

    def _lock(self, gpu: int) -> threading.Lock:
        with self._guard:
            return self._locks.setdefault(gpu, threading.Lock())

    def enter(self, gpu: int, slice_ids: Iterable[str], bdf: Optional[str] = None) -> float:
        """Block until the previous memory-only container of ``gpu`` is ready, or ``timeout``
        seconds after it was let through (a container let through long ago — a churn start — holds
        nothing back), then record ``slice_ids`` as the last one; returns the seconds waited.
        ``bdf``: the GPU's PCI address (the slice ids' prefix), for the KFD probe's GPU filter."""
        ids = list(slice_ids)
        with self._lock(gpu):
            prev = self._last.get(gpu)
            t0 = self.clock()
            waited, timed_out = 0.0, False
            if prev is not None and prev[0] not in ids:
                deadline = prev[1] + self.timeout
                ok = self.probe.ready(prev[0], prev[2], prev[3])
                while not ok and self.clock() < deadline:
                    self.sleep(self.poll)
                    ok = self.probe.ready(prev[0], prev[2], prev[3])
                timed_out = not ok
                waited = self.clock() - t0
            if ids:
                self._last[gpu] = (ids[0], self.clock(), bdf, self.probe.snapshot(bdf))
            self.order.append((gpu, ids[0] if ids else ""))
            self.waits += 1 if waited > 0 else 0
            self.timeouts += 1 if timed_out else 0
            self.waited_s += waited
            _count(waited, timed_out)
            if timed_out:
                log.warning("start gate GPU %d: %s not ready %.0fs after it started, letting %s start", gpu,
                            prev[0], self.timeout, ids)
            return waited

    def forget(self, slice_id: str) -> None:
        """A slice that left (its pod ended): nothing waits for it any more."""
        with self._guard:
            for g, s in list(self._last.items()):
                if s[0] == slice_id:
                    del self._last[g]


_metrics = None


def _count(waited: float, timed_out: bool) -> None:
    global _metrics
    if _metrics is None:
        from prometheus_client import Counter

        from ..utils.metrics import REGISTRY
        r = REGISTRY.registry
        _metrics = (Counter("nos_start_gate_waits_total", "memory-only container starts held by the start gate",
                            registry=r),
                    Counter("nos_start_gate_timeouts_total",
                            "memory-only container starts let through after the gate timed out", registry=r),
                    Counter("nos_start_gate_wait_seconds_total",
                            "seconds memory-only container starts waited at the start gate", registry=r))
    if waited > 0:
        _metrics[0].inc()
        _metrics[2].inc(waited)
    if timed_out:
        _metrics[1].inc()
