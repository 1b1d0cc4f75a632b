"""Agent-side handles for the spawned GPU helper (``walkai_nos_amd/cmd/gpuhelper.py``).

The node agents never touch the GPU through HIP themselves; they start the helper as a child
process (``subprocess``: fork + exec of a fresh interpreter, before anything in the agent has
initialised a GPU) and read its one JSON line.  Running helpers are registered in a
:class:`HelperRegistry` so the actuator can stop them before a mode flip — a helper still probing
the old partitions would hold KFD contexts and make the flip fail with "busy".
"""
from __future__ import annotations

import contextlib
import json
import logging
import os
import subprocess
import sys
import threading
import time
from typing import Any, Dict, List, Optional, Sequence

from ..utils.metrics import REGISTRY
from .barrier import CommitBarrier

log = logging.getLogger("nos.gpuhelper")

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class HelperRegistry:
    """Live helper processes of one agent, and the gate that keeps new ones out during a flip."""

    def __init__(self) -> None:
        self._lock = threading.Lock()
        self._cond = threading.Condition(self._lock)
        self._held = 0
        self._procs: List[subprocess.Popen] = []

    @contextlib.contextmanager
    def held(self):
        """No helper starts while held: a probe round that begins between :meth:`quiesce` and the
        amd-smi switch would open KFD contexts on the partitions being destroyed."""
        with self._cond:
            self._held += 1
        try:
            yield self
        finally:
            with self._cond:
                self._held -= 1
                self._cond.notify_all()

    def spawn(self, cmd: Sequence[str], timeout: float, **kw: Any) -> subprocess.Popen:
        """Start and register a helper once the gate is open (atomically: quiesce never misses it)."""
        with self._cond:
            if not self._cond.wait_for(lambda: self._held == 0, timeout):
                raise TimeoutError(f"gpu helper {list(cmd)[-1:]} held back for {timeout}s by a partition flip")
            p = subprocess.Popen(list(cmd), **kw)
            self._procs.append(p)
            return p

    def add(self, p: subprocess.Popen) -> None:
        with self._lock:
            self._procs.append(p)

    def remove(self, p: subprocess.Popen) -> None:
        with self._lock:
            if p in self._procs:
                self._procs.remove(p)

    def running(self) -> int:
        with self._lock:
            return sum(1 for p in self._procs if p.poll() is None)

    def quiesce(self, grace: float = 10.0) -> int:
        """Terminate every running helper (SIGTERM, then SIGKILL after ``grace``); returns how many."""
        with self._lock:
            procs = [p for p in self._procs if p.poll() is None]
        for p in procs:
            p.terminate()
        for p in procs:
            try:
                p.wait(grace)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        return len(procs)


DEFAULT_REGISTRY = HelperRegistry()


NATIVE_HELPER = "nos-gpuhelper"


def native_helper() -> Optional[str]:
    """Path of the native commit-barrier helper (``csrc/gpuhelper.cpp``), when it is built and not
    disabled with ``NOS_NATIVE_HELPER=0``."""
    from ..ops import native
    if os.environ.get("NOS_NATIVE_HELPER", "1") == "0" or not native.available(NATIVE_HELPER):
        return None
    return native.lib_path(NATIVE_HELPER)


def run_helper(args: Sequence[str], timeout: float = 180.0, registry: Optional[HelperRegistry] = None,
               program: Optional[str] = None) -> Dict[str, Any]:
    """Run the helper — ``program`` (a native executable) or ``python -m walkai_nos_amd.cmd.gpuhelper``
    — with ``args`` and return its JSON line."""
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + (os.pathsep + env["PYTHONPATH"] if env.get("PYTHONPATH") else "")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    reg = registry or DEFAULT_REGISTRY
    cmd = [program, *args] if program else [sys.executable, "-m", "walkai_nos_amd.cmd.gpuhelper", *args]
    p = reg.spawn(cmd, timeout, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        out, err = p.communicate(timeout=timeout)
    except subprocess.TimeoutExpired:
        p.kill()
        out, err = p.communicate()
        raise TimeoutError(f"gpu helper {args[0]} timed out after {timeout}s")
    finally:
        reg.remove(p)
    line = next((ln for ln in reversed(out.splitlines()) if ln.startswith("{")), None)
    if p.returncode != 0 or line is None:
        raise RuntimeError(f"gpu helper {args[0]} failed (rc={p.returncode}): {err.strip()[-500:]}")
    return json.loads(line)


class SpawnedNodeBarrier(CommitBarrier):
    """Node commit barrier over every logical device, run in a fresh helper process.

    One vote per logical device of the re-enumerated device map (HIP ordinal order); the helper
    must see exactly that many HIP devices, so a partition that did not come up is a veto even if
    every vote was 1.  Backends: ``xgmi`` — a ring of peer-to-peer token writes over xGMI
    (``csrc/p2p_barrier.hip``); ``rccl`` — an ncclCommInitAll clique and a grouped all-reduce
    (``csrc/rccl_barrier.cpp``); both run in the native ``nos-gpuhelper`` when it is built (no
    interpreter start-up on the flip path; ``rccl`` falls back to the Python helper); ``local``
    sums on the CPU (tests)."""

    def __init__(self, n_devices: int, backend: str = "rccl", timeout: float = 180.0,
                 registry: Optional[HelperRegistry] = None, native: Optional[bool] = None):
        self.n = n_devices
        self.backend = backend
        self.timeout = timeout
        self.registry = registry
        self.program = native_helper() if backend in ("rccl", "xgmi") and native is not False else None
        if (native or backend == "xgmi") and self.program is None:
            raise RuntimeError(f"native helper {NATIVE_HELPER} is not built (needed for the {backend} barrier)")
        self.last: Dict[str, Any] = {}

    def vote_all(self, votes: Sequence[bool]) -> bool:
        v = [1 if x else 0 for x in votes]
        t0 = time.perf_counter()
        try:
            res = run_helper(["barrier", "--votes", ",".join(map(str, v)), "--expect", str(self.n),
                              "--backend", self.backend], self.timeout, self.registry, self.program)
        except (RuntimeError, TimeoutError) as e:
            log.error("commit barrier helper: %s", e)
            self.last = {"error": str(e)}
            return False
        REGISTRY.phase_seconds.labels(phase="commit_barrier").observe(time.perf_counter() - t0)
        res["wall_ms"] = round(1e3 * (time.perf_counter() - t0), 3)
        self.last = res
        if res.get("error"):
            log.error("commit barrier: %s", res["error"])
            return False
        return len(v) == self.n and int(res.get("sum", -1)) == self.n

    def vote(self, ok: bool) -> bool:
        return self.vote_all([ok] * self.n)


def spawned_probe_round(targets: List[tuple], backend: str = "hip", timeout: float = 300.0,
                        registry: Optional[HelperRegistry] = None) -> Dict[str, Any]:
    """Probe every target in one helper process; label -> result (or {"error": ...})."""
    res = run_helper(["probe", "--targets", json.dumps([list(t) for t in targets]), "--backend", backend],
                     timeout, registry)
    return dict(res.get("slices", {}))
