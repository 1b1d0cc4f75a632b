"""Node-atomic partition commit barrier.

BASELINE.json asks that partition-state commits across the GPUs of one node be node-atomic with
an RCCL barrier over xGMI.  The agent is the single writer of its node, so the
barrier is a *post-commit health vote*: every participant (one per logical device after the
flip) contributes 1 if its local apply + verify succeeded, an all-reduce(sum) runs over the
node's devices, and the agent publishes the new ``status-partitioning-plan`` only if the sum
equals the number of participants.  Otherwise the plan is rolled back and retried.

Backends (same :class:`CommitBarrier` interface):

* :class:`RcclBarrier` — ``libnos_barrier.so``: its own RCCL communicator (``ncclCommInitRank``),
  a 4-byte ``ncclAllReduce``; unique id exchanged through any key/value store (a
  ``torch.distributed.TCPStore`` in the agent, a dict in-process);
* :class:`TorchBarrier` — ``torch.distributed.all_reduce`` on an existing process group (``nccl``
  = RCCL on ROCm, or ``gloo`` for CPU tests);
* :class:`LocalBarrier` — in-process, for the simulator and unit tests (votes from threads).
"""
from __future__ import annotations

import ctypes
import threading
import time
from typing import Any, Dict, List, Optional, Tuple

from ..utils.metrics import REGISTRY


class CommitBarrier:
    def vote(self, ok: bool) -> bool:
        """Contribute this participant's vote; True iff every participant voted ok."""
        raise NotImplementedError

    def close(self) -> None:
        return


class LocalBarrier(CommitBarrier):
    """N participants in one process (threads or a sequential simulator loop)."""

    def __init__(self, n: int, timeout: float = 30.0):
        self.n = n
        self.timeout = timeout
        self._cv = threading.Condition()
        self._votes: List[bool] = []
        self._gen = 0
        self._result: Dict[int, bool] = {}

    def vote(self, ok: bool) -> bool:
        with self._cv:
            gen = self._gen
            self._votes.append(bool(ok))
            if len(self._votes) == self.n:
                self._result[gen] = all(self._votes)
                self._votes = []
                self._gen += 1
                self._cv.notify_all()
                return self._result[gen]
            end = time.monotonic() + self.timeout
            while gen not in self._result:
                rem = end - time.monotonic()
                if rem <= 0:
                    # close the generation: every voter of it (and any late one) sees False, and
                    # the next round starts clean instead of being completed by a stale vote
                    self._result[gen] = False
                    self._votes = []
                    self._gen += 1
                    self._cv.notify_all()
                    return False
                self._cv.wait(rem)
            return self._result[gen]

    def vote_all(self, votes: List[bool]) -> bool:
        """Sequential helper: all N votes from one thread."""
        return all(votes) and len(votes) == self.n


# per (group, device): the side stream and vote buffer of the RCCL barrier, created once
_TORCH_BARRIER_STATE: Dict[Tuple[int, str], Tuple[Any, Any]] = {}


class TorchBarrier(CommitBarrier):
    """One int32 all-reduce per commit. With RCCL the vote runs on its own non-blocking HIP stream:
    on the legacy default stream it would wait for every blocking stream of the process — e.g. the
    CU-masked streams of the partitions' inference work — and serialise each commit behind the
    GPU's queued work."""

    def __init__(self, group: Any = None, device: Optional[Any] = None):
        import torch
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        backend = dist.get_backend(group)
        self.device = device if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu"))
        key = (id(group), str(self.device))
        st = _TORCH_BARRIER_STATE.get(key)
        if st is None:
            if self.device.type == "cuda":
                stream = torch.cuda.Stream(device=self.device)
                with torch.cuda.stream(stream):
                    buf = torch.zeros(1, dtype=torch.int32, device=self.device)
                stream.synchronize()
            else:
                stream, buf = None, torch.zeros(1, dtype=torch.int32)
            st = _TORCH_BARRIER_STATE[key] = (stream, buf)
        self._stream, self._buf = st

    def vote(self, ok: bool) -> bool:
        import contextlib

        import torch
        t0 = time.perf_counter()
        ctx = torch.cuda.stream(self._stream) if self._stream is not None else contextlib.nullcontext()
        with ctx:
            self._buf.fill_(1 if ok else 0)
            self.dist.all_reduce(self._buf, group=self.group)
            res = int(self._buf.item()) == self.world
        REGISTRY.phase_seconds.labels(phase="commit_barrier").observe(time.perf_counter() - t0)
        return res


class RankCommitBarrier(TorchBarrier):
    """The agent's commit path on a one-process-per-GPU job (the multi-GPU bench).

    The actuator produces one vote per logical device of the node (``Actuator._votes``) and hands
    the barrier the devices behind them (``set_participants``); this rank keeps only the votes of
    the partitions on *its* GPU, ANDs them with ``local_check()`` (e.g. "my data plane drained and
    my device answers"), and the all-reduce over the ranks (RCCL over xGMI, or gloo) says whether
    every GPU of the node committed.  One rank's veto therefore rolls the plan back on every rank
    (each runs the same control-plane replica, so they roll back identically)."""

    def __init__(self, rank: int, world: int, local_check=None, group: Any = None, device: Optional[Any] = None):
        super().__init__(group, device)
        self.rank = rank
        self.local_check = local_check
        self._gpus: Optional[List[int]] = None
        self.last_local: Optional[bool] = None

    def set_participants(self, devices: List[Any]) -> None:
        self._gpus = [int(getattr(d, "gpu_index", d)) for d in devices]

    def vote_all(self, votes: List[bool]) -> bool:
        mine = [v for v, g in zip(votes, self._gpus or []) if g == self.rank] if self._gpus else list(votes)
        local = all(mine)
        if local and self.local_check is not None:
            local = bool(self.local_check())
        self.last_local = local
        return self.vote(local)


class RcclBarrier(CommitBarrier):
    """Native RCCL communicator over the node's devices (``csrc/rccl_barrier.cpp``)."""

    def __init__(self, nranks: int, rank: int, device: int, store: Any, key: str = "nos/commit"):
        from ..ops.native import load
        L = load("libnos_barrier.so")
        L.nos_barrier_last_error.restype = ctypes.c_char_p
        L.nos_barrier_unique_id.argtypes = [ctypes.c_char_p, ctypes.c_int]
        L.nos_barrier_init.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                       ctypes.POINTER(ctypes.c_void_p)]
        L.nos_barrier_allreduce.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.POINTER(ctypes.c_int32)]
        L.nos_barrier_destroy.argtypes = [ctypes.c_void_p]
        self.L = L
        self.nranks = nranks
        size = L.nos_barrier_id_size()
        if rank == 0:
            buf = ctypes.create_string_buffer(size)
            self._check(L.nos_barrier_unique_id(buf, size))
            _store_set(store, key, buf.raw)
        uid = _store_get(store, key)
        h = ctypes.c_void_p()
        self._check(L.nos_barrier_init(nranks, rank, uid, device, ctypes.byref(h)))
        self.handle = h

    def _check(self, rc: int) -> None:
        if rc != 0:
            raise RuntimeError(f"rccl barrier: {self.L.nos_barrier_last_error().decode()} (rc={rc})")

    def vote(self, ok: bool) -> bool:
        t0 = time.perf_counter()
        out = ctypes.c_int32(0)
        self._check(self.L.nos_barrier_allreduce(self.handle, 1 if ok else 0, ctypes.byref(out)))
        REGISTRY.phase_seconds.labels(phase="commit_barrier").observe(time.perf_counter() - t0)
        return out.value == self.nranks

    def close(self) -> None:
        if self.handle:
            self._check(self.L.nos_barrier_destroy(self.handle))
            self.handle = None


def _store_set(store: Any, key: str, value: bytes) -> None:
    if isinstance(store, dict):
        store[key] = value
    else:
        store.set(key, value)


def _store_get(store: Any, key: str, timeout: float = 60.0) -> bytes:
    if isinstance(store, dict):
        end = time.monotonic() + timeout
        while key not in store:
            if time.monotonic() > end:
                raise TimeoutError(key)
            time.sleep(0.001)
        return store[key]
    return store.get(key)
