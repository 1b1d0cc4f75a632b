"""Single-process RCCL commit barrier over every local GPU (``ncclCommInitAll`` clique).

The partition agent is one process per node; after a plan is applied it votes once per local
logical device (did that device verify?) and the grouped 4-byte all-reduce over xGMI tells it
whether the whole node committed.  Created per commit and destroyed before the next mode flip.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional, Sequence

from ..ops.native import load
from .barrier import CommitBarrier


class RcclNodeBarrier(CommitBarrier):
    def __init__(self, n_devices: int, devices: Optional[Sequence[int]] = None):
        L = load("libnos_barrier.so")
        L.nos_barrier_last_error.restype = ctypes.c_char_p
        L.nos_barrier_init_all.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_void_p)]
        L.nos_barrier_allreduce_all.argtypes = [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32),
                                                ctypes.POINTER(ctypes.c_int32)]
        L.nos_barrier_destroy_all.argtypes = [ctypes.c_void_p]
        self.L = L
        self.devices: List[int] = list(devices) if devices is not None else list(range(n_devices))
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        h = ctypes.c_void_p()
        self._check(L.nos_barrier_init_all(len(self.devices), arr, ctypes.byref(h)))
        self.handle = h

    def _check(self, rc: int) -> None:
        if rc != 0:
            raise RuntimeError(f"rccl node barrier: {self.L.nos_barrier_last_error().decode()} (rc={rc})")

    def vote_all(self, votes: Sequence[bool]) -> bool:
        """One vote per local device; extra/missing votes are padded with the last/True."""
        v = [bool(x) for x in votes][: len(self.devices)]
        v += [True] * (len(self.devices) - len(v))
        arr = (ctypes.c_int32 * len(v))(*[1 if x else 0 for x in v])
        out = ctypes.c_int32(0)
        self._check(self.L.nos_barrier_allreduce_all(self.handle, arr, ctypes.byref(out)))
        return out.value == len(self.devices) and all(votes)

    def vote(self, ok: bool) -> bool:
        return self.vote_all([ok] * len(self.devices))

    def close(self) -> None:
        if self.handle:
            self._check(self.L.nos_barrier_destroy_all(self.handle))
            self.handle = None
