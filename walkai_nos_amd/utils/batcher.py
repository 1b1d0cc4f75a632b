"""Batching window for pending pods.

Reference: ``pkg/util/batcher.go:25-130`` (a batch window whose *timeout* starts at the
first item and whose *idle* timer resets on every add; the batch is emitted on a 1-slot
channel).  In the reference fork the Batcher is only used by tests; here it
drives the partitioner's pending-pod batch window (``batchWindowTimeoutSeconds`` /
``batchWindowIdleSeconds``, docs ``dynamic-gpu-partitioning/configuration.md:6-40``).

The batcher is clock-driven (``poll(now)``) rather than goroutine-driven so that the
controller runtime and the simulator can run it deterministically; a background thread
helper is provided for real deployments.
"""
from __future__ import annotations

import threading
import time
from typing import Callable, Generic, List, Optional, TypeVar

T = TypeVar("T")


class Batcher(Generic[T]):
    def __init__(self, timeout_s: float, idle_s: float, clock: Callable[[], float] = time.monotonic):
        if timeout_s <= 0 or idle_s <= 0:
            raise ValueError("batch window timeout and idle must be > 0")
        self.timeout_s = float(timeout_s)
        self.idle_s = float(idle_s)
        self._clock = clock
        self._items: List[T] = []
        self._first_at: Optional[float] = None
        self._last_at: Optional[float] = None
        self._ready: Optional[List[T]] = None  # 1-slot "channel"
        self._lock = threading.Lock()
        self._started = False

    def start(self) -> None:
        with self._lock:
            self._started = True

    def stop(self) -> None:
        with self._lock:
            self._started = False
            self._items.clear()
            self._first_at = self._last_at = None

    def add(self, item: T) -> bool:
        """Non-blocking add; returns False (item dropped) when the batcher is not started
        or a finished batch is still waiting to be received (reference semantics)."""
        with self._lock:
            if not self._started or self._ready is not None:
                return False
            now = self._clock()
            if self._first_at is None:
                self._first_at = now
            self._last_at = now
            self._items.append(item)
            return True

    def poll(self, now: Optional[float] = None) -> None:
        """Move the current batch to the ready slot when a window expired."""
        with self._lock:
            if not self._items or self._ready is not None:
                return
            now = self._clock() if now is None else now
            assert self._first_at is not None and self._last_at is not None
            if now - self._first_at >= self.timeout_s or now - self._last_at >= self.idle_s:
                self._ready = self._items
                self._items = []
                self._first_at = self._last_at = None

    def ready(self) -> Optional[List[T]]:
        """Receive the ready batch (non-blocking)."""
        self.poll()
        with self._lock:
            out, self._ready = self._ready, None
            return out

    def flush(self) -> List[T]:
        """Force-emit whatever is buffered (used at shutdown and by the simulator)."""
        with self._lock:
            out = (self._ready or []) + self._items
            self._ready = None
            self._items = []
            self._first_at = self._last_at = None
            return out

    def deadline(self) -> Optional[float]:
        """Absolute clock time at which the current batch will be emitted."""
        with self._lock:
            if not self._items:
                return None
            assert self._first_at is not None and self._last_at is not None
            return min(self._first_at + self.timeout_s, self._last_at + self.idle_s)

    def __len__(self) -> int:
        with self._lock:
            return len(self._items)
