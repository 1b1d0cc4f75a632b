"""Lease-based leader election (controller-runtime's, used by the gpupartitioner with
``leaderElect: true`` and ``resourceName: gpu-partitioner.nebuly.com``).

A ``coordination.k8s.io/v1`` Lease holds ``holderIdentity``, ``renewTime`` and
``leaseDurationSeconds``.  A candidate acquires it when it is free or expired, renews it every
``retry_period``, and steps down when it cannot renew within ``renew_deadline``; with
``release_on_cancel`` the holder clears the lease when stopping.  Works against both the in-memory
API server and the REST client.
"""
from __future__ import annotations

import datetime as _dt
import logging
import socket
import threading
import time
import uuid
from typing import Any, Callable, Optional

from .errors import AlreadyExists, Conflict, NotFound

log = logging.getLogger("nos.leader")


def _fmt(t: float) -> str:
    return _dt.datetime.fromtimestamp(t, _dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def _parse(s: Optional[str]) -> float:
    if not s:
        return 0.0
    return _dt.datetime.fromisoformat(s.replace("Z", "+00:00")).timestamp()


class LeaderElector:
    def __init__(self, client: Any, name: str, namespace: str = "nos-system", identity: Optional[str] = None,
                 lease_duration: float = 15.0, renew_deadline: float = 10.0, retry_period: float = 2.0,
                 release_on_cancel: bool = True, clock: Callable[[], float] = time.time):
        self.client = client
        self.name = name
        self.namespace = namespace
        self.identity = identity or f"{socket.gethostname()}_{uuid.uuid4().hex[:8]}"
        self.lease_duration = lease_duration
        self.renew_deadline = renew_deadline
        self.retry_period = retry_period
        self.release_on_cancel = release_on_cancel
        self.clock = clock
        self._leader = False
        self._last_renew = 0.0
        self._stop = threading.Event()
        self._thread: Optional[threading.Thread] = None

    def is_leader(self) -> bool:
        if self._leader and self.clock() - self._last_renew > self.renew_deadline:
            log.warning("lost leadership of %s: renew deadline exceeded", self.name)
            self._leader = False
        return self._leader

    def _lease(self, holder: str, acquire_time: Optional[str] = None) -> dict:
        now = _fmt(self.clock())
        return {"apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
                "metadata": {"name": self.name, "namespace": self.namespace},
                "spec": {"holderIdentity": holder, "leaseDurationSeconds": int(self.lease_duration),
                         "acquireTime": acquire_time or now, "renewTime": now}}

    def tick(self) -> bool:
        """One acquire-or-renew attempt."""
        now = self.clock()
        try:
            lease = self.client.get("Lease", self.name, self.namespace)
        except NotFound:
            try:
                self.client.create(self._lease(self.identity))
                self._become(now)
            except (AlreadyExists, Conflict):
                self._leader = False
            return self._leader
        spec = lease.get("spec", {})
        holder = spec.get("holderIdentity") or ""
        expired = now - _parse(spec.get("renewTime")) > float(spec.get("leaseDurationSeconds") or self.lease_duration)
        if holder == self.identity or not holder or expired:
            new = self._lease(self.identity, spec.get("acquireTime") if holder == self.identity else None)
            new["metadata"]["resourceVersion"] = lease["metadata"].get("resourceVersion", "")
            try:
                self.client.update(new)
                self._become(now)
            except (Conflict, NotFound):
                self._leader = False
        else:
            self._leader = False
        return self._leader

    def _become(self, now: float) -> None:
        if not self._leader:
            log.info("%s acquired leadership of %s", self.identity, self.name)
        self._leader = True
        self._last_renew = now

    def release(self) -> None:
        if not self._leader:
            return
        try:
            lease = self.client.get("Lease", self.name, self.namespace)
            if lease.get("spec", {}).get("holderIdentity") == self.identity:
                lease["spec"]["holderIdentity"] = ""
                self.client.update(lease)
        except (NotFound, Conflict):
            pass
        self._leader = False

    def start_background(self) -> None:
        def loop() -> None:
            while not self._stop.is_set():
                try:
                    self.tick()
                except Exception as e:  # noqa: BLE001
                    log.warning("leader election: %s", e)
                self._stop.wait(self.retry_period)
        self._thread = threading.Thread(target=loop, name="leader-election", daemon=True)
        self._thread.start()

    def stop(self) -> None:
        self._stop.set()
        if self.release_on_cancel:
            self.release()
