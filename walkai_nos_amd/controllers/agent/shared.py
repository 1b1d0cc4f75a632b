"""Reporter/actuator handshake (reference ``internal/controllers/migagent/shared.go:24-57``).

A mutex plus ``last_parsed_plan_id`` plus a one-slot "report token":

* the reporter's ``on_report_done`` is a non-blocking put of the token;
* the actuator's ``at_least_one_report_since_last_apply`` is a non-blocking take (it *consumes*
  the token, even on no-op paths — SURVEY Q12, preserved);
* ``on_apply_done`` drains the slot.

This enforces report → apply → report → apply, so the actuator never plans against a stale view
of the devices it has just changed.
"""
from __future__ import annotations

import threading
from typing import Optional


class SharedState:
    def __init__(self, helpers=None) -> None:
        self.lock = threading.RLock()
        self.last_parsed_plan_id: str = ""
        self.last_commit: Optional[str] = None
        self.commit_seq = 0  # bumped on every successful commit (probe-on-commit trigger)
        self._token = False
        self._token_lock = threading.Lock()
        # spawned GPU helpers (probe, commit barrier) of this agent; stopped before every flip
        from ...parallel.spawned import HelperRegistry
        self.helpers = helpers if helpers is not None else HelperRegistry()

    def record_commit(self, ok: bool) -> None:
        with self.lock:
            self.last_commit = "ok" if ok else "failed"
            if ok:
                self.commit_seq += 1

    def on_report_done(self) -> None:
        with self._token_lock:
            self._token = True

    def on_apply_done(self) -> None:
        with self._token_lock:
            self._token = False

    def at_least_one_report_since_last_apply(self) -> bool:
        with self._token_lock:
            had = self._token
            self._token = False
            return had
