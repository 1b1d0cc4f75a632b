"""What the planner learns from the pods it has seen finish: their run times, and from those the
expected cost of draining a GPU for a pod that does not fit yet.

The reference has no notion of time at all: a MIG geometry change waits for nothing, because
free MIG instances are re-created around used ones (ref ``internal/controllers/migagent/actuator.go:225-229``).
A sliced MI355X GPU (``models/xcp/slices.py``) is the same for slices that fit, but a pod bigger
than the GPU's unused room needs some running pods to leave first — a *drain*, during which the
groups those pods free stay idle.  How long that takes, and how much capacity it idles, depends
on how long the pods on the GPU still have to run, which the planner can only estimate from the
run times of the pods that already finished and from how long each running pod has run so far.

* :class:`LifetimeModel` — the last ``window`` observed run times (seconds); the conditional
  residual of a pod that has run ``age`` seconds is drawn from the observed run times longer
  than ``age`` (a pod older than every observation is given half its age again);
* :func:`drain_cost` — Monte Carlo over those residuals (a fixed seed: the planner is
  deterministic): expected idle group-seconds until ``need`` groups are free, and the expected
  time until then;
* :class:`LifetimeTracker` — the pod controller's bookkeeping: running pods it has seen (start
  times), and the run time of every one that has since finished or vanished.
"""
from __future__ import annotations

import bisect
import collections
import random
from typing import Any, Deque, Dict, Iterable, List, Optional, Sequence, Tuple

from ...kube import objects as ko

#: (groups the pod holds, seconds it has run)
PodAge = Tuple[int, float]


class LifetimeModel:
    def __init__(self, window: int = 256, min_samples: int = 8):
        self.window = window
        self.min_samples = min_samples
        self._recent: Deque[float] = collections.deque(maxlen=window)
        self._sorted: List[float] = []

    def observe(self, seconds: float) -> None:
        if seconds <= 0:
            return
        if len(self._recent) == self.window:
            old = self._recent[0]
            i = bisect.bisect_left(self._sorted, old)
            if i < len(self._sorted) and self._sorted[i] == old:
                self._sorted.pop(i)
        self._recent.append(seconds)
        bisect.insort(self._sorted, seconds)

    @property
    def n(self) -> int:
        return len(self._sorted)

    def ready(self) -> bool:
        return self.n >= self.min_samples

    def quantile(self, q: float) -> Optional[float]:
        if not self._sorted:
            return None
        return self._sorted[min(self.n - 1, max(0, int(q * self.n)))]

    def median(self) -> Optional[float]:
        return self.quantile(0.5)

    def sample_residual(self, age: float, rng: random.Random) -> float:
        """Seconds a pod that has run ``age`` seconds still runs (one draw)."""
        i = bisect.bisect_right(self._sorted, age)
        if i >= self.n:
            return max(1.0, 0.5 * age)
        return self._sorted[rng.randrange(i, self.n)] - age

    def expected_residual(self, age: float) -> float:
        i = bisect.bisect_right(self._sorted, age)
        if i >= self.n:
            return max(1.0, 0.5 * age)
        tail = self._sorted[i:]
        return sum(tail) / len(tail) - age


def drain_cost(pods: Sequence[PodAge], capacity: int, need: int, model: LifetimeModel,
               samples: int = 96, seed: int = 0) -> Tuple[float, float]:
    """(expected idle group-seconds, expected seconds) until ``need`` of ``capacity`` groups are
    free on a GPU running ``pods`` if no new pod is placed on it meanwhile."""
    free0 = capacity - sum(g for g, _ in pods)
    if free0 >= need:
        return 0.0, 0.0
    rng = random.Random(seed)
    cost = wait = 0.0
    for _ in range(samples):
        ends = sorted((model.sample_residual(a, rng), g) for g, a in pods)
        free, t, c = free0, 0.0, 0.0
        for r, g in ends:
            c += free * (r - t)
            t = r
            free += g
            if free >= need:
                break
        cost += c
        wait += t
    return cost / samples, wait / samples


class LifetimeTracker:
    """Start times of the running pods the planner watches, and the run times of finished ones."""

    def __init__(self, model: Optional[LifetimeModel] = None):
        self.model = model or LifetimeModel()
        self._running: Dict[str, Tuple[float, float]] = {}   # uid -> (start, last seen running)

    def update(self, pods: Iterable[Dict[str, Any]], now: float) -> Dict[str, float]:
        """Feed every pod the planner can see that uses its resources; returns ``ns/name`` ->
        seconds run so far of the running ones. A pod that was running and is now terminal (or
        gone) adds its run time: start to its finish time when the pod records one, else to the
        last time it was seen running."""
        ages: Dict[str, float] = {}
        seen = set()
        for p in pods:
            uid = p.get("metadata", {}).get("uid") or ko.key(p)
            phase = ko.pod_phase(p)
            start = _ts(p.get("status", {}).get("startTime"))
            if phase == "Running":
                if start is None:
                    start = self._running.get(uid, (now, now))[0]
                self._running[uid] = (start, now)
                seen.add(uid)
                ages["/".join(ko.key(p))] = max(0.0, now - start)
            elif phase in ("Succeeded", "Failed") and uid in self._running:
                begun, _ = self._running.pop(uid)
                end = _finished_at(p)
                self.model.observe((end if end is not None else now) - begun)
        for uid in [u for u in self._running if u not in seen]:
            begun, last = self._running.pop(uid)
            self.model.observe(last - begun)
        return ages


def _ts(s: Optional[str]) -> Optional[float]:
    d = ko.parse_rfc3339(s)
    return d.timestamp() if d is not None else None


def _finished_at(pod: Dict[str, Any]) -> Optional[float]:
    out = None
    for cs in pod.get("status", {}).get("containerStatuses") or []:
        t = _ts(((cs.get("state") or {}).get("terminated") or {}).get("finishedAt"))
        if t is not None and (out is None or t > out):
            out = t
    return out
