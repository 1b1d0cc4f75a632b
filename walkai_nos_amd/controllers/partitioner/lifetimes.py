"""What the planner learns from the pods it has seen finish: their run times, and from those the
expected cost of draining a GPU for a pod that does not fit yet.

The reference has no notion of time at all: a MIG geometry change waits for nothing, because
free MIG instances are re-created around used ones (ref ``internal/controllers/migagent/actuator.go:225-229``).
A sliced MI355X GPU (``models/xcp/slices.py``) is the same for slices that fit, but a pod bigger
than the GPU's unused room needs some running pods to leave first — a *drain*, during which the
groups those pods free stay idle.  How long that takes, and how much capacity it idles, depends
on how long the pods on the GPU still have to run, which the planner can only estimate from the
run times of the pods that already finished and from how long each running pod has run so far.

* :class:`LifetimeModel` — a Kaplan–Meier estimate of the run-time distribution from the last
  ``window`` finished pods (events) and the pods running now (right-censored at their age: each
  has run at least that long). Learning from finished pods alone is survival-biased — a node whose
  long-running inference Deployments never finish would feed the model only its short pods, and
  the median, which sets the reservation thresholds (``sliced.py``), would fire early. The
  conditional residual of a pod that has run ``age`` seconds is drawn from the estimate beyond
  ``age``; past the estimate's support (the mass of pods that outlive every observation) a pod is
  given its age again (a heavy tail's expected residual, not the half-age of an exhausted sample);
* :func:`drain_cost` — Monte Carlo over those residuals (a fixed seed: the planner is
  deterministic): expected idle group-seconds until ``need`` groups are free, and the expected
  time until then. A pod that declares a bound (``spec.activeDeadlineSeconds``: kubelet ends it
  that long after its start) has its residual capped at what is left of the bound, so a GPU whose
  pods are about to hit their deadlines is priced as the cheap drain it is;
* :class:`LifetimeTracker` — the pod controller's bookkeeping: running pods it has seen (start
  times), and the run time of every one that has since finished or vanished.
"""
from __future__ import annotations

import bisect
import collections
import random
from typing import Any, Deque, Dict, Iterable, List, Optional, Sequence, Tuple

from ...kube import objects as ko

#: (groups the pod holds, seconds it has run[, its declared bound: spec.activeDeadlineSeconds])
PodAge = Tuple  # (int, float) or (int, float, Optional[float])


def declared_bound(pod: Dict[str, Any]) -> Optional[float]:
    """``spec.activeDeadlineSeconds`` (kubelet ends the pod that long after its start), or None."""
    v = (pod.get("spec") or {}).get("activeDeadlineSeconds")
    try:
        return float(v) if v is not None and float(v) > 0 else None
    except (TypeError, ValueError):
        return None


class LifetimeModel:
    def __init__(self, window: int = 256, min_samples: int = 8):
        self.window = window
        self.min_samples = min_samples
        self._recent: Deque[float] = collections.deque(maxlen=window)
        self._sorted: List[float] = []        # finished run times (events)
        self._censored: List[float] = []      # ages of the pods running now (sorted)
        self._km: Optional[Tuple[List[float], List[float]]] = None

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
        self._km = None

    def censor(self, ages: Iterable[float]) -> None:
        """The ages of the pods running now (replaces the previous set): right-censored observations."""
        self._censored = sorted(a for a in ages if a > 0)
        self._km = None

    @property
    def n(self) -> int:
        """Finished pods observed (the estimate is ready once ``min_samples`` have finished)."""
        return len(self._sorted)

    def ready(self) -> bool:
        return self.n >= self.min_samples

    def survival(self) -> Tuple[List[float], List[float]]:
        """The Kaplan–Meier step function: event times t_k and S(t_k) just after each."""
        if self._km is None:
            times: List[float] = []
            surv: List[float] = []
            s = 1.0
            ev, ce = self._sorted, self._censored
            n_at_risk = len(ev) + len(ce)
            i = c = 0
            while i < len(ev):
                t = ev[i]
                while c < len(ce) and ce[c] < t:     # censored before t: leave the risk set
                    n_at_risk -= 1
                    c += 1
                d = 0
                while i < len(ev) and ev[i] == t:
                    d += 1
                    i += 1
                if n_at_risk > 0:
                    s *= 1.0 - d / n_at_risk
                times.append(t)
                surv.append(s)
                n_at_risk -= d
            self._km = (times, surv)
        return self._km

    def _s_at(self, t: float) -> float:
        times, surv = self.survival()
        k = bisect.bisect_right(times, t)
        return surv[k - 1] if k else 1.0

    def quantile(self, q: float) -> Optional[float]:
        """Smallest run time t with P(T <= t) > q (without censored pods: the order statistic
        ``sorted[int(q * n)]``); beyond the estimate's support (at least 1 - q of the pods outlive
        every finished one) the largest age seen, a lower bound."""
        if not self._sorted:
            return None
        times, surv = self.survival()
        for t, s in zip(times, surv):
            if 1.0 - s > q + 1e-12:
                return t
        return max(times[-1], self._censored[-1] if self._censored else 0.0)

    def median(self) -> Optional[float]:
        return self.quantile(0.5)

    def sample_residual(self, age: float, rng: random.Random) -> float:
        """Seconds a pod that has run ``age`` seconds still runs (one draw)."""
        times, surv = self.survival()
        s0 = self._s_at(age)
        k0 = bisect.bisect_right(times, age)
        if k0 >= len(times) or s0 <= 0.0:
            return max(1.0, age)
        u = rng.random() * s0                 # S(T) = u: the draw's survival level
        for k in range(k0, len(times)):
            if surv[k] <= u:
                return times[k] - age
        return max(1.0, age, times[-1] - age)  # it outlives every finished pod

    def expected_residual(self, age: float) -> float:
        times, surv = self.survival()
        s0 = self._s_at(age)
        k0 = bisect.bisect_right(times, age)
        if k0 >= len(times) or s0 <= 0.0:
            return max(1.0, age)
        e, prev = 0.0, s0
        for k in range(k0, len(times)):
            e += (prev - surv[k]) / s0 * (times[k] - age)
            prev = surv[k]
        e += prev / s0 * max(1.0, age, times[-1] - age)
        return e


def drain_cost(pods: Sequence[PodAge], capacity: int, need: int, model: LifetimeModel,
               samples: int = 96, seed: int = 0, used: Optional[int] = None) -> Tuple[float, float]:
    """(expected idle group-seconds, expected seconds) until ``need`` of ``capacity`` groups are
    free on a GPU running ``pods`` if no new pod is placed on it meanwhile. ``used`` (the GPU
    model's used groups) is authoritative for what is occupied: groups ``pods`` does not account
    for — a pod bound but not yet Running, or one the agent's status-pods annotation does not list
    yet — count as a pod that has just started, so a stale annotation never makes a busy GPU look
    free (and the cheapest drain victim)."""
    pods = [(p[0], p[1], p[2] if len(p) > 2 else None) for p in pods]
    held = sum(g for g, _, _ in pods)
    if used is not None and used > held:
        pods = pods + [(used - held, 0.0, None)]
        held = used
    free0 = capacity - held
    if free0 >= need:
        return 0.0, 0.0
    rng = random.Random(seed)
    cost = wait = 0.0
    for _ in range(samples):
        ends = sorted((_bounded(model.sample_residual(a, rng), a, b), g) for g, a, b in pods)
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


def _bounded(residual: float, age: float, bound: Optional[float]) -> float:
    """A residual run time no longer than what is left of the pod's declared bound."""
    return residual if bound is None else min(residual, max(0.0, bound - age))


class LifetimeTracker:
    """Start times of the running pods the planner watches, the run times of finished ones, and
    the ages of the running ones as the model's censored observations."""

    def __init__(self, model: Optional[LifetimeModel] = None):
        self.model = model or LifetimeModel()
        self._running: Dict[str, Tuple[float, float]] = {}   # uid -> (start, last seen running)
        self._done: Dict[str, float] = {}                      # terminal pods already counted

    def update(self, pods: Iterable[Dict[str, Any]], now: float) -> Dict[str, float]:
        """Feed every pod the planner can see that uses its resources — running and terminal
        (Succeeded / Failed) alike; returns ``ns/name`` -> seconds run so far of the running ones.
        A pod that was running and is now terminal adds its run time, start to the finish time it
        records; a terminal pod never seen running adds start to finish too (it ran between two
        passes), once; a pod that vanished adds start to the last time it was seen running."""
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
            elif phase in ("Succeeded", "Failed"):
                seen.add(uid)
                end = _finished_at(p)
                if uid in self._running:
                    begun, _ = self._running.pop(uid)
                    self.model.observe((end if end is not None else now) - begun)
                    self._done[uid] = now
                elif uid not in self._done and start is not None and end is not None:
                    self.model.observe(end - start)   # started and finished between two passes
                    self._done[uid] = now
        for uid in [u for u in self._running if u not in seen]:
            begun, last = self._running.pop(uid)
            self.model.observe(last - begun)
        for uid in [u for u, t in self._done.items() if u not in seen and now - t > 0]:
            del self._done[uid]               # terminal pods are forgotten once they are deleted
        self.model.censor(ages.values())
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
