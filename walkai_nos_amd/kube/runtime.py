"""A minimal controller runtime (the controller-runtime v0.13 behaviours nos relies on).

What the reference gets from controller-runtime and reproduces here:

* a per-controller **work queue** with key de-duplication, "a key is never processed by two
  workers at once", ``RequeueAfter`` delays and per-key exponential back-off on error
  (5 ms doubling to 1000 s, like ``workqueue.DefaultControllerRateLimiter``);
* ``MaxConcurrentReconciles`` worker threads per controller
  (``mig_controller.go:204`` = 1, ``node_controller.go:113`` = 5);
* event **predicates** filtering watch events before they enqueue
  (``pkg/util/predicate/predicates.go``);
* a **Manager** that wires watches, runs controllers, periodic runnables, leader election
  (:mod:`walkai_nos_amd.kube.leader`) and serves ``/healthz`` ``/readyz`` ``/metrics``.

Two execution modes share one code path: ``start()`` runs worker threads against the wall
clock (production / agents), while ``run_until_idle()`` drives every queue synchronously on a
virtual clock, which is what the integration tests and the cluster simulator use to get
deterministic, fast runs.
"""
from __future__ import annotations

import heapq
import logging
import threading
import time
from dataclasses import dataclass
from typing import Any, Callable, Dict, Iterable, List, Optional, Sequence, Set, Tuple

from ..utils.metrics import REGISTRY, Metrics

log = logging.getLogger("nos.runtime")

Obj = Dict[str, Any]


@dataclass(frozen=True)
class Request:
    name: str
    namespace: str = ""


@dataclass
class Result:
    requeue: bool = False
    requeue_after: float = 0.0


class SimClock:
    """Virtual clock for deterministic runs."""

    def __init__(self, start: float = 1_700_000_000.0):
        self._now = float(start)
        self._lock = threading.Lock()

    def __call__(self) -> float:
        with self._lock:
            return self._now

    def advance(self, dt: float) -> None:
        with self._lock:
            self._now += max(0.0, dt)

    def set(self, t: float) -> None:
        with self._lock:
            self._now = max(self._now, t)


class WorkQueue:
    BASE_DELAY = 0.005
    MAX_DELAY = 1000.0

    def __init__(self, clock: Callable[[], float] = time.monotonic):
        self.clock = clock
        self._cv = threading.Condition()
        self._ready: List[Request] = []
        self._queued: Set[Request] = set()
        self._processing: Set[Request] = set()
        self._dirty: Set[Request] = set()
        self._delayed: List[Tuple[float, int, Request]] = []
        self._seq = 0
        self._failures: Dict[Request, int] = {}
        self._shutdown = False

    def add(self, req: Request) -> None:
        with self._cv:
            if req in self._processing:
                self._dirty.add(req)
                return
            if req in self._queued:
                return
            self._queued.add(req)
            self._ready.append(req)
            self._cv.notify()

    def add_after(self, req: Request, delay: float) -> None:
        if delay <= 0:
            self.add(req)
            return
        with self._cv:
            self._seq += 1
            heapq.heappush(self._delayed, (self.clock() + delay, self._seq, req))
            self._cv.notify()

    def add_rate_limited(self, req: Request) -> None:
        with self._cv:
            n = self._failures.get(req, 0)
            self._failures[req] = n + 1
        self.add_after(req, min(self.BASE_DELAY * (2 ** n), self.MAX_DELAY))

    def forget(self, req: Request) -> None:
        with self._cv:
            self._failures.pop(req, None)

    def _promote(self) -> None:
        now = self.clock()
        while self._delayed and self._delayed[0][0] <= now:
            _, _, req = heapq.heappop(self._delayed)
            if req in self._processing:
                self._dirty.add(req)
            elif req not in self._queued:
                self._queued.add(req)
                self._ready.append(req)

    def get_nowait(self) -> Optional[Request]:
        with self._cv:
            self._promote()
            return self._pop()

    def _pop(self) -> Optional[Request]:
        for i, req in enumerate(self._ready):
            if req not in self._processing:
                self._ready.pop(i)
                self._queued.discard(req)
                self._processing.add(req)
                return req
        return None

    def get(self, timeout: Optional[float] = None) -> Optional[Request]:
        deadline = None if timeout is None else time.monotonic() + timeout
        with self._cv:
            while not self._shutdown:
                self._promote()
                req = self._pop()
                if req is not None:
                    return req
                wait = 0.05
                if self._delayed:
                    wait = max(0.0, min(wait, self._delayed[0][0] - self.clock()))
                if deadline is not None:
                    rem = deadline - time.monotonic()
                    if rem <= 0:
                        return None
                    wait = min(wait, rem)
                self._cv.wait(wait)
            return None

    def done(self, req: Request) -> None:
        with self._cv:
            self._processing.discard(req)
            if req in self._dirty:
                self._dirty.discard(req)
                if req not in self._queued:
                    self._queued.add(req)
                    self._ready.append(req)
                self._cv.notify()

    def next_due(self) -> Optional[float]:
        with self._cv:
            return self._delayed[0][0] if self._delayed else None

    def has_ready(self) -> bool:
        with self._cv:
            self._promote()
            return any(r not in self._processing for r in self._ready)

    def shutdown(self) -> None:
        with self._cv:
            self._shutdown = True
            self._cv.notify_all()

    def __len__(self) -> int:
        with self._cv:
            return len(self._ready) + len(self._delayed)


# ---- predicates ----------------------------------------------------------------------
class Predicate:
    """controller-runtime ``predicate.Predicate``; default accepts everything."""

    def create(self, obj: Obj) -> bool:
        return True

    def update(self, old: Obj, new: Obj) -> bool:
        return True

    def delete(self, obj: Obj) -> bool:
        return True


class FuncPredicate(Predicate):
    def __init__(self, create: Optional[Callable[[Obj], bool]] = None,
                 update: Optional[Callable[[Obj, Obj], bool]] = None,
                 delete: Optional[Callable[[Obj], bool]] = None):
        self._c, self._u, self._d = create, update, delete

    def create(self, obj: Obj) -> bool:
        return True if self._c is None else self._c(obj)

    def update(self, old: Obj, new: Obj) -> bool:
        return True if self._u is None else self._u(old, new)

    def delete(self, obj: Obj) -> bool:
        return True if self._d is None else self._d(obj)


Reconciler = Callable[[Request], Optional[Result]]
Mapper = Callable[[Obj], Iterable[Request]]


def _own_key(obj: Obj) -> List[Request]:
    md = obj.get("metadata", {})
    return [Request(md.get("name", ""), md.get("namespace", "") or "")]


@dataclass
class Watch:
    kind: str
    predicates: Sequence[Predicate] = ()
    mapper: Mapper = _own_key


class Controller:
    def __init__(self, name: str, reconciler: Reconciler, watches: Sequence[Watch],
                 max_concurrent_reconciles: int = 1, clock: Callable[[], float] = time.monotonic,
                 metrics: Optional[Metrics] = None):
        self.name = name
        self.reconciler = reconciler
        self.watches = list(watches)
        self.max_concurrent = max(1, int(max_concurrent_reconciles))
        self.queue = WorkQueue(clock)
        self.metrics = metrics or REGISTRY
        self._threads: List[threading.Thread] = []
        self._stop = threading.Event()
        #: workers only process items while this returns True (leader election)
        self.gate: Optional[Callable[[], bool]] = None

    def handler_for(self, w: Watch) -> Callable[[str, Obj, Optional[Obj]], None]:
        def handle(etype: str, obj: Obj, old: Optional[Obj]) -> None:
            if etype == "ADDED":
                ok = all(p.create(obj) for p in w.predicates)
            elif etype == "MODIFIED":
                ok = all(p.update(old if old is not None else obj, obj) for p in w.predicates)
            else:
                ok = all(p.delete(obj) for p in w.predicates)
            if ok:
                for req in w.mapper(obj):
                    self.queue.add(req)
        return handle

    def process_one(self, req: Request) -> None:
        t0 = time.perf_counter()
        outcome = "success"
        try:
            res = self.reconciler(req) or Result()
        except Exception as e:  # noqa: BLE001 - reconcile errors are requeued with back-off
            outcome = "error"
            log.warning("controller %s: reconcile %s failed: %s", self.name, req, e, exc_info=log.isEnabledFor(logging.DEBUG))
            self.queue.add_rate_limited(req)
        else:
            if res.requeue_after > 0:
                self.queue.forget(req)
                self.queue.add_after(req, res.requeue_after)
                outcome = "requeue_after"
            elif res.requeue:
                self.queue.add_rate_limited(req)
                outcome = "requeue"
            else:
                self.queue.forget(req)
        finally:
            self.queue.done(req)
            self.metrics.reconcile_total.labels(controller=self.name, result=outcome).inc()
            self.metrics.reconcile_seconds.labels(controller=self.name).observe(time.perf_counter() - t0)

    # threaded mode
    def start(self) -> None:
        for i in range(self.max_concurrent):
            t = threading.Thread(target=self._worker, name=f"{self.name}-{i}", daemon=True)
            t.start()
            self._threads.append(t)

    def _worker(self) -> None:
        while not self._stop.is_set():
            if self.gate is not None and not self.gate():
                self._stop.wait(0.2)
                continue
            req = self.queue.get(timeout=0.1)
            if req is not None:
                self.process_one(req)

    def stop(self) -> None:
        self._stop.set()
        self.queue.shutdown()
        for t in self._threads:
            t.join(timeout=2)


@dataclass
class Runnable:
    """Periodic task run by the manager (e.g. an exporter tick)."""
    name: str
    fn: Callable[[], None]
    interval: float
    next_at: float = 0.0
    needs_leader: bool = True


class Manager:
    """Owns the client, the controllers and the runnables of one component process."""

    def __init__(self, client: Any, clock: Callable[[], float] = time.monotonic,
                 leader_election: Any = None, metrics: Optional[Metrics] = None):
        self.client = client
        self.clock = clock
        self.controllers: List[Controller] = []
        self.runnables: List[Runnable] = []
        self.health_checks: Dict[str, Callable[[], bool]] = {"ping": lambda: True}
        self.ready_checks: Dict[str, Callable[[], bool]] = {"ping": lambda: True}
        self.leader_election = leader_election
        self.metrics = metrics or REGISTRY
        self._cancels: List[Callable[[], None]] = []
        self._started = False
        self._stop = threading.Event()
        self._bg: List[threading.Thread] = []

    def new_controller(self, name: str, reconciler: Reconciler, watches: Sequence[Watch],
                       max_concurrent_reconciles: int = 1) -> Controller:
        c = Controller(name, reconciler, watches, max_concurrent_reconciles, clock=self.clock, metrics=self.metrics)
        self.controllers.append(c)
        if self._started:
            self._wire(c)
        return c

    def add_runnable(self, name: str, fn: Callable[[], None], interval: float, needs_leader: bool = True) -> None:
        self.runnables.append(Runnable(name, fn, interval, self.clock(), needs_leader))

    def add_healthz_check(self, name: str, fn: Callable[[], bool]) -> None:
        self.health_checks[name] = fn

    def add_readyz_check(self, name: str, fn: Callable[[], bool]) -> None:
        self.ready_checks[name] = fn

    def healthy(self) -> bool:
        return all(f() for f in self.health_checks.values())

    def ready(self) -> bool:
        return all(f() for f in self.ready_checks.values())

    def is_leader(self) -> bool:
        return self.leader_election is None or self.leader_election.is_leader()

    def _wire(self, c: Controller) -> None:
        for w in c.watches:
            self._cancels.append(self.client.watch(w.kind, c.handler_for(w)))

    def wire(self) -> None:
        if self._started:
            return
        self._started = True
        for c in self.controllers:
            self._wire(c)

    # ---- synchronous (virtual clock) mode -------------------------------------------
    def run_pending(self, max_iterations: int = 100_000) -> int:
        """Process every item that is ready *now* (and whatever it enqueues) across all
        controllers, then due runnables. Returns the number of reconciles executed."""
        self.wire()
        if self.leader_election is not None:
            self.leader_election.tick()
        n = 0
        progressed = True
        while progressed and n < max_iterations:
            progressed = False
            for c in self.controllers:
                if not self.is_leader() and getattr(c, "needs_leader", True) and self.leader_election is not None:
                    continue
                req = c.queue.get_nowait()
                while req is not None and n < max_iterations:
                    c.process_one(req)
                    n += 1
                    progressed = True
                    req = c.queue.get_nowait()
            now = self.clock()
            for r in self.runnables:
                if r.next_at <= now and (not r.needs_leader or self.is_leader()):
                    r.next_at = now + r.interval
                    r.fn()
                    progressed = True
        return n

    def next_due(self) -> Optional[float]:
        ts = [t for t in (c.queue.next_due() for c in self.controllers) if t is not None]
        ts += [r.next_at for r in self.runnables]
        return min(ts) if ts else None

    # ---- threaded mode ------------------------------------------------------------
    def start(self, block: bool = False) -> None:
        self.wire()
        if self.leader_election is not None:
            self.leader_election.start_background()
        for c in self.controllers:
            c.gate = self.is_leader
            c.start()
        t = threading.Thread(target=self._runnable_loop, name="runnables", daemon=True)
        t.start()
        self._bg.append(t)
        if block:
            try:
                while not self._stop.is_set():
                    time.sleep(0.2)
            except KeyboardInterrupt:
                pass
            self.stop()

    def _runnable_loop(self) -> None:
        while not self._stop.is_set():
            now = self.clock()
            for r in self.runnables:
                if r.next_at <= now and (not r.needs_leader or self.is_leader()):
                    r.next_at = now + r.interval
                    try:
                        r.fn()
                    except Exception as e:  # noqa: BLE001
                        log.warning("runnable %s failed: %s", r.name, e)
            self._stop.wait(0.05)

    def stop(self) -> None:
        self._stop.set()
        for c in self.controllers:
            c.stop()
        for cancel in self._cancels:
            cancel()
        if self.leader_election is not None:
            self.leader_election.stop()


def run_until_idle(managers: Sequence[Manager], clock: SimClock, horizon: float = 60.0,
                   max_steps: int = 10_000, on_step: Optional[Callable[[], None]] = None) -> float:
    """Drive several managers (one per simulated process) sharing one API server on a virtual
    clock until nothing is ready and the next delayed item lies beyond ``horizon`` seconds.
    Returns the virtual time elapsed."""
    t0 = clock()
    for _ in range(max_steps):
        work = 0
        for m in managers:
            work += m.run_pending()
        if on_step is not None:
            on_step()
        if work:
            continue
        dues = [d for d in (m.next_due() for m in managers) if d is not None]
        if not dues:
            break
        nxt = min(dues)
        if nxt - t0 > horizon:
            break
        clock.set(nxt)
    return clock() - t0
