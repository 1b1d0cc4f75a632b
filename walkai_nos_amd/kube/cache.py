"""Informer cache for the real-cluster client: reads from a list+watch mirror, writes to the API.

controller-runtime reconcilers read through the manager's informer cache (ref
``internal/controllers/gpupartitioner/mig_controller.go:60,113-119`` — ``c.Get``/``c.List`` hit the
cache, not the API server) and only writes go over the wire.  :class:`CachedClient` gives the
:class:`~walkai_nos_amd.kube.rest.RESTClient` the same shape:

* per cached kind one informer: an initial LIST, then a WATCH from its resourceVersion (the REST
  client's watch thread re-lists on ``410 Gone``), keeping ``{(namespace, name): object}``;
* ``get``/``list`` of a cached kind are served from that store, with label and field selectors
  applied locally (the same matchers the in-memory API server uses) — ``copy=False`` hands out the
  stored objects for read-only hot paths, as controller-runtime does with deep copies disabled;
* every write goes to the API server, and its response (the object as stored) is written through
  to the cache, so a controller never reads its own write back older than it made it;
* ``watch`` registrations fan out from the informer (one HTTP watch per kind, however many
  controllers watch it);
* ``revision`` counts cache events, so the pod controller's read-only plan memo (keyed on the API
  revision) works against a real cluster exactly as against the in-memory server.

Kinds that are not cached (Lease, Secret, Event, ...) pass straight through.
"""
from __future__ import annotations

import copy as _copy
import logging
import threading
from typing import Any, Callable, Dict, Iterable, List, Optional, Tuple

from . import objects as ko
from .errors import NotFound

log = logging.getLogger("nos.kube.cache")

Obj = Dict[str, Any]
Handler = Callable[[str, Obj, Optional[Obj]], None]

DEFAULT_CACHED = ("Node", "Pod", "ConfigMap", "ElasticQuota", "CompositeElasticQuota")


def _rv(o: Optional[Obj]) -> int:
    try:
        return int(((o or {}).get("metadata") or {}).get("resourceVersion") or 0)
    except (TypeError, ValueError):
        return 0


class Informer:
    def __init__(self, api: Any, kind: str):
        self.api = api
        self.kind = kind
        self.store: Dict[Tuple[str, str], Obj] = {}
        self.handlers: List[Handler] = []
        self.synced = threading.Event()
        self.lock = threading.RLock()
        self.events = 0
        self.assumed: Dict[Tuple[str, str], str] = {}  # pods bound by us, not yet confirmed by the watch
        self._stop: Optional[Callable[[], None]] = None

    def start(self) -> None:
        def on_event(t: str, o: Obj, old: Optional[Obj]) -> None:
            self.apply(t, o)
        # the watch lists first (every object arrives as ADDED), then streams; the store is complete
        # for readers once that first LIST has been applied — signalled from the watch's own thread,
        # in order with its events. A second LIST of our own would race the stream: a DELETED
        # delivered between that LIST's response and applying it would be undone by a stale ADDED,
        # and nothing would ever remove the zombie.
        self._stop = self.api.watch(self.kind, on_event, replay=True, on_synced=self.synced.set)

    def apply(self, t: str, o: Obj) -> None:
        k = (ko.namespace(o), ko.name(o))
        with self.lock:
            old = self.store.get(k)
            if t == "DELETED":
                self.assumed.pop(k, None)
                if old is None:
                    return
                self.store.pop(k, None)
            else:
                node = self.assumed.get(k)
                if node is not None:
                    if ko.pod_node_name(o):
                        self.assumed.pop(k, None)  # the watch confirmed the binding
                    else:
                        # an event older than the binding: keep the pod assumed on its node
                        o = _copy.deepcopy(o)
                        o.setdefault("spec", {})["nodeName"] = node
                        ko.set_condition(o, "PodScheduled", "True", "", "")
                if old is not None and _rv(o) and _rv(old) > _rv(o):
                    return  # a stale event (e.g. the watch replaying what a write-through already stored)
                if old is not None and old == o:
                    return
                self.store[k] = o
                t = "ADDED" if old is None else "MODIFIED"
            self.events += 1
            handlers = list(self.handlers)
        for h in handlers:
            try:
                h(t, o, old)
            except Exception as e:  # noqa: BLE001 - one handler must not starve the others
                log.warning("informer %s handler: %s", self.kind, e)

    def stop(self) -> None:
        if self._stop is not None:
            self._stop()


class CachedClient:
    """Cache-backed reads, pass-through writes (see module docstring)."""

    def __init__(self, api: Any, kinds: Iterable[str] = DEFAULT_CACHED, sync_timeout: float = 60.0):
        self.api = api
        self.kinds = tuple(kinds)
        self.sync_timeout = sync_timeout
        self._informers: Dict[str, Informer] = {}
        self._lock = threading.Lock()

    # -- informers ---------------------------------------------------------------------------
    def informer(self, kind: str) -> Optional[Informer]:
        if kind not in self.kinds:
            return None
        with self._lock:
            inf = self._informers.get(kind)
            if inf is None:
                inf = self._informers[kind] = Informer(self.api, kind)
                inf.start()
        if not inf.synced.wait(self.sync_timeout):
            raise TimeoutError(f"informer for {kind} did not sync within {self.sync_timeout}s")
        return inf

    @property
    def revision(self) -> int:
        return sum(i.events for i in self._informers.values())

    # -- reads -------------------------------------------------------------------------------
    def get(self, kind: str, name: str, namespace: str = "") -> Obj:
        inf = self.informer(kind)
        if inf is None:
            return self.api.get(kind, name, namespace)
        with inf.lock:
            o = inf.store.get((namespace, name))
        if o is None:
            raise NotFound(f"{kind} {namespace}/{name} not found (cache)")
        return _copy.deepcopy(o)

    def list(self, kind: str, namespace: Optional[str] = None, label_selector: Optional[str] = None,
             field_selector: Optional[str] = None, copy: bool = True) -> List[Obj]:
        inf = self.informer(kind)
        if inf is None:
            return self.api.list(kind, namespace, label_selector, field_selector)
        with inf.lock:
            objs = list(inf.store.values())
        out = []
        for o in objs:
            if namespace and ko.namespace(o) != namespace:
                continue
            if not ko.selector_matches(label_selector, ko.labels(o)):
                continue
            if not ko.field_selector_matches(field_selector, o):
                continue
            out.append(_copy.deepcopy(o) if copy else o)
        out.sort(key=lambda o: (ko.namespace(o), ko.name(o)))
        return out

    # -- writes (through to the API server, then into the cache) -----------------------------------
    def _through(self, kind: str, res: Any) -> Any:
        inf = self._informers.get(kind)
        if inf is not None and isinstance(res, dict) and res.get("metadata", {}).get("name"):
            res.setdefault("kind", kind)
            inf.apply("MODIFIED", res)
        return res

    def create(self, obj: Obj) -> Obj:
        return self._through(obj["kind"], self.api.create(obj))

    def update(self, obj: Obj) -> Obj:
        return self._through(obj["kind"], self.api.update(obj))

    def patch(self, kind: str, name: str, patch: Obj, namespace: str = "") -> Obj:
        return self._through(kind, self.api.patch(kind, name, patch, namespace))

    def delete(self, kind: str, name: str, namespace: str = "") -> None:
        self.api.delete(kind, name, namespace)

    def bind(self, pod_name: str, namespace: str, node_name: str) -> Obj:
        """POST pods/binding, then *assume* the binding in the cache (kube-scheduler's assumed
        pods): the API answers a Binding with a Status, not the pod, and until the watch delivers
        the bound pod a scheduling cycle reading the cache would still see it Pending and unbound —
        and place the next pod on capacity this one already holds. The assumed copy keeps the
        cached resourceVersion, so the watch's MODIFIED (a newer version) replaces it."""
        out = self.api.bind(pod_name, namespace, node_name)
        inf = self._informers.get("Pod")
        if inf is not None:
            with inf.lock:
                inf.assumed[(namespace, pod_name)] = node_name
                cur = inf.store.get((namespace, pod_name))
                assumed = _copy.deepcopy(cur) if cur is not None and not ko.pod_node_name(cur) else None
            if assumed is not None:
                inf.apply("MODIFIED", assumed)
        return out

    def watch(self, kind: str, handler: Handler, replay: bool = True) -> Callable[[], None]:
        inf = self.informer(kind)
        if inf is None:
            return self.api.watch(kind, handler, replay)
        with inf.lock:
            inf.handlers.append(handler)
            current = list(inf.store.values()) if replay else []
        for o in current:
            handler("ADDED", o, None)

        def cancel() -> None:
            with inf.lock:
                if handler in inf.handlers:
                    inf.handlers.remove(handler)
        return cancel

    def close(self) -> None:
        for inf in self._informers.values():
            inf.stop()
        close = getattr(self.api, "close", None)
        if close is not None:
            close()
