"""In-memory Kubernetes API server — the framework's envtest analogue.

The reference's integration tier runs its controllers against a real ``kube-apiserver`` +
``etcd`` (envtest, ``Makefile:17,95``; suites ``internal/controllers/migagent/suite_int_test.go``).
Neither binary exists in this environment, so this module implements the API-server
semantics the operator depends on:

* objects keyed by (kind, namespace, name) with monotonically increasing ``resourceVersion``,
  ``uid`` and ``creationTimestamp``;
* optimistic concurrency on ``update`` (409 Conflict on a stale resourceVersion);
* RFC 7386 JSON merge patch (``client.MergeFrom`` in controller-runtime);
* label and field selectors (``spec.nodeName``, ``status.phase``, ...);
* watch streams delivered synchronously to registered handlers (ADDED/MODIFIED/DELETED,
  with the old object for MODIFIED, as controller-runtime's ``UpdateEvent`` has);
* the ``pods/binding`` and ``pods/eviction`` subresources used by the scheduler.

Everything is guarded by one re-entrant lock; handlers run outside the lock so a handler can
call back into the server.
"""
from __future__ import annotations

import itertools
import threading
import time
import uuid
from typing import Any, Callable, Dict, List, Optional, Tuple

from . import objects as ko
from .errors import AlreadyExists, Conflict, NotFound

Obj = Dict[str, Any]
Handler = Callable[[str, Obj, Optional[Obj]], None]

NAMESPACED = {"Pod", "ConfigMap", "Secret", "ElasticQuota", "CompositeElasticQuota", "Lease", "Event", "DaemonSet",
              "Deployment"}


def fast_copy(o: Any) -> Any:
    """Deep copy for JSON-shaped data (dict/list/scalars); ~5x faster than ``copy.deepcopy``."""
    if isinstance(o, dict):
        return {k: fast_copy(v) for k, v in o.items()}
    if isinstance(o, list):
        return [fast_copy(v) for v in o]
    return o


def merge_patch(target: Any, patch: Any) -> Any:
    """RFC 7386 JSON merge patch."""
    if not isinstance(patch, dict):
        return fast_copy(patch)
    if not isinstance(target, dict):
        target = {}
    out = dict(target)
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


def create_merge_patch(original: Any, modified: Any) -> Any:
    """Compute the merge patch turning ``original`` into ``modified`` (controller-runtime MergeFrom)."""
    if not isinstance(original, dict) or not isinstance(modified, dict):
        return fast_copy(modified)
    patch: Dict[str, Any] = {}
    for k in original:
        if k not in modified:
            patch[k] = None
    for k, v in modified.items():
        if k not in original:
            patch[k] = fast_copy(v)
        elif original[k] != v:
            if isinstance(v, dict) and isinstance(original[k], dict):
                patch[k] = create_merge_patch(original[k], v)
            else:
                patch[k] = fast_copy(v)
    return patch


class InMemoryAPIServer:
    """A thread-safe in-process API server with watch support."""

    def __init__(self, clock: Callable[[], float] = time.time):
        self._lock = threading.RLock()
        self._objs: Dict[Tuple[str, str, str], Obj] = {}
        self._by_kind: Dict[str, Dict[Tuple[str, str, str], Obj]] = {}  # kind index of _objs
        self._rv = itertools.count(1)
        self.last_resource_version = 0
        self._handlers: Dict[str, List[Handler]] = {}
        self.clock = clock
        # request counters, useful for tests / benchmarks
        self.stats: Dict[str, int] = {"create": 0, "update": 0, "patch": 0, "delete": 0, "get": 0, "list": 0}
        # bumped by every write (create / update / patch / delete / bind): equal revisions mean no
        # object changed in between, so read-only reconciles may reuse their last answer
        self.revision = 0

    # ---- watch ------------------------------------------------------------------------
    def watch(self, kind: str, handler: Handler, replay: bool = True,
              on_synced: Optional[Callable[[], None]] = None) -> Callable[[], None]:
        with self._lock:
            self._handlers.setdefault(kind, []).append(handler)
            existing = [fast_copy(o) for o in self._by_kind.get(kind, {}).values()] if replay else []
        for o in existing:
            handler("ADDED", o, None)
        if on_synced is not None:
            on_synced()

        def cancel() -> None:
            with self._lock:
                hs = self._handlers.get(kind, [])
                if handler in hs:
                    hs.remove(handler)

        return cancel

    def _emit(self, kind: str, etype: str, obj: Obj, old: Optional[Obj]) -> None:
        """Deliver one event to every watcher. The handlers of one event share a single copy of
        the objects (watch handlers only map events to requests; they must not mutate them)."""
        with self._lock:
            self.revision += 1
            handlers = list(self._handlers.get(kind, []))
        if not handlers:
            return
        o, prev = fast_copy(obj), (fast_copy(old) if old is not None else None)
        for h in handlers:
            h(etype, o, prev)

    def _next_rv(self) -> str:
        """The next resourceVersion (caller holds the lock)."""
        self.last_resource_version = next(self._rv)
        return str(self.last_resource_version)

    # ---- CRUD -------------------------------------------------------------------------
    @staticmethod
    def _k(kind: str, ns: str, name: str) -> Tuple[str, str, str]:
        return (kind, ns if kind in NAMESPACED else "", name)

    def create(self, obj: Obj) -> Obj:
        kind = obj["kind"]
        o = fast_copy(obj)
        md = ko.meta(o)
        if not md.get("name"):
            gen = md.get("generateName")
            if not gen:
                raise ValueError("object has no name")
            md["name"] = gen + uuid.uuid4().hex[:5]
        if kind in NAMESPACED:
            md.setdefault("namespace", "default")
        with self._lock:
            k = self._k(kind, md.get("namespace", ""), md["name"])
            if k in self._objs:
                raise AlreadyExists(f"{kind} {k[1]}/{k[2]} already exists")
            md["resourceVersion"] = self._next_rv()
            md.setdefault("uid", str(uuid.uuid4()))
            md.setdefault("creationTimestamp", ko.now_rfc3339(self.clock()))
            md.setdefault("labels", md.get("labels") or {})
            md.setdefault("annotations", md.get("annotations") or {})
            self._objs[k] = o
            self._by_kind.setdefault(kind, {})[k] = o
            self.stats["create"] += 1
            out = fast_copy(o)
        self._emit(kind, "ADDED", out, None)
        return out

    def get(self, kind: str, name: str, namespace: str = "") -> Obj:
        with self._lock:
            self.stats["get"] += 1
            o = self._objs.get(self._k(kind, namespace, name))
            if o is None:
                raise NotFound(f"{kind} {namespace}/{name} not found")
            return fast_copy(o)

    def list(self, kind: str, namespace: Optional[str] = None, label_selector: Optional[str] = None,
             field_selector: Optional[str] = None, copy: bool = True) -> List[Obj]:
        """Objects of ``kind`` matching the selectors, sorted by (namespace, name). ``copy=False``
        returns the stored objects themselves — for read-only callers on hot paths (the stored
        objects are never mutated in place: every write replaces them), like controller-runtime's
        cache reads with deep copies disabled."""
        with self._lock:
            self.stats["list"] += 1
            out = []
            for (_, ns, _), o in self._by_kind.get(kind, {}).items():
                if namespace and kind in NAMESPACED and ns != namespace:
                    continue
                if not ko.selector_matches(label_selector, ko.labels(o)):
                    continue
                if not ko.field_selector_matches(field_selector, o):
                    continue
                out.append(fast_copy(o) if copy else o)
        out.sort(key=lambda o: (ko.namespace(o), ko.name(o)))
        return out

    def _replace(self, kind: str, k: Tuple[str, str, str], new: Obj, verb: str) -> Obj:
        with self._lock:
            old = self._objs.get(k)
            if old is None:
                raise NotFound(f"{kind} {k[1]}/{k[2]} not found")
            md = ko.meta(new)
            for f in ("uid", "creationTimestamp", "name"):
                md[f] = old["metadata"].get(f)
            if kind in NAMESPACED:
                md["namespace"] = old["metadata"].get("namespace")
            self.stats[verb] += 1
            md["resourceVersion"] = old["metadata"]["resourceVersion"]
            if new == old:
                # a no-op write neither bumps the resourceVersion nor emits a watch event
                return fast_copy(old)
            md["resourceVersion"] = self._next_rv()
            self._objs[k] = new
            self._by_kind.setdefault(kind, {})[k] = new
            out, prev = fast_copy(new), fast_copy(old)
        self._emit(kind, "MODIFIED", out, prev)
        return out

    def update(self, obj: Obj) -> Obj:
        kind = obj["kind"]
        k = self._k(kind, ko.namespace(obj), ko.name(obj))
        with self._lock:
            cur = self._objs.get(k)
            if cur is None:
                raise NotFound(f"{kind} {k[1]}/{k[2]} not found")
            rv = ko.resource_version(obj)
            if rv and rv != cur["metadata"]["resourceVersion"]:
                raise Conflict(f"{kind} {k[1]}/{k[2]}: resourceVersion {rv} is stale")
            return self._replace(kind, k, fast_copy(obj), "update")

    def patch(self, kind: str, name: str, patch: Obj, namespace: str = "") -> Obj:
        """JSON merge patch (``application/merge-patch+json``)."""
        k = self._k(kind, namespace, name)
        with self._lock:
            cur = self._objs.get(k)
            if cur is None:
                raise NotFound(f"{kind} {namespace}/{name} not found")
            rv = (patch.get("metadata") or {}).get("resourceVersion")
            if rv and rv != cur["metadata"]["resourceVersion"]:
                raise Conflict(f"{kind} {namespace}/{name}: resourceVersion {rv} is stale")
            new = merge_patch(fast_copy(cur), patch)
            return self._replace(kind, k, new, "patch")

    def delete(self, kind: str, name: str, namespace: str = "") -> None:
        k = self._k(kind, namespace, name)
        with self._lock:
            o = self._objs.pop(k, None)
            if o is None:
                raise NotFound(f"{kind} {namespace}/{name} not found")
            self._by_kind.get(kind, {}).pop(k, None)
            self.stats["delete"] += 1
            # the DELETED event carries the deletion's own resourceVersion, as the API server's does
            o = fast_copy(o)
            o["metadata"]["resourceVersion"] = self._next_rv()
        self._emit(kind, "DELETED", o, None)

    # ---- subresources -------------------------------------------------------------------
    def bind(self, pod_name: str, namespace: str, node_name: str) -> Obj:
        """``pods/binding``: set spec.nodeName and PodScheduled=True."""
        k = self._k("Pod", namespace, pod_name)
        with self._lock:
            cur = self._objs.get(k)
            if cur is None:
                raise NotFound(f"Pod {namespace}/{pod_name} not found")
            if ko.pod_node_name(cur):
                raise Conflict(f"pod {namespace}/{pod_name} is already bound to {ko.pod_node_name(cur)}")
            new = fast_copy(cur)
            new["spec"]["nodeName"] = node_name
            ko.set_condition(new, "PodScheduled", "True", "", "")
            return self._replace("Pod", k, new, "update")

    def kinds(self) -> List[str]:
        with self._lock:
            return sorted({k for (k, _, _) in self._objs})
