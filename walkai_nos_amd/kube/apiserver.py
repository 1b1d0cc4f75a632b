"""Kubernetes REST facade over :class:`~walkai_nos_amd.kube.memory.InMemoryAPIServer`.

Serves the subset of the API server's HTTP surface the components speak through
:class:`~walkai_nos_amd.kube.rest.RESTClient`: LIST/GET (label and field selectors), POST, PUT,
merge PATCH (object and ``/status``), DELETE, ``pods/binding`` and ``?watch=1`` streams resumed
from a ``resourceVersion`` (newline-delimited JSON events, ``BOOKMARK`` while idle, ``ERROR``
410 when the requested version is older than the event log).

This is what lets the real component binaries (``python -m walkai_nos_amd.cmd.gpupartitioner``,
``...cmd.partitionagent``) run as separate processes against one control plane, with a kubeconfig,
the way the reference's envtest suites start ``kube-apiserver`` + ``etcd``
(``Makefile:17,95``).  It is used by the process-level end-to-end test and as a local
development cluster::

    python -m walkai_nos_amd.kube.apiserver --bind 127.0.0.1:8001 --kubeconfig-out /tmp/nos.kubeconfig

There is no authentication, admission or defaulting beyond what the in-memory server does.
"""
from __future__ import annotations

import argparse
import json
import logging
import threading
import time
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from typing import Any, Dict, List, Optional, Tuple

from .errors import AlreadyExists, Conflict, NotFound
from .memory import InMemoryAPIServer
from .rest import RESOURCES

log = logging.getLogger("nos.kube.apiserver")

Obj = Dict[str, Any]

# (group/version prefix, plural) -> kind
_KINDS: Dict[Tuple[str, str], str] = {(prefix, plural): kind for kind, (prefix, plural, _) in RESOURCES.items()}
_PREFIXES = sorted({prefix for prefix, _ in _KINDS}, key=len, reverse=True)


class _Route:
    __slots__ = ("kind", "namespace", "name", "sub")

    def __init__(self, kind: str, namespace: str, name: str, sub: str):
        self.kind, self.namespace, self.name, self.sub = kind, namespace, name, sub


def parse_path(path: str) -> Optional[_Route]:
    """``/api/v1/namespaces/ns/pods/name/status`` -> Route(Pod, ns, name, status)."""
    for prefix in _PREFIXES:
        if path == prefix or path.startswith(prefix + "/"):
            segs = [urllib.parse.unquote(s) for s in path[len(prefix):].split("/") if s]
            break
    else:
        return None
    ns = ""
    if len(segs) >= 3 and segs[0] == "namespaces":
        ns, segs = segs[1], segs[2:]
    if not segs or (prefix, segs[0]) not in _KINDS:
        return None
    kind = _KINDS[(prefix, segs[0])]
    name = segs[1] if len(segs) > 1 else ""
    sub = segs[2] if len(segs) > 2 else ""
    return _Route(kind, ns, name, sub)


class EventLog:
    """Every watch event of every served kind, in delivery order, with its resourceVersion: a
    watch from version ``v`` replays the events newer than ``v`` and then follows new ones."""

    def __init__(self, api: InMemoryAPIServer, max_events: int = 200_000):
        self.cond = threading.Condition()
        self.events: Dict[str, List[Tuple[int, str, Obj]]] = {k: [] for k in RESOURCES}
        self.dropped_below: Dict[str, int] = {k: 0 for k in RESOURCES}
        self.max_events = max_events
        self.closed = False
        self._cancel = [api.watch(k, self._recorder(k), replay=False) for k in RESOURCES]

    def _recorder(self, kind: str):
        def rec(etype: str, obj: Obj, _old: Optional[Obj]) -> None:
            obj = dict(obj, kind=kind)
            rv = int(obj.get("metadata", {}).get("resourceVersion") or 0)
            with self.cond:
                ev = self.events[kind]
                ev.append((rv, etype, obj))
                if len(ev) > self.max_events:
                    cut = len(ev) // 2
                    self.dropped_below[kind] = max(r for r, _, _ in ev[:cut])
                    del ev[:cut]
                self.cond.notify_all()
        return rec

    def close(self) -> None:
        for c in self._cancel:
            c()
        with self.cond:
            self.closed = True
            self.cond.notify_all()


class _Handler(BaseHTTPRequestHandler):
    facade: "APIFacade"
    protocol_version = "HTTP/1.0"   # one request per connection; a watch stream ends with the connection

    def log_message(self, fmt: str, *args: Any) -> None:  # route access logs to logging, not stderr
        log.debug("%s " + fmt, self.address_string(), *args)

    # -- plumbing -------------------------------------------------------------------------
    def _send(self, code: int, body: Any) -> None:
        raw = json.dumps(body).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(raw)))
        self.end_headers()
        self.wfile.write(raw)

    def _status(self, code: int, reason: str, msg: str) -> None:
        self._send(code, {"kind": "Status", "apiVersion": "v1", "status": "Failure", "reason": reason,
                          "message": f"{reason}: {msg}", "code": code})

    def _body(self) -> Any:
        n = int(self.headers.get("Content-Length") or 0)
        return json.loads(self.rfile.read(n)) if n else {}

    def _dispatch(self, method: str) -> None:
        url = urllib.parse.urlsplit(self.path)
        q = {k: v[-1] for k, v in urllib.parse.parse_qs(url.query).items()}
        r = parse_path(url.path)
        if r is None:
            return self._status(404, "NotFound", f"no route for {url.path}")
        api = self.facade.api
        try:
            if method == "GET" and not r.name:
                if q.get("watch") in ("1", "true"):
                    return self._watch(r.kind, q.get("resourceVersion", ""))
                rv = api.last_resource_version
                items = api.list(r.kind, r.namespace or None, q.get("labelSelector") or None,
                                 q.get("fieldSelector") or None)
                return self._send(200, {"kind": f"{r.kind}List", "apiVersion": "v1",
                                        "metadata": {"resourceVersion": str(rv)}, "items": items})
            if method == "GET":
                return self._send(200, api.get(r.kind, r.name, r.namespace))
            if method == "POST" and r.sub == "binding" and r.kind == "Pod":
                body = self._body()
                return self._send(201, api.bind(r.name, r.namespace, body["target"]["name"]))
            if method == "POST" and not r.name:
                obj = self._body()
                obj.setdefault("kind", r.kind)
                if r.namespace:
                    obj.setdefault("metadata", {}).setdefault("namespace", r.namespace)
                return self._send(201, api.create(obj))
            if method == "PUT" and r.name:
                obj = self._body()
                obj.setdefault("kind", r.kind)
                return self._send(200, api.update(obj))
            if method == "PATCH" and r.name and r.sub in ("", "status"):
                return self._send(200, api.patch(r.kind, r.name, self._body(), r.namespace))
            if method == "DELETE" and r.name:
                api.delete(r.kind, r.name, r.namespace)
                return self._send(200, {"kind": "Status", "apiVersion": "v1", "status": "Success"})
            return self._status(405, "MethodNotAllowed", f"{method} {url.path}")
        except NotFound as e:
            return self._status(404, "NotFound", str(e))
        except AlreadyExists as e:
            return self._status(409, "AlreadyExists", str(e))
        except Conflict as e:
            return self._status(409, "Conflict", str(e))
        except (ValueError, KeyError, TypeError) as e:
            return self._status(400, "BadRequest", str(e))

    def _watch(self, kind: str, since: str) -> None:
        ev_log = self.facade.events
        since_rv = int(since or 0)
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.end_headers()

        def write(obj: Obj) -> None:
            self.wfile.write(json.dumps(obj).encode() + b"\n")
            self.wfile.flush()

        with ev_log.cond:
            if since_rv and since_rv < ev_log.dropped_below[kind]:
                write({"type": "ERROR", "object": {"kind": "Status", "code": 410, "reason": "Expired"}})
                return
        pos, last_sent = 0, time.monotonic()
        events = ev_log.events[kind]
        try:
            while True:
                with ev_log.cond:
                    if pos > len(events):   # the log was compacted under us: resume by version
                        pos = 0
                    while pos >= len(events) and not ev_log.closed:
                        if not ev_log.cond.wait(timeout=self.facade.bookmark_every):
                            break
                    if ev_log.closed:
                        return
                    batch = events[pos:]
                    pos = len(events)
                fresh = [(rv, t, o) for rv, t, o in batch if rv > since_rv]
                for rv, t, o in fresh:
                    write({"type": t, "object": o})
                    since_rv = max(since_rv, rv)
                if fresh:
                    last_sent = time.monotonic()
                elif time.monotonic() - last_sent >= self.facade.bookmark_every:
                    rv = max(since_rv, self.facade.api.last_resource_version)
                    write({"type": "BOOKMARK", "object": {"kind": kind, "metadata": {"resourceVersion": str(rv)}}})
                    last_sent = time.monotonic()
        except (BrokenPipeError, ConnectionResetError):
            return

    def do_GET(self) -> None:  # noqa: N802 - http.server API
        self._dispatch("GET")

    def do_POST(self) -> None:  # noqa: N802
        self._dispatch("POST")

    def do_PUT(self) -> None:  # noqa: N802
        self._dispatch("PUT")

    def do_PATCH(self) -> None:  # noqa: N802
        self._dispatch("PATCH")

    def do_DELETE(self) -> None:  # noqa: N802
        self._dispatch("DELETE")


class APIFacade:
    """An HTTP API server over ``api`` on ``bind`` (``host:port``; port 0 picks a free one)."""

    def __init__(self, api: Optional[InMemoryAPIServer] = None, bind: str = "127.0.0.1:0",
                 bookmark_every: float = 30.0):
        self.api = api if api is not None else InMemoryAPIServer()
        self.events = EventLog(self.api)
        self.bookmark_every = bookmark_every
        host, _, port = bind.rpartition(":")
        handler = type("BoundHandler", (_Handler,), {"facade": self})
        self.httpd = ThreadingHTTPServer((host or "127.0.0.1", int(port or 0)), handler)
        self.httpd.daemon_threads = True
        self._thread: Optional[threading.Thread] = None

    @property
    def url(self) -> str:
        host, port = self.httpd.server_address[:2]
        return f"http://{host}:{port}"

    def start(self) -> "APIFacade":
        self._thread = threading.Thread(target=self.httpd.serve_forever, name="nos-apiserver", daemon=True)
        self._thread.start()
        return self

    def stop(self) -> None:
        self.events.close()
        self.httpd.shutdown()
        self.httpd.server_close()

    def write_kubeconfig(self, path: str) -> str:
        import yaml
        cfg = {"apiVersion": "v1", "kind": "Config", "current-context": "nos-local",
               "clusters": [{"name": "nos-local", "cluster": {"server": self.url}}],
               "users": [{"name": "nos-local", "user": {}}],
               "contexts": [{"name": "nos-local", "context": {"cluster": "nos-local", "user": "nos-local"}}]}
        with open(path, "w") as f:
            yaml.safe_dump(cfg, f)
        return path


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(description="in-memory Kubernetes API server (development / e2e tests)")
    ap.add_argument("--bind", default="127.0.0.1:8001")
    ap.add_argument("--kubeconfig-out", default="", help="write a kubeconfig pointing at this server")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    f = APIFacade(bind=args.bind).start()
    if args.kubeconfig_out:
        f.write_kubeconfig(args.kubeconfig_out)
    log.info("serving %s", f.url)
    try:
        while True:
            time.sleep(3600)
    except KeyboardInterrupt:
        f.stop()
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
