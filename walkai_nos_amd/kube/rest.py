"""Kubernetes REST client for real clusters (stdlib ``urllib`` + ``ssl``; no client library needed).

Implements the same interface as :class:`~walkai_nos_amd.kube.memory.InMemoryAPIServer` — get,
list (label/field selectors), create, update, merge patch, delete, bind and watch — so every
controller runs unchanged against a real API server.  Credentials come from the in-cluster service
account (``/var/run/secrets/kubernetes.io/serviceaccount``) or a kubeconfig: server, CA (file or
inline ``-data``), and a bearer token (inline or ``tokenFile``) or a client certificate/key pair
(files or inline ``-data``, the ``kind``/kubeadm default).  Reads of long-running components go
through :class:`~walkai_nos_amd.kube.cache.CachedClient` (an informer cache in front of this
client), as controller-runtime's reconcilers read from theirs.
Watches are long-poll HTTP streams (``?watch=1``) consumed on a daemon thread per kind, with
re-list on ``410 Gone``.

This path cannot be exercised without a cluster in this environment; it is covered by unit tests
against a local HTTP stub that speaks the same JSON.
"""
from __future__ import annotations

import json
import logging
import os
import ssl
import threading
import urllib.error
import urllib.parse
import urllib.request
from typing import Any, Callable, Dict, List, Optional, Tuple

from .errors import AlreadyExists, APIError, Conflict, Forbidden, NotFound

log = logging.getLogger("nos.kube.rest")

Obj = Dict[str, Any]
SA_DIR = "/var/run/secrets/kubernetes.io/serviceaccount"

# kind -> (group/version path prefix, plural, namespaced)
RESOURCES: Dict[str, Tuple[str, str, bool]] = {
    "Node": ("/api/v1", "nodes", False),
    "Pod": ("/api/v1", "pods", True),
    "ConfigMap": ("/api/v1", "configmaps", True),
    "Secret": ("/api/v1", "secrets", True),
    "Event": ("/api/v1", "events", True),
    "Namespace": ("/api/v1", "namespaces", False),
    "Lease": ("/apis/coordination.k8s.io/v1", "leases", True),
    "DaemonSet": ("/apis/apps/v1", "daemonsets", True),
    "ElasticQuota": ("/apis/nos.nebuly.com/v1alpha1", "elasticquotas", True),
    "CompositeElasticQuota": ("/apis/nos.nebuly.com/v1alpha1", "compositeelasticquotas", True),
}


class RESTClient:
    def __init__(self, server: str, token: str = "", ca_file: Optional[str] = None, insecure: bool = False,
                 timeout: float = 30.0, cert_file: Optional[str] = None, key_file: Optional[str] = None):
        self.server = server.rstrip("/")
        self.token = token
        self.timeout = timeout
        self.cert_file = cert_file
        if self.server.startswith("https"):
            ctx = ssl.create_default_context(cafile=ca_file) if ca_file else ssl.create_default_context()
            if insecure:
                ctx.check_hostname = False
                ctx.verify_mode = ssl.CERT_NONE
            if cert_file:
                ctx.load_cert_chain(cert_file, key_file)  # mutual TLS (client-certificate users)
            self._ctx: Optional[ssl.SSLContext] = ctx
        else:
            self._ctx = None
        self._watchers: List[threading.Event] = []

    @staticmethod
    def in_cluster() -> "RESTClient":
        host = os.environ["KUBERNETES_SERVICE_HOST"]
        port = os.environ.get("KUBERNETES_SERVICE_PORT", "443")
        with open(os.path.join(SA_DIR, "token")) as f:
            token = f.read().strip()
        return RESTClient(f"https://{host}:{port}", token, os.path.join(SA_DIR, "ca.crt"))

    # -- plumbing -------------------------------------------------------------------------
    def _path(self, kind: str, name: str = "", namespace: str = "", sub: str = "") -> str:
        prefix, plural, namespaced = RESOURCES[kind]
        p = prefix
        if namespaced and namespace:
            p += f"/namespaces/{urllib.parse.quote(namespace)}"
        p += f"/{plural}"
        if name:
            p += f"/{urllib.parse.quote(name)}"
        if sub:
            p += f"/{sub}"
        return p

    def _req(self, method: str, path: str, body: Any = None, content_type: str = "application/json",
             query: Optional[Dict[str, str]] = None, stream: bool = False, timeout: Optional[float] = None):
        url = self.server + path
        if query:
            url += "?" + urllib.parse.urlencode({k: v for k, v in query.items() if v})
        data = json.dumps(body).encode() if body is not None else None
        req = urllib.request.Request(url, data=data, method=method)
        req.add_header("Accept", "application/json")
        if data is not None:
            req.add_header("Content-Type", content_type)
        if self.token:
            req.add_header("Authorization", f"Bearer {self.token}")
        try:
            resp = urllib.request.urlopen(req, timeout=timeout or self.timeout, context=self._ctx)  # noqa: S310
        except urllib.error.HTTPError as e:
            msg = e.read().decode(errors="replace")[:500]
            raise {404: NotFound, 409: Conflict if "AlreadyExists" not in msg else AlreadyExists,
                   403: Forbidden}.get(e.code, APIError)(f"{method} {path}: {e.code} {msg}") from None
        if stream:
            return resp
        with resp:
            raw = resp.read()
        return json.loads(raw) if raw else {}

    @staticmethod
    def _with_kind(o: Obj, kind: str) -> Obj:
        o.setdefault("kind", kind)
        return o

    # -- verbs ---------------------------------------------------------------------------
    def get(self, kind: str, name: str, namespace: str = "") -> Obj:
        return self._with_kind(self._req("GET", self._path(kind, name, namespace)), kind)

    def list(self, kind: str, namespace: Optional[str] = None, label_selector: Optional[str] = None,
             field_selector: Optional[str] = None, copy: bool = True) -> List[Obj]:
        # every REST response is a fresh decode: ``copy`` only matters for the in-memory server
        doc = self._req("GET", self._path(kind, "", namespace or ""),
                        query={"labelSelector": label_selector or "", "fieldSelector": field_selector or ""})
        return [self._with_kind(o, kind) for o in doc.get("items", [])]

    def create(self, obj: Obj) -> Obj:
        md = obj.get("metadata", {})
        return self._req("POST", self._path(obj["kind"], "", md.get("namespace", "")), obj)

    def update(self, obj: Obj) -> Obj:
        md = obj.get("metadata", {})
        return self._req("PUT", self._path(obj["kind"], md["name"], md.get("namespace", "")), obj)

    def patch(self, kind: str, name: str, patch: Obj, namespace: str = "") -> Obj:
        sub = ""
        if set(patch) == {"status"} and kind in ("Pod", "Node", "ElasticQuota", "CompositeElasticQuota"):
            sub = "status"
        return self._req("PATCH", self._path(kind, name, namespace, sub), patch,
                         content_type="application/merge-patch+json")

    def delete(self, kind: str, name: str, namespace: str = "") -> None:
        self._req("DELETE", self._path(kind, name, namespace))

    def bind(self, pod_name: str, namespace: str, node_name: str) -> Obj:
        body = {"apiVersion": "v1", "kind": "Binding", "metadata": {"name": pod_name, "namespace": namespace},
                "target": {"apiVersion": "v1", "kind": "Node", "name": node_name}}
        return self._req("POST", self._path("Pod", pod_name, namespace, "binding"), body)

    def watch(self, kind: str, handler: Callable[[str, Obj, Optional[Obj]], None], replay: bool = True,
              on_synced: Optional[Callable[[], None]] = None) -> Callable[[], None]:
        """Stream ``kind`` to ``handler`` from a watch thread: LIST (replayed as ADDED when
        ``replay``), then WATCH from the list's resourceVersion, re-listing on ``410 Gone``.
        ``on_synced`` is called once, on the watch thread, right after the first LIST has been
        delivered — the informer's "has synced", ordered with every later event of the stream."""
        stop = threading.Event()
        synced_once = threading.Event()
        self._watchers.append(stop)
        cache: Dict[Tuple[str, str], Obj] = {}

        def loop() -> None:
            rv = ""
            while not stop.is_set():
                try:
                    if not rv:
                        doc = self._req("GET", self._path(kind))
                        rv = doc.get("metadata", {}).get("resourceVersion", "")
                        seen = set()
                        for o in doc.get("items", []):
                            o = self._with_kind(o, kind)
                            k = (o["metadata"].get("namespace", ""), o["metadata"]["name"])
                            seen.add(k)
                            old = cache.get(k)
                            cache[k] = o
                            if replay or old is not None:
                                handler("ADDED" if old is None else "MODIFIED", o, old)
                        # a re-list after 410 Gone replaces the mirror: objects deleted while the watch
                        # was down get their DELETED now (an informer's Replace)
                        for k in [k for k in cache if k not in seen]:
                            gone = cache.pop(k)
                            handler("DELETED", gone, gone)
                        if on_synced is not None and not synced_once.is_set():
                            synced_once.set()
                            on_synced()
                    resp = self._req("GET", self._path(kind), query={"watch": "1", "resourceVersion": rv,
                                                                     "allowWatchBookmarks": "true"},
                                     stream=True, timeout=300)
                    with resp:
                        for line in resp:
                            if stop.is_set():
                                return
                            ev = json.loads(line)
                            t, o = ev.get("type"), ev.get("object", {})
                            if t == "ERROR":
                                rv = ""  # 410 Gone: re-list
                                break
                            rv = o.get("metadata", {}).get("resourceVersion", rv)
                            if t == "BOOKMARK":
                                continue
                            o = self._with_kind(o, kind)
                            k = (o["metadata"].get("namespace", ""), o["metadata"]["name"])
                            old = cache.get(k)
                            if t == "DELETED":
                                cache.pop(k, None)
                            else:
                                cache[k] = o
                            handler(t, o, old)
                except Exception as e:  # noqa: BLE001 - keep watching through transient errors
                    log.warning("watch %s: %s", kind, e)
                    stop.wait(1.0)

        threading.Thread(target=loop, name=f"watch-{kind}", daemon=True).start()
        return stop.set

    def close(self) -> None:
        for s in self._watchers:
            s.set()


def _materialize(data_b64: Optional[str], path: Optional[str], base: str, suffix: str) -> Optional[str]:
    """A kubeconfig credential as a file path: inline ``*-data`` (base64) is written to a private
    temporary file (ssl only loads certificates from files); relative paths resolve against the
    kubeconfig's directory, as kubectl does."""
    import base64
    import tempfile
    if data_b64:
        fd, name = tempfile.mkstemp(prefix="nos-kube-", suffix=suffix)
        with os.fdopen(fd, "wb") as f:
            f.write(base64.b64decode(data_b64))
        os.chmod(name, 0o600)
        return name
    if path:
        return path if os.path.isabs(path) else os.path.join(base, path)
    return None


def from_kubeconfig(path: str, context: Optional[str] = None) -> RESTClient:
    """kubeconfig support: the (current) context's cluster server, CA (file or inline data) and
    user credentials — bearer token (inline or ``tokenFile``) or client certificate + key (files or
    inline data)."""
    import yaml
    with open(path) as f:
        cfg = yaml.safe_load(f)
    base = os.path.dirname(os.path.abspath(path))
    ctx_name = context or cfg.get("current-context")
    ctx = next(c["context"] for c in cfg["contexts"] if c["name"] == ctx_name)
    cluster = next(c["cluster"] for c in cfg["clusters"] if c["name"] == ctx["cluster"])
    user = next((u["user"] for u in cfg.get("users", []) if u["name"] == ctx.get("user")), {}) or {}
    token = user.get("token", "")
    if not token and user.get("tokenFile"):
        with open(_materialize(None, user["tokenFile"], base, "")) as f:
            token = f.read().strip()
    ca = _materialize(cluster.get("certificate-authority-data"), cluster.get("certificate-authority"), base, ".crt")
    cert = _materialize(user.get("client-certificate-data"), user.get("client-certificate"), base, ".crt")
    key = _materialize(user.get("client-key-data"), user.get("client-key"), base, ".key")
    return RESTClient(cluster["server"], token, ca, insecure=bool(cluster.get("insecure-skip-tls-verify")),
                      cert_file=cert, key_file=key)

