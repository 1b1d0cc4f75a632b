"""Informer-cache client (reads from a list+watch mirror, writes through) and kubeconfig
credentials (client certificate / inline data / token file)."""
import base64
import os
import subprocess
import tempfile

import pytest

from walkai_nos_amd.kube import objects as ko
from walkai_nos_amd.kube.cache import CachedClient
from walkai_nos_amd.kube.errors import NotFound
from walkai_nos_amd.kube.memory import InMemoryAPIServer
from walkai_nos_amd.kube.rest import from_kubeconfig


def backing():
    api = InMemoryAPIServer()
    api.create(ko.new_node("n1", {"nos.nebuly.com/gpu-partitioning": "xcp"}))
    api.create(ko.new_node("n2"))
    api.create(ko.new_pod("p1", "default", requests={"amd.com/cpx_nps1": 1}))
    return api


def test_reads_come_from_the_cache_and_writes_go_through():
    api = backing()
    c = CachedClient(api, kinds=("Node", "Pod"))
    assert [ko.name(n) for n in c.list("Node")] == ["n1", "n2"]
    assert len(c.list("Pod")) == 1          # informers start (LIST + WATCH) on first use
    before = dict(api.stats)
    for _ in range(20):
        assert ko.name(c.get("Node", "n1")) == "n1"
        assert [ko.name(n) for n in c.list("Node", label_selector="nos.nebuly.com/gpu-partitioning=xcp")] == ["n1"]
        assert [ko.name(p) for p in c.list("Pod", field_selector="status.phase=Pending")] == ["p1"]
    assert api.stats.get("get", 0) == before.get("get", 0)      # no API round trip per read
    assert api.stats.get("list", 0) == before.get("list", 0)
    with pytest.raises(NotFound):
        c.get("Node", "nope")
    # a write is visible to the very next read (write-through), and bumps the revision
    rev = c.revision
    c.patch("Node", "n2", {"metadata": {"annotations": {"a": "1"}}})
    assert ko.annotations(c.get("Node", "n2"))["a"] == "1"
    assert c.revision > rev
    # changes made by someone else arrive through the watch
    api.patch("Node", "n1", {"metadata": {"labels": {"x": "y"}}})
    assert ko.labels(c.get("Node", "n1"))["x"] == "y"
    api.delete("Pod", "p1", "default")
    assert c.list("Pod") == []
    # reads hand out copies: mutating one never corrupts the cache
    n = c.get("Node", "n1")
    n["metadata"]["labels"]["x"] = "mutated"
    assert ko.labels(c.get("Node", "n1"))["x"] == "y"


def test_watch_fan_out_and_uncached_kinds_pass_through():
    api = backing()
    c = CachedClient(api, kinds=("Node",))
    seen_a, seen_b = [], []
    c.watch("Node", lambda t, o, old: seen_a.append((t, ko.name(o))))
    cancel = c.watch("Node", lambda t, o, old: seen_b.append((t, ko.name(o))), replay=False)
    api.patch("Node", "n2", {"metadata": {"labels": {"k": "v"}}})
    assert ("ADDED", "n1") in seen_a and ("MODIFIED", "n2") in seen_a
    assert seen_b == [("MODIFIED", "n2")]
    cancel()
    api.patch("Node", "n2", {"metadata": {"labels": {"k": "w"}}})
    assert seen_b == [("MODIFIED", "n2")]
    # Pods are not cached here: reads go to the API server
    before = api.stats.get("list", 0)
    assert [ko.name(p) for p in c.list("Pod")] == ["p1"]
    assert api.stats.get("list", 0) == before + 1


def test_stale_events_never_roll_the_cache_back():
    api = backing()
    c = CachedClient(api, kinds=("Node",))
    inf = c.informer("Node")
    c.patch("Node", "n1", {"metadata": {"labels": {"fresh": "1"}}})
    cur = c.get("Node", "n1")
    stale_rv = str(int(cur["metadata"]["resourceVersion"]) - 1)
    old = dict(cur, metadata=dict(cur["metadata"], resourceVersion=stale_rv, labels={"stale": "1"}))
    inf.apply("MODIFIED", old)
    assert "stale" not in ko.labels(c.get("Node", "n1"))


def test_pod_controller_memo_works_through_the_cache():
    from walkai_nos_amd.controllers.partitioner.pod_controller import PodController
    api = backing()
    c = CachedClient(api, kinds=("Node", "Pod"))
    ctl = PodController(c)
    assert ctl.reconcile(ctl.plan_key) == ctl.reconcile(ctl.plan_key)
    assert c.revision == c.revision  # exposed, so the memo keys on it


def _self_signed(d):
    key, crt = os.path.join(d, "k.pem"), os.path.join(d, "c.pem")
    subprocess.run(["openssl", "req", "-x509", "-newkey", "rsa:2048", "-nodes", "-subj", "/CN=nos-test", "-days", "1",
                    "-keyout", key, "-out", crt], check=True, capture_output=True)
    return key, crt


def test_kubeconfig_client_certificate_and_inline_data():
    import yaml
    with tempfile.TemporaryDirectory() as d:
        key, crt = _self_signed(d)
        b64 = lambda p: base64.b64encode(open(p, "rb").read()).decode()  # noqa: E731
        cfg = {"current-context": "kind", "contexts": [{"name": "kind", "context": {"cluster": "c", "user": "u"}}],
               "clusters": [{"name": "c", "cluster": {"server": "https://127.0.0.1:6443",
                                                      "certificate-authority-data": b64(crt)}}],
               "users": [{"name": "u", "user": {"client-certificate-data": b64(crt), "client-key-data": b64(key)}}]}
        path = os.path.join(d, "kubeconfig")
        with open(path, "w") as f:
            yaml.safe_dump(cfg, f)
        c = from_kubeconfig(path)
        assert c.server == "https://127.0.0.1:6443" and c.token == "" and c.cert_file
        assert open(c.cert_file, "rb").read() == open(crt, "rb").read()
        assert oct(os.stat(c.cert_file).st_mode & 0o777) == "0o600"
        # file references relative to the kubeconfig + a token file
        with open(os.path.join(d, "tok"), "w") as f:
            f.write("s3cr3t\n")
        cfg["clusters"][0]["cluster"] = {"server": "https://10.0.0.1", "certificate-authority": "c.pem"}
        cfg["users"][0]["user"] = {"tokenFile": "tok"}
        with open(path, "w") as f:
            yaml.safe_dump(cfg, f)
        c = from_kubeconfig(path)
        assert c.token == "s3cr3t" and c.cert_file is None


class _DelayedPodEvents:
    """An API server whose Pod watch events are held back until ``flush()`` (a slow watch)."""

    def __init__(self, api):
        self.api = api
        self.held = []

    def __getattr__(self, name):
        return getattr(self.api, name)

    def watch(self, kind, handler, replay=True, on_synced=None):
        if kind != "Pod":
            return self.api.watch(kind, handler, replay, on_synced)
        live = [False]

        def hold(t, o, old):
            if live[0]:
                self.held.append((handler, t, o, old))
            else:
                handler(t, o, old)
        cancel = self.api.watch(kind, hold, replay, on_synced)
        live[0] = True
        return cancel

    def flush(self):
        held, self.held = self.held, []
        for h, t, o, old in held:
            h(t, o, old)


def test_bind_is_assumed_until_the_watch_confirms_it():
    """a scheduling cycle that starts before the binding's watch event must still see
    the pod on its node, or it places the next pod on capacity that pod already holds."""
    from walkai_nos_amd.quota.scheduler import NosScheduler
    api = InMemoryAPIServer()
    api.create(ko.new_node("n1", allocatable={"cpu": "8", "memory": "8Gi", "pods": "10", "amd.com/spx_nps1": "1"}))
    for name in ("a", "b"):
        api.create(ko.new_pod(name, "default", requests={"amd.com/spx_nps1": 1}, scheduler_name="nos-scheduler"))
    slow = _DelayedPodEvents(api)
    c = CachedClient(slow, kinds=("Node", "Pod"))
    s = NosScheduler(c)
    s.reconcile(NosScheduler.KEY)                       # binds a; its watch event is held back
    assert ko.pod_node_name(api.get("Pod", "a", "default")) == "n1"
    assert ko.pod_node_name(c.get("Pod", "a", "default")) == "n1"   # assumed in the cache
    # an older event (e.g. a status patch made before the binding) must not un-assume it
    stale = c.get("Pod", "a", "default")
    stale["spec"].pop("nodeName")
    c.informer("Pod").apply("MODIFIED", stale)
    assert ko.pod_node_name(c.get("Pod", "a", "default")) == "n1"
    s.reconcile(NosScheduler.KEY)                       # a new cycle before the watch caught up
    assert not ko.pod_node_name(api.get("Pod", "b", "default"))     # n1's only GPU is taken
    slow.flush()
    assert ko.pod_node_name(c.get("Pod", "a", "default")) == "n1"
    assert c.informer("Pod").assumed == {}


class _ListRacesWatch:
    """Watch replays p1, then p1 is deleted before the informer could have listed again; a LIST
    issued now would return the stale view that still holds p1."""

    def __init__(self):
        self.api = backing()
        self.lists = 0

    def __getattr__(self, name):
        return getattr(self.api, name)

    def list(self, kind, *a, **kw):
        self.lists += 1
        stale = self.api.list(kind, *a, **kw)
        return stale

    def watch(self, kind, handler, replay=True, on_synced=None):
        snapshot = self.api.list(kind)
        for o in snapshot:
            handler("ADDED", o, None)
        if kind == "Pod":
            gone = self.api.get("Pod", "p1", "default")
            handler("DELETED", gone, gone)              # arrives on the watch before "synced"
        if on_synced is not None:
            on_synced()
        return lambda: None


def test_informer_syncs_from_its_watch_without_a_second_list():
    """no second LIST after the watch's own replay, so a DELETED that arrives in between
    can never be undone by a stale ADDED (a zombie pod the planner would keep planning for)."""
    api = _ListRacesWatch()
    c = CachedClient(api, kinds=("Pod",))
    assert c.list("Pod") == []
    assert api.lists == 0
