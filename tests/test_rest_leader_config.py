"""REST client against a local HTTP stub, Lease leader election, ComponentConfig loading."""
import json
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from walkai_nos_amd.api.config import (CapacitySchedulingArgs, GpuAgentConfig, GpuPartitionerConfig, MigAgentConfig,
                                       dump_config, load_config)
from walkai_nos_amd.kube.errors import Conflict, NotFound
from walkai_nos_amd.kube.leader import LeaderElector
from walkai_nos_amd.kube.memory import InMemoryAPIServer
from walkai_nos_amd.kube.rest import RESTClient


class _Stub(BaseHTTPRequestHandler):
    calls = []
    node = {"apiVersion": "v1", "kind": "Node", "metadata": {"name": "n1", "resourceVersion": "5",
                                                              "annotations": {}}}

    def _send(self, code, body):
        data = json.dumps(body).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def do_GET(self):  # noqa: N802
        _Stub.calls.append(("GET", self.path, self.headers.get("Authorization")))
        if self.path.startswith("/api/v1/nodes/n1"):
            return self._send(200, _Stub.node)
        if self.path.startswith("/api/v1/nodes/missing"):
            return self._send(404, {"kind": "Status", "code": 404})
        if self.path.startswith("/api/v1/nodes?watch=1") or "watch=1" in self.path:
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.end_headers()
            for ev in ({"type": "MODIFIED", "object": dict(_Stub.node, metadata={"name": "n1", "resourceVersion": "6"})},
                       {"type": "DELETED", "object": dict(_Stub.node, metadata={"name": "n1", "resourceVersion": "7"})}):
                self.wfile.write((json.dumps(ev) + "\n").encode())
                self.wfile.flush()
            time.sleep(0.5)
            return None
        if self.path.startswith("/api/v1/nodes"):
            return self._send(200, {"metadata": {"resourceVersion": "5"}, "items": [_Stub.node]})
        return self._send(404, {})

    def do_PATCH(self):  # noqa: N802
        body = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
        _Stub.calls.append(("PATCH", self.path, self.headers.get("Content-Type"), body))
        if self.path.endswith("/conflict"):
            return self._send(409, {"reason": "Conflict"})
        return self._send(200, _Stub.node)

    def do_POST(self):  # noqa: N802
        body = json.loads(self.rfile.read(int(self.headers["Content-Length"])))
        _Stub.calls.append(("POST", self.path, body))
        return self._send(201, body)

    def log_message(self, *a):
        return


@pytest.fixture
def stub():
    srv = ThreadingHTTPServer(("127.0.0.1", 0), _Stub)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    _Stub.calls.clear()
    yield f"http://127.0.0.1:{srv.server_address[1]}"
    srv.shutdown()


def test_rest_client_verbs(stub):
    c = RESTClient(stub, token="tok")
    assert c.get("Node", "n1")["metadata"]["name"] == "n1"
    assert _Stub.calls[-1][2] == "Bearer tok"
    with pytest.raises(NotFound):
        c.get("Node", "missing")
    assert [n["kind"] for n in c.list("Node", label_selector="a=b")] == ["Node"]
    assert "labelSelector=a%3Db" in _Stub.calls[-1][1]
    c.patch("Node", "n1", {"metadata": {"annotations": {"x": "1"}}})
    assert _Stub.calls[-1][2] == "application/merge-patch+json"
    c.patch("Pod", "p", {"status": {"phase": "Running"}}, "ns")
    assert _Stub.calls[-1][1] == "/api/v1/namespaces/ns/pods/p/status"
    with pytest.raises(Conflict):
        c.patch("Node", "conflict", {"metadata": {}})
    c.bind("p", "ns", "n1")
    assert _Stub.calls[-1][1] == "/api/v1/namespaces/ns/pods/p/binding"
    assert _Stub.calls[-1][2]["target"]["name"] == "n1"


def test_rest_client_watch_stream(stub):
    c = RESTClient(stub)
    events = []
    done = threading.Event()

    def h(t, o, old):
        events.append((t, o["metadata"].get("resourceVersion")))
        if t == "DELETED":
            done.set()

    cancel = c.watch("Node", h)
    assert done.wait(5)
    cancel()
    assert events[:3] == [("ADDED", "5"), ("MODIFIED", "6"), ("DELETED", "7")]


def test_leader_election_single_holder_and_failover():
    t = [1000.0]
    api = InMemoryAPIServer()
    a = LeaderElector(api, "gpu-partitioner.nebuly.com", identity="a", lease_duration=15, renew_deadline=10,
                      clock=lambda: t[0])
    b = LeaderElector(api, "gpu-partitioner.nebuly.com", identity="b", lease_duration=15, renew_deadline=10,
                      clock=lambda: t[0])
    assert a.tick() and not b.tick()
    t[0] += 5
    assert a.tick() and not b.tick()  # renewal keeps a
    t[0] += 20                         # a stops renewing: lease expires, b takes over
    assert b.tick() and not a.is_leader()
    b.release()
    assert a.tick()


def test_component_configs_load_validate_and_roundtrip():
    text = """apiVersion: config.nos.nebuly.com/v1alpha1
kind: GpuPartitionerConfig
health: {healthProbeBindAddress: ":8081"}
metrics: {bindAddress: "127.0.0.1:8080"}
webhook: {port: 9443}
leaderElection: {leaderElect: true, resourceName: gpu-partitioner.nebuly.com, leaderElectionReleaseOnCancel: true}
batchWindowTimeoutSeconds: 60
batchWindowIdleSeconds: 10
knownMigGeometriesFile: known_mig_geometries.yaml
devicePluginConfigMap: {name: nos-device-plugin-config, namespace: nos-system}
devicePluginDelaySeconds: 5
"""
    cfg = load_config(text)
    assert isinstance(cfg, GpuPartitionerConfig) and cfg.leaderElection.leaderElect
    assert cfg.batchWindowTimeoutSeconds == 60 and cfg.devicePluginConfigMap.namespace == "nos-system"
    assert load_config(dump_config(cfg, "GpuPartitionerConfig")) == cfg
    with pytest.raises(ValueError):
        load_config(text.replace("batchWindowIdleSeconds: 10", "batchWindowIdleSeconds: 0"))
    with pytest.raises(ValueError):
        load_config(text + "unknownField: 1\n")
    agent = load_config("kind: MigAgentConfig\nleaderElection: {leaderElect: false}\nreportConfigIntervalSeconds: 10\n")
    assert isinstance(agent, MigAgentConfig) and agent.reportConfigIntervalSeconds == 10
    assert load_config("kind: MigAgentConfig\n").reportConfigIntervalSeconds == 10  # Q5: omitted -> 10 s
    assert isinstance(load_config("kind: SliceAgentConfig\n"), GpuAgentConfig)
    args = load_config("apiVersion: kubescheduler.config.k8s.io/v1beta3\nkind: CapacitySchedulingArgs\n"
                       "amdGpuResourceMemoryGB: 288\n")
    assert isinstance(args, CapacitySchedulingArgs) and args.nvidiaGpuResourceMemoryGB == 288


class _RelistStub(BaseHTTPRequestHandler):
    lists = 0

    def _send(self, code, body):
        data = json.dumps(body).encode()
        self.send_response(code)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(data)))
        self.end_headers()
        self.wfile.write(data)

    def do_GET(self):  # noqa: N802
        if "watch=1" in self.path:
            self.send_response(200)
            self.send_header("Content-Type", "application/json")
            self.end_headers()
            if _RelistStub.lists == 1:  # the first watch expires: 410 Gone -> re-list
                self.wfile.write((json.dumps({"type": "ERROR", "object": {"code": 410}}) + "\n").encode())
            self.wfile.flush()
            time.sleep(0.3)
            return None
        _RelistStub.lists += 1
        names = ["a", "b"] if _RelistStub.lists == 1 else ["a"]  # "b" was deleted while the watch was down
        return self._send(200, {"metadata": {"resourceVersion": str(10 + _RelistStub.lists)},
                                "items": [{"metadata": {"name": n, "resourceVersion": "1"}} for n in names]})

    def log_message(self, *a):
        return


def test_rest_watch_relist_drops_objects_deleted_during_the_gap():
    srv = ThreadingHTTPServer(("127.0.0.1", 0), _RelistStub)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    _RelistStub.lists = 0
    try:
        c = RESTClient(f"http://127.0.0.1:{srv.server_address[1]}")
        events = []
        done = threading.Event()

        def h(t, o, old):
            events.append((t, o["metadata"]["name"]))
            if t == "DELETED":
                done.set()

        cancel = c.watch("Node", h)
        assert done.wait(10)
        cancel()
        c.close()
        assert ("ADDED", "a") in events and ("ADDED", "b") in events
        assert ("DELETED", "b") in events and ("DELETED", "a") not in events
    finally:
        srv.shutdown()
