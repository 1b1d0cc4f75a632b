"""Process-level end to end: the real component binaries over HTTP (VERDICT r2 #1 follow-up).

``python -m walkai_nos_amd.cmd.gpupartitioner`` and ``python -m walkai_nos_amd.cmd.partitionagent``
run as separate OS processes with a kubeconfig pointing at the REST facade of the in-memory API
server (``kube/apiserver.py``).  The test plays the rest of the node and the cluster:

* kubelet — the Registration endpoint the agent's nos partition device plugin registers with
  (``deviceplugin/server.py``), a ListAndWatch reader per registered resource, admission through the
  plugin's ``Allocate`` over gRPC, and the PodResources endpoint the agent reads in-use devices from;
* kube-scheduler — :class:`~walkai_nos_amd.sim.cluster.KubeScheduler` (allocatable minus requests,
  no GPU knowledge) over the same REST client.

Scenario on a 1-GPU node (fake amd-smi inside the agent process): whole-GPU SPX at start; eight
1/8 pods make the partitioner ask for CPX and the agent flip; all eight are admitted on distinct
partitions; a whole-GPU pod arrives, the partitioner drains the busy GPU, the plugin reports every
CPX partition Unhealthy (a 1/8 pod arriving meanwhile is not placed); the 1/8 pods finish, the
agent flips back to SPX and the whole-GPU pod runs.  Reference counterpart: the envtest suites
(``internal/controllers/migagent/suite_int_test.go``) plus the kind-based e2e of the Helm chart.
"""
import os
import subprocess
import sys
import tempfile
import threading
import time
from types import SimpleNamespace

import grpc
import pytest

from walkai_nos_amd import constant
from walkai_nos_amd.api import v1alpha1 as api
from walkai_nos_amd.api.config import GpuPartitionerConfig, MigAgentConfig, dump_config
from walkai_nos_amd.device.podresources import PodResourcesServer
from walkai_nos_amd.device.protos import dp
from walkai_nos_amd.deviceplugin.partitions import draining_gpus
from walkai_nos_amd.deviceplugin.server import RegistrationServer
from walkai_nos_amd.kube import objects as ko
from walkai_nos_amd.kube.apiserver import APIFacade, parse_path
from walkai_nos_amd.kube.rest import from_kubeconfig
from walkai_nos_amd.sim.cluster import KubeScheduler

NODE = "node-0"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_parse_path_routes():
    r = parse_path("/api/v1/namespaces/team-a/pods/p1/status")
    assert (r.kind, r.namespace, r.name, r.sub) == ("Pod", "team-a", "p1", "status")
    r = parse_path("/api/v1/namespaces/team-a")
    assert (r.kind, r.name) == ("Namespace", "team-a")
    r = parse_path("/apis/nos.nebuly.com/v1alpha1/namespaces/ns/elasticquotas")
    assert (r.kind, r.namespace, r.name) == ("ElasticQuota", "ns", "")
    assert parse_path("/apis/unknown/v1/things") is None


def test_rest_client_against_the_facade_crud_watch_and_resume():
    f = APIFacade(bookmark_every=0.2).start()
    try:
        with tempfile.TemporaryDirectory() as d:
            c = from_kubeconfig(f.write_kubeconfig(os.path.join(d, "kc")))
            c.create(ko.new_node("n1", {"a": "b"}))
            seen, synced = [], threading.Event()
            c.watch("Pod", lambda t, o, old: seen.append((t, ko.name(o))), on_synced=synced.set)
            assert synced.wait(5)
            c.create(ko.new_pod("p1", "ns", requests={"amd.com/cpx_nps1": 1}))
            c.patch("Pod", "p1", {"status": {"phase": "Running"}}, "ns")
            c.bind("p1", "ns", "n1")
            with pytest.raises(Exception) as e:
                c.create(ko.new_pod("p1", "ns"))
            assert type(e.value).__name__ == "AlreadyExists"
            assert [ko.name(n) for n in c.list("Node", label_selector="a=b")] == ["n1"]
            assert c.list("Pod", field_selector="spec.nodeName=n1")[0]["status"]["phase"] == "Running"
            c.delete("Pod", "p1", "ns")
            deadline = time.time() + 5
            while len(seen) < 4 and time.time() < deadline:
                time.sleep(0.05)
            assert seen == [("ADDED", "p1"), ("MODIFIED", "p1"), ("MODIFIED", "p1"), ("DELETED", "p1")]
            time.sleep(0.5)                              # bookmarks keep an idle stream alive
            c.create(ko.new_pod("p2", "ns"))
            deadline = time.time() + 5
            while len(seen) < 5 and time.time() < deadline:
                time.sleep(0.05)
            assert seen[-1] == ("ADDED", "p2")
            c.close()
    finally:
        f.stop()


class _Kubelet:
    """The node's kubelet, as far as the agent and its device plugin can tell."""

    def __init__(self, d, client):
        self.dir = os.path.join(d, "device-plugins")
        os.makedirs(self.dir)
        self.client = client
        self.reg = RegistrationServer(os.path.join(self.dir, "kubelet.sock")).start()
        self.devices = {}       # resource -> [(id, health)] (latest ListAndWatch response)
        self.readers = {}       # resource -> (endpoint, thread)
        self.used = {}          # (ns, pod) -> (resource, device id)
        self.admission_failures = []
        self.lock = threading.Lock()
        self.podres = PodResourcesServer(os.path.join(d, "pod-resources.sock"), self._used, self._alloc).start()

    def _used(self):
        with self.lock:
            return [(p, ns, [(r, [i])]) for (ns, p), (r, i) in self.used.items()]

    def _alloc(self):
        with self.lock:
            return [(r, [i for i, _ in ds]) for r, ds in self.devices.items()]

    def _read(self, resource, endpoint):
        ch = grpc.insecure_channel("unix://" + os.path.join(self.dir, endpoint))
        law = ch.unary_stream(f"/{dp.SERVICE}/ListAndWatch", request_serializer=dp.Empty.SerializeToString,
                              response_deserializer=dp.ListAndWatchResponse.FromString)
        try:
            for resp in law(dp.Empty()):
                with self.lock:
                    self.devices[resource] = [(x.ID, x.health) for x in resp.devices]
        except grpc.RpcError:
            pass
        finally:
            ch.close()

    def sync(self):
        latest = {r.resource_name: r.endpoint for r in self.reg.registered}
        for res, ep in latest.items():
            cur = self.readers.get(res)
            if cur is None or cur[0] != ep or not cur[1].is_alive():
                t = threading.Thread(target=self._read, args=(res, ep), daemon=True)
                t.start()
                self.readers[res] = (ep, t)

    def admit(self, pod, node):
        """kubelet admission: a healthy free device of the requested resource, handed out by the
        plugin's Allocate; a pod nothing can serve fails as UnexpectedAdmissionError."""
        r = next(k for k in pod["spec"]["containers"][0]["resources"]["requests"] if k.startswith("amd.com/"))
        key = (ko.namespace(pod), ko.name(pod))
        with self.lock:
            taken = {i for _, i in self.used.values()}
            free = [i for i, h in self.devices.get(r, []) if h == dp.HEALTHY and i not in taken]
        try:
            if not free:
                raise RuntimeError(f"no healthy {r}")
            ch = grpc.insecure_channel("unix://" + os.path.join(self.dir, self.readers[r][0]))
            req = dp.AllocateRequest()
            req.container_requests.add(devicesIDs=[free[0]])
            resp = ch.unary_unary(f"/{dp.SERVICE}/Allocate", request_serializer=dp.AllocateRequest.SerializeToString,
                                  response_deserializer=dp.AllocateResponse.FromString)(req, timeout=5)
            ch.close()
            assert resp.container_responses[0].devices[0].host_path == "/dev/kfd"
        except Exception as e:  # noqa: BLE001 - an admission failure is a result, not a test error
            self.admission_failures.append((key, str(e)))
            self.client.patch("Pod", key[1], {"status": {"phase": "Failed", "reason": "UnexpectedAdmissionError"}},
                              key[0])
            return
        with self.lock:
            self.used[key] = (r, free[0])
        self.client.patch("Pod", key[1], {"status": {"phase": "Running"}}, key[0])

    def finish(self, ns, name):
        with self.lock:
            self.used.pop((ns, name), None)
        self.client.patch("Pod", name, {"status": {"phase": "Succeeded"}}, ns)
        self.client.delete("Pod", name, ns)

    def stop(self):
        self.reg.stop()
        self.podres.stop()


def _spawn(module, cfg_path, kubeconfig, log_path, env=None):
    e = dict(os.environ, PYTHONPATH=REPO, **(env or {}))
    return subprocess.Popen([sys.executable, "-m", module, "--config", cfg_path, "--kubeconfig", kubeconfig],
                            stdout=open(log_path, "w"), stderr=subprocess.STDOUT, env=e, cwd=REPO)


def _tail(path, n=40):
    with open(path) as f:
        return "".join(f.readlines()[-n:])


def test_partitioner_and_agent_processes_flip_drain_and_flip_back():
    facade = APIFacade(bookmark_every=2.0).start()
    procs, kubelet = [], None
    with tempfile.TemporaryDirectory() as d:
        try:
            kc = facade.write_kubeconfig(os.path.join(d, "kubeconfig"))
            client = from_kubeconfig(kc)
            labels = {api.LABEL_GPU_PARTITIONING: api.PARTITIONING_KIND_XCP,
                      constant.LABEL_AMD_GPU_PRODUCT: "AMD_Instinct_MI355X", constant.LABEL_AMD_GPU_COUNT: "1",
                      constant.LABEL_AMD_GPU_VRAM: "288G", constant.LABEL_AMD_GPU_CU_COUNT: "256"}
            client.create(ko.new_node(NODE, labels))
            kubelet = _Kubelet(d, client)
            agent_cfg = MigAgentConfig(healthProbeBindAddress="0", metricsBindAddress="0",
                                       reportConfigIntervalSeconds=1.0, amdSmiBackend="fake", fakeGpus=1,
                                       podResourcesSocket=os.path.join(d, "pod-resources.sock"),
                                       commitBarrier="none", probeOnCommit=False, devicePlugin="nos",
                                       devicePluginDir=kubelet.dir)
            part_cfg = GpuPartitionerConfig(healthProbeBindAddress="0", metricsBindAddress="0",
                                            batchWindowTimeoutSeconds=1.0, batchWindowIdleSeconds=0.3,
                                            planningPolicy="pack",
                                            packing={"minStintSeconds": 0, "unservedAfterSeconds": 1,
                                                     "drainGainAfterSeconds": 1, "replanEverySeconds": 0.2})
            paths = {}
            for name, cfg, kind in (("agent", agent_cfg, "MigAgentConfig"),
                                    ("partitioner", part_cfg, "GpuPartitionerConfig")):
                paths[name] = os.path.join(d, f"{name}.yaml")
                with open(paths[name], "w") as f:
                    f.write(dump_config(cfg, kind))
            logs = {n: os.path.join(d, f"{n}.log") for n in paths}
            procs.append(_spawn("walkai_nos_amd.cmd.partitionagent", paths["agent"], kc, logs["agent"],
                                {constant.ENV_NODE_NAME: NODE}))
            procs.append(_spawn("walkai_nos_amd.cmd.gpupartitioner", paths["partitioner"], kc, logs["partitioner"]))
            sched = KubeScheduler(client, {NODE: SimpleNamespace(name=NODE)}, on_bind=kubelet.admit)

            def run_until(cond, timeout, what):
                deadline = time.time() + timeout
                while time.time() < deadline:
                    for p in procs:
                        if p.poll() is not None:
                            raise AssertionError(f"a component exited ({p.returncode}) while waiting for {what}:\n"
                                                 + "\n".join(_tail(x) for x in logs.values()))
                    kubelet.sync()
                    sched.reconcile(KubeScheduler.KEY)
                    if cond():
                        return
                    time.sleep(0.2)
                raise AssertionError(f"timed out waiting for {what}\n" + "\n".join(
                    f"--- {n}\n{_tail(x)}" for n, x in logs.items()) + f"\nkubelet devices {kubelet.devices}\n"
                    f"node annotations {ko.annotations(client.get('Node', NODE))}")

            def alloc(r):
                return int(ko.node_allocatable(client.get("Node", NODE)).get(f"amd.com/{r}", "0"))

            def phase(name):
                return ko.pod_phase(client.get("Pod", name, "default"))

            # 1. the agent reports the whole GPU and its plugin serves it
            run_until(lambda: alloc("spx_nps1") == 1 and kubelet.devices.get("amd.com/spx_nps1"), 30,
                      "the SPX partition to be served")
            # 2. eight 1/8 pods: the partitioner asks for CPX, the agent flips, kubelet admits all eight
            for i in range(8):
                client.create(ko.new_pod(f"c{i}", requests={"amd.com/cpx_nps1": 1}))
            run_until(lambda: all(phase(f"c{i}") == "Running" for i in range(8)), 60, "the eight 1/8 pods to run")
            assert len({i for _, i in kubelet.used.values()}) == 8
            assert alloc("spx_nps1") == 0
            # 3. a whole-GPU pod: the busy GPU is drained; every CPX partition reported Unhealthy
            client.create(ko.new_pod("big", requests={"amd.com/spx_nps1": 1}))
            run_until(lambda: 0 in draining_gpus(ko.annotations(client.get("Node", NODE))), 60, "the drain")
            run_until(lambda: [h for _, h in kubelet.devices["amd.com/cpx_nps1"]] == [dp.UNHEALTHY] * 8
                      and alloc("cpx_nps1") == 0, 20, "the plugin to withhold the draining GPU")
            client.create(ko.new_pod("late", requests={"amd.com/cpx_nps1": 1}))
            for i in range(4):      # half of the 1/8 pods finish; their partitions are not refilled
                kubelet.finish("default", f"c{i}")
            t_end = time.time() + 3
            run_until(lambda: time.time() > t_end, 10, "a few scheduling rounds")
            assert phase("late") == "Pending" and not ko.pod_node_name(client.get("Pod", "late", "default"))
            # 4. the rest finish: the agent flips back to SPX and the whole-GPU pod runs
            for i in range(4, 8):
                kubelet.finish("default", f"c{i}")
            run_until(lambda: phase("big") == "Running", 60, "the whole-GPU pod to run")
            assert kubelet.used[("default", "big")][0] == "amd.com/spx_nps1"
            assert kubelet.admission_failures == []
        finally:
            for p in procs:
                p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=10)
                except subprocess.TimeoutExpired:
                    p.kill()
            if kubelet is not None:
                kubelet.stop()
            facade.stop()
