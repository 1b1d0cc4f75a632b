"""Process-level end to end: the real component binaries over HTTP (VERDICT r2 #1 follow-up).

``python -m walkai_nos_amd.cmd.gpupartitioner`` and ``python -m walkai_nos_amd.cmd.partitionagent``
run as separate OS processes with a kubeconfig pointing at the REST facade of the in-memory API
server (``kube/apiserver.py``).  The test plays the rest of the node and the cluster:

* kubelet — ``testing/kubelet.py``: the Registration endpoint the agent's nos partition device
  plugin registers with, a ListAndWatch reader per registered resource, admission through the
  plugin's ``Allocate`` over gRPC, and the PodResources endpoint the agent reads in-use devices from;
* kube-scheduler — :class:`~walkai_nos_amd.sim.cluster.KubeScheduler` (allocatable minus requests,
  no GPU knowledge) over the same REST client.

``cmd/devcluster.py`` (``nos-devcluster``) wires these together; the last test runs its ``--demo``.

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

import pytest

from walkai_nos_amd.cmd.devcluster import DevCluster
from walkai_nos_amd.device.protos import dp
from walkai_nos_amd.deviceplugin.partitions import draining_gpus
from walkai_nos_amd.kube import objects as ko
from walkai_nos_amd.kube.apiserver import APIFacade, parse_path
from walkai_nos_amd.kube.rest import from_kubeconfig

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


def test_partitioner_and_agent_processes_flip_drain_and_flip_back():
    with tempfile.TemporaryDirectory() as d:
        c = DevCluster(d, nodes=1, gpus=1, bookmark_every=2.0)
        try:
            c.start()
            kubelet = c.kubelets[NODE]
            client = c.client

            def cpx_health():
                return [h for _, h in kubelet.devices.get("amd.com/cpx_nps1", [])]

            # 1. the agent reports the whole GPU and its plugin serves it
            c.run_until(lambda: c.allocatable(NODE, "spx_nps1") == 1 and kubelet.healthy("amd.com/spx_nps1"), 30,
                        "the SPX partition to be served")
            # 2. eight 1/8 pods: the partitioner asks for CPX, the agent flips, kubelet admits all eight
            for i in range(8):
                c.submit(f"c{i}", "cpx_nps1")
            c.run_until(lambda: all(c.phase(f"c{i}") == "Running" for i in range(8)), 60, "the eight 1/8 pods to run")
            assert len({i for _, i in kubelet.used.values()}) == 8
            assert c.allocatable(NODE, "spx_nps1") == 0
            # 3. a whole-GPU pod: the busy GPU is drained; every CPX partition reported Unhealthy
            c.submit("big", "spx_nps1")
            c.run_until(lambda: 0 in draining_gpus(ko.annotations(client.get("Node", NODE))), 60, "the drain")
            c.run_until(lambda: cpx_health() == [dp.UNHEALTHY] * 8 and c.allocatable(NODE, "cpx_nps1") == 0, 20,
                        "the plugin to withhold the draining GPU")
            c.submit("late", "cpx_nps1")
            for i in range(4):      # half of the 1/8 pods finish; their partitions are not refilled
                kubelet.finish("default", f"c{i}")
            t_end = time.time() + 3
            c.run_until(lambda: time.time() > t_end, 10, "a few scheduling rounds")
            assert c.phase("late") == "Pending" and not ko.pod_node_name(client.get("Pod", "late", "default"))
            # 4. the rest finish: the agent flips back to SPX and the whole-GPU pod runs
            for i in range(4, 8):
                kubelet.finish("default", f"c{i}")
            c.run_until(lambda: c.phase("big") == "Running", 60, "the whole-GPU pod to run")
            assert kubelet.used[("default", "big")][0] == "amd.com/spx_nps1"
            assert kubelet.admission_failures == []
        finally:
            c.stop()


@pytest.mark.parametrize("layout", ["slices", None])
def test_sliced_gpu_runs_cpx_and_dpx_pods_at_once_over_processes(layout):
    """VERDICT r3 #1 (mixed geometry): the real partitioner and partition agent processes on a
    1-GPU node labelled ``nos.nebuly.com/xcp-layout=slices`` — or carrying no layout label at all
    (the partitioner's ``defaultXcpLayout``, slices). A 1/2 pod and two 1/8 pods run on the one GPU
    at the same time, on disjoint CU masks handed out by the plugin's ``Allocate``, with no amd-smi
    switch; a 1/4 pod is then re-carved in next to them (no drain); when they finish, a whole-GPU
    pod takes the GPU."""
    import json
    from walkai_nos_amd.api import v1alpha1 as api
    from walkai_nos_amd.cmd.devcluster import fast_partitioner_config
    from walkai_nos_amd.models.slicing.cumask import XCDS
    with tempfile.TemporaryDirectory() as d:
        c = DevCluster(d, nodes=1, gpus=1, bookmark_every=2.0, layout=layout,
                       partitioner=fast_partitioner_config(sliceReserveAfterSeconds=1))
        try:
            c.start()
            kubelet = c.kubelets[NODE]
            assert (api.LABEL_XCP_LAYOUT in ko.labels(c.client.get("Node", NODE))) == (layout is not None)
            c.run_until(lambda: ko.annotations(c.client.get("Node", NODE)).get(api.ANNOTATION_SLICED_GPUS_STATUS) == "0",
                        30, "the GPU to be served sliced")
            c.submit("half", "dpx_nps1")
            c.submit("e0", "cpx_nps1")
            c.submit("e1", "cpx_nps1")
            c.run_until(lambda: all(c.phase(n) == "Running" for n in ("half", "e0", "e1")), 60,
                        "the 1/2 and 1/8 pods to run together")

            def cus(name):
                mask = kubelet.envs[("default", name)]["HSA_CU_MASK"]
                out = set()
                for r in mask.split(":", 1)[1].split(","):
                    a, _, b = r.partition("-")
                    out.update(range(int(a), int(b or a) + 1))
                return out
            sets = {n: cus(n) for n in ("half", "e0", "e1")}
            assert [len(sets[n]) for n in ("half", "e0", "e1")] == [128, 32, 32]
            assert not (sets["half"] & sets["e0"]) and not (sets["half"] & sets["e1"]) and not (sets["e0"] & sets["e1"])
            assert all({c_ % XCDS for c_ in v} == set(range(XCDS)) for v in sets.values())   # every slice spans all XCDs
            assert kubelet.envs[("default", "e0")]["NOS_HBM_LIMIT_BYTES"] == str(36 * 10**9)
            # a 1/4 pod: the free groups are re-carved next to the running pods
            c.submit("quarter", "qpx_nps1")
            c.run_until(lambda: c.phase("quarter") == "Running", 60, "the 1/4 pod")
            assert all(c.phase(n) == "Running" for n in ("half", "e0", "e1"))
            # everything leaves; a whole-GPU pod takes the GPU (no mask: all 256 CUs)
            c.submit("whole", "spx_nps1")
            for n in ("half", "e0", "e1", "quarter"):
                kubelet.finish("default", n)
            c.run_until(lambda: c.phase("whole") == "Running", 60, "the whole-GPU pod")
            assert "HSA_CU_MASK" not in kubelet.envs[("default", "whole")]
            path = os.path.join(d, NODE, "fake-amdsmi.json")
            if os.path.exists(path):                     # written on every amd-smi mode change
                with open(path) as f:
                    assert [g["compute"].upper() for g in json.load(f)] == ["SPX"]
            assert kubelet.admission_failures == []
        finally:
            c.stop()


def test_devcluster_demo_runs_to_completion():
    """``nos-devcluster --demo`` end to end (two nodes): eight 1/8 pods, then a whole-GPU pod."""
    with tempfile.TemporaryDirectory() as d:
        r = subprocess.run([sys.executable, "-m", "walkai_nos_amd.cmd.devcluster", "--nodes", "2", "--gpus", "1",
                            "--demo", "--dir", d], capture_output=True, text=True, timeout=240,
                           env=dict(os.environ, PYTHONPATH=REPO))
        assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
        assert "the whole-GPU pod runs on node-" in r.stdout and "every pod finished" in r.stdout


def test_quota_processes_borrow_and_reclaim():
    """nos-operator and nos-scheduler as processes too: team A borrows team B's idle guaranteed
    share (a second whole GPU), team B's pod then reclaims it — nos-scheduler preempts A's
    over-quota pod and binds B's, the operator keeps `used` and the in/over-quota labels current."""
    from walkai_nos_amd.api import v1alpha1 as api

    def quota(ns):
        return {"apiVersion": api.API_VERSION, "kind": api.KIND_ELASTIC_QUOTA,
                "metadata": {"name": f"q-{ns}", "namespace": ns},
                "spec": {"min": {api.RESOURCE_GPU_MEMORY: "288"}}}

    with tempfile.TemporaryDirectory() as d:
        c = DevCluster(d, nodes=2, gpus=1, quota=True)
        try:
            c.start()
            c.run_until(lambda: all(c.allocatable(n, "spx_nps1") == 1 for n in c.kubelets), 30, "both GPUs served")
            for ns in ("team-a", "team-b"):
                c.client.create(quota(ns))
            for name in ("a1", "a2"):
                c.submit(name, "spx_nps1", namespace="team-a", scheduler_name="nos-scheduler")
            c.run_until(lambda: all(c.phase(n, "team-a") == "Running" for n in ("a1", "a2")), 60,
                        "team A's two whole-GPU pods (one borrowed)")

            def caps():
                return sorted(ko.labels(p).get(api.LABEL_CAPACITY_INFO, "") for p in c.client.list("Pod", "team-a"))
            c.run_until(lambda: caps() == [api.CAPACITY_IN_QUOTA, api.CAPACITY_OVER_QUOTA], 30, "capacity labels")
            c.submit("b1", "spx_nps1", namespace="team-b", scheduler_name="nos-scheduler")
            c.run_until(lambda: c.phase("b1", "team-b") == "Running", 90, "team B's reclaiming pod")
            assert len(c.client.list("Pod", "team-a")) == 1       # the over-quota pod was preempted

            def used(ns):
                q = c.client.get(api.KIND_ELASTIC_QUOTA, f"q-{ns}", ns)
                return (q.get("status", {}).get("used") or {}).get(api.RESOURCE_GPU_MEMORY)
            c.run_until(lambda: used("team-a") == "288" and used("team-b") == "288", 30, "quota status")
        finally:
            c.stop()


def test_quota_reclaim_that_needs_a_mode_flip_over_processes():
    """Team A borrows both GPUs in CPX (16 x 1/8 GPU); team B reclaims a whole SPX GPU.  No node
    offers spx, so ordinary preemption cannot help: nos-scheduler evicts every pod of one GPU (all
    over-quota, per the agent's status-pods annotation), holds B's request against its quota so A
    cannot take the GPU back, and the partitioner flips the idle GPU for B."""
    from walkai_nos_amd.api import v1alpha1 as api

    def quota(ns):
        return {"apiVersion": api.API_VERSION, "kind": api.KIND_ELASTIC_QUOTA,
                "metadata": {"name": f"q-{ns}", "namespace": ns},
                "spec": {"min": {api.RESOURCE_GPU_MEMORY: "288"}}}

    with tempfile.TemporaryDirectory() as d:
        c = DevCluster(d, nodes=1, gpus=2, quota=True)
        try:
            c.start()
            c.run_until(lambda: c.allocatable("node-0", "spx_nps1") == 2, 30, "two idle GPUs")
            for ns in ("team-a", "team-b"):
                c.client.create(quota(ns))
            for i in range(16):
                c.submit(f"a{i}", "cpx_nps1", namespace="team-a", scheduler_name="nos-scheduler")
            c.run_until(lambda: all(c.phase(f"a{i}", "team-a") == "Running" for i in range(16)), 90,
                        "team A on both GPUs in CPX")
            c.submit("b0", "spx_nps1", namespace="team-b", scheduler_name="nos-scheduler")
            # team A keeps resubmitting (as a Job controller would): the held quota keeps them pending
            for i in range(16, 20):
                c.submit(f"a{i}", "cpx_nps1", namespace="team-a", scheduler_name="nos-scheduler")
            c.run_until(lambda: c.phase("b0", "team-b") == "Running", 120, "team B's whole GPU")
            running_a = [p for p in c.client.list("Pod", "team-a") if p.get("status", {}).get("phase") == "Running"]
            assert len(running_a) == 8                      # one GPU's worth of A's pods was evicted
            b0 = c.client.get("Pod", "b0", "team-b")
            assert ko.annotations(b0).get(api.ANNOTATION_QUOTA_RECLAIM) == "node-0"
            assert all(c.phase(f"a{i}", "team-a") == "Pending" for i in range(16, 20))
        finally:
            c.stop()


def test_quota_reclaim_on_a_sliced_gpu_over_processes():
    """ERQ on a sliced GPU with every component a process: team A borrows team B's half of the one
    GPU (8 x 1/8 pods, min 144 GB each); team B's 1/2 pod reclaims it. nos-scheduler evicts only the
    A pods whose row groups B's slice needs (4 of them: an aligned half), the agent re-carves the
    freed groups into B's slice without a mode switch, and A keeps its guaranteed half running."""
    import json
    from walkai_nos_amd.api import v1alpha1 as api
    from walkai_nos_amd.cmd.devcluster import fast_partitioner_config

    def quota(ns):
        return {"apiVersion": api.API_VERSION, "kind": api.KIND_ELASTIC_QUOTA,
                "metadata": {"name": f"q-{ns}", "namespace": ns},
                "spec": {"min": {api.RESOURCE_GPU_MEMORY: "144"}}}

    with tempfile.TemporaryDirectory() as d:
        c = DevCluster(d, nodes=1, gpus=1, quota=True, bookmark_every=2.0, layout="slices",
                       partitioner=fast_partitioner_config(sliceReserveAfterSeconds=1))
        try:
            c.start()
            kubelet = c.kubelets[NODE]
            c.run_until(lambda: ko.annotations(c.client.get("Node", NODE)).get(api.ANNOTATION_SLICED_GPUS_STATUS) == "0",
                        30, "the GPU to be served sliced")
            for ns in ("team-a", "team-b"):
                c.client.create(quota(ns))
            for i in range(8):
                c.submit(f"a{i}", "cpx_nps1", namespace="team-a", scheduler_name="nos-scheduler")
            c.run_until(lambda: all(c.phase(f"a{i}", "team-a") == "Running" for i in range(8)), 90,
                        "team A on the whole GPU in 1/8 slices")
            c.submit("b0", "dpx_nps1", namespace="team-b", scheduler_name="nos-scheduler")
            c.run_until(lambda: c.phase("b0", "team-b") == "Running", 120, "team B's half of the GPU")
            running_a = [ko.name(p) for p in c.client.list("Pod", "team-a")
                         if p.get("status", {}).get("phase") == "Running"]
            assert len(running_a) == 4, running_a            # only the pods on B's half were evicted
            mask = kubelet.envs[("team-b", "b0")]["HSA_CU_MASK"]
            b_cus = set()
            for r in mask.split(":", 1)[1].split(","):
                lo, _, hi = r.partition("-")
                b_cus.update(range(int(lo), int(hi or lo) + 1))
            assert len(b_cus) == 128
            for n in running_a:                              # B's CUs are disjoint from A's survivors
                m = kubelet.envs[("team-a", n)]["HSA_CU_MASK"]
                a_cus = set()
                for r in m.split(":", 1)[1].split(","):
                    lo, _, hi = r.partition("-")
                    a_cus.update(range(int(lo), int(hi or lo) + 1))
                assert not (a_cus & b_cus), (n, m, mask)
            path = os.path.join(d, NODE, "fake-amdsmi.json")
            if os.path.exists(path):                         # written on every amd-smi mode change
                with open(path) as f:
                    assert [g["compute"].upper() for g in json.load(f)] == ["SPX"]
            assert kubelet.admission_failures == []
        finally:
            c.stop()


def test_slice_agent_process_serves_cu_mask_slices():
    """A cumask node: the partitioner plans CU-mask slices for pending slice pods, the slice agent
    process materialises them in its slice store and its device plugin serves them; kubelet's
    Allocate hands each pod the HSA_CU_MASK of disjoint CU rows and its HBM budget."""
    from walkai_nos_amd.api import v1alpha1 as api
    with tempfile.TemporaryDirectory() as d:
        c = DevCluster(d, nodes=1, gpus=1, kind=api.PARTITIONING_KIND_CUMASK)
        try:
            c.start()
            k = c.kubelets[NODE]
            c.submit("s0", "gpu-64cu.72gb")
            c.submit("s1", "gpu-64cu.72gb")
            c.submit("m0", "gpu-36gb")
            c.run_until(lambda: all(c.phase(n) == "Running" for n in ("s0", "s1", "m0")), 90,
                        "the three slice pods to run")
            masks = [k.envs[("default", n)].get("HSA_CU_MASK", "") for n in ("s0", "s1")]
            assert all(m.startswith("0:") for m in masks) and masks[0] != masks[1], masks

            def cus(m):
                out = set()
                for part in m.split(":", 1)[1].split(","):
                    lo, _, hi = part.partition("-")
                    out |= set(range(int(lo), int(hi or lo) + 1))
                return out
            a, b = cus(masks[0]), cus(masks[1])
            assert len(a) == len(b) == 64 and not (a & b)
            limits = [int(k.envs[("default", n)]["NOS_HBM_LIMIT_BYTES"]) for n in ("s0", "s1", "m0")]
            assert limits[0] == limits[1] == 72 * 10**9 and limits[2] == 36 * 10**9
        finally:
            c.stop()


def test_cluster_info_exporter_process_posts_the_cluster():
    """nos-clusterinfoexporter as a process against the API: its first snapshot (sent at start)
    reaches the endpoint with the cluster's partition inventory and a bearer token."""
    import json as _json
    from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

    got = []

    class Sink(BaseHTTPRequestHandler):
        def do_POST(self):  # noqa: N802
            body = self.rfile.read(int(self.headers.get("Content-Length") or 0))
            got.append((self.headers.get("Authorization"), _json.loads(body)))
            self.send_response(200)
            self.end_headers()

        def log_message(self, *a):
            pass
    sink = ThreadingHTTPServer(("127.0.0.1", 0), Sink)
    threading.Thread(target=sink.serve_forever, daemon=True).start()
    with tempfile.TemporaryDirectory() as d:
        c = DevCluster(d, nodes=1, gpus=2)
        proc = None
        try:
            c.start()
            c.run_until(lambda: c.allocatable(NODE, "spx_nps1") == 2, 30, "the node to report")
            proc = subprocess.Popen([sys.executable, "-m", "walkai_nos_amd.cmd.clusterinfoexporter",
                                     "--endpoint", f"http://127.0.0.1:{sink.server_address[1]}/ingest",
                                     "--interval", "1h", "--api-token", "t0k", "--kubeconfig", c.kubeconfig],
                                    env=dict(os.environ, PYTHONPATH=REPO), stdout=subprocess.DEVNULL,
                                    stderr=subprocess.DEVNULL)
            deadline = time.time() + 30
            while not got and time.time() < deadline:
                time.sleep(0.1)
            assert got, "no snapshot posted"
            auth, payload = got[0]
            assert auth == "Bearer t0k"
            assert {"gpu": "spx_nps1", "allocated": 0, "available": 2} in payload["gpus"], payload
        finally:
            if proc is not None:
                proc.terminate()
                proc.wait(timeout=10)
            c.stop()
            sink.shutdown()


def test_memory_partition_switch_over_processes():
    """NPS2 pods on an NPS1 node: the partitioner writes a node-wide memory-partition spec, the
    agent process switches the (idle) node, its plugin serves amd.com/cpx_nps2 and the pods run."""
    with tempfile.TemporaryDirectory() as d:
        c = DevCluster(d, nodes=1, gpus=2)
        try:
            c.start()
            c.run_until(lambda: c.allocatable(NODE, "spx_nps1") == 2, 30, "the node to report")
            for i in range(5):
                c.submit(f"n{i}", "cpx_nps2")
            c.run_until(lambda: all(c.phase(f"n{i}") == "Running" for i in range(5)), 120, "the NPS2 pods")
            anns = ko.annotations(c.client.get("Node", NODE))
            assert anns["nos.nebuly.com/spec-memory-partition"] == "nps2"
            c.run_until(lambda: ko.annotations(c.client.get("Node", NODE)).get(
                "nos.nebuly.com/status-memory-partition") == "nps2", 30, "the NPS status")
            assert c.kubelets[NODE].admission_failures == []
        finally:
            c.stop()


def test_component_restarts_and_a_kubelet_restart():
    """Crash / upgrade scenarios over processes: the partition agent restarts (the GPUs keep their
    modes: the fake backend persists them as devices do) and resumes reporting and serving; the
    partitioner restarts and keeps planning from the node annotations; kubelet restarts (plugin
    sockets wiped, kubelet.sock recreated) and the agent's plugins re-register by themselves."""
    from walkai_nos_amd.deviceplugin.server import RegistrationServer
    with tempfile.TemporaryDirectory() as d:
        c = DevCluster(d, nodes=1, gpus=2)
        try:
            c.start()
            k = c.kubelets[NODE]
            c.run_until(lambda: c.allocatable(NODE, "spx_nps1") == 2, 30, "the node to report")
            for i in range(8):
                c.submit(f"c{i}", "cpx_nps1")
            c.run_until(lambda: all(c.phase(f"c{i}") == "Running" for i in range(8)), 60, "the 1/8 pods")
            settled = {"nos.nebuly.com/status-gpu-0-cpx_nps1-used": "8", "nos.nebuly.com/status-gpu-1-spx_nps1-free": "1"}

            def status():
                return {k_: v for k_, v in ko.annotations(c.client.get("Node", NODE)).items() if "status-gpu" in k_}
            c.run_until(lambda: status() == settled, 30, "the layout to be reported")
            c.restart("partitionagent-node-0")
            c.run_until(lambda: status() == settled and len(k.healthy("amd.com/spx_nps1")) == 1
                        and len(k.healthy("amd.com/cpx_nps1")) == 8, 30,
                        "the restarted agent to report and serve the same layout")
            c.submit("s0", "spx_nps1")
            c.run_until(lambda: c.phase("s0") == "Running", 30, "a whole-GPU pod after the agent restart")

            c.restart("gpupartitioner")
            for i in range(8):
                k.finish("default", f"c{i}")
            for i in range(2):
                c.submit(f"d{i}", "dpx_nps1")
            c.run_until(lambda: all(c.phase(f"d{i}") == "Running" for i in range(2)), 60,
                        "1/2 pods planned by the restarted partitioner")

            k.reg.stop()
            for f in os.listdir(k.dir):
                os.unlink(os.path.join(k.dir, f))
            k.reg = RegistrationServer(os.path.join(k.dir, "kubelet.sock")).start()
            k.readers.clear()
            c.run_until(lambda: {r.resource_name for r in k.reg.registered} >= {"amd.com/dpx_nps1", "amd.com/spx_nps1"},
                        30, "re-registration after the kubelet restart")
            k.finish("default", "d0")
            c.submit("d2", "dpx_nps1")
            c.run_until(lambda: c.phase("d2") == "Running", 30, "admission after the kubelet restart")
            assert k.admission_failures == []
        finally:
            c.stop()


def test_sliced_agent_restart_keeps_the_slices_over_processes():
    """A sliced GPU across a partition-agent restart: the slice layout lives in the agent's state
    file (``sliceStateFile``), so the restarted agent reports the same sliced GPU and serves the
    same slice ids — the running pods' devices stay healthy, no slice is re-carved under them — and
    a pod submitted afterwards is carved into the free groups next to them."""
    from walkai_nos_amd.api import v1alpha1 as api
    from walkai_nos_amd.cmd.devcluster import fast_partitioner_config
    with tempfile.TemporaryDirectory() as d:
        c = DevCluster(d, nodes=1, gpus=1, bookmark_every=2.0, layout="slices",
                       partitioner=fast_partitioner_config(sliceReserveAfterSeconds=1))
        try:
            c.start()
            k = c.kubelets[NODE]
            c.run_until(lambda: ko.annotations(c.client.get("Node", NODE)).get(api.ANNOTATION_SLICED_GPUS_STATUS) == "0",
                        30, "the GPU to be served sliced")
            c.submit("half", "dpx_nps1")
            c.submit("e0", "cpx_nps1")
            c.run_until(lambda: c.phase("half") == "Running" and c.phase("e0") == "Running", 60, "the first pods")
            ids = {n: k.used[("default", n)][1] for n in ("half", "e0")}
            c.restart("partitionagent-node-0")
            c.run_until(lambda: ko.annotations(c.client.get("Node", NODE)).get(api.ANNOTATION_SLICED_GPUS_STATUS) == "0"
                        and set(ids.values()) <= set(k.healthy("amd.com/dpx_nps1") + k.healthy("amd.com/cpx_nps1")),
                        30, "the restarted agent to serve the same slices")
            c.submit("quarter", "qpx_nps1")
            c.run_until(lambda: c.phase("quarter") == "Running", 60, "a 1/4 pod next to the running ones")
            assert all(c.phase(n) == "Running" for n in ("half", "e0"))
            assert {n: k.used[("default", n)][1] for n in ("half", "e0")} == ids
            assert k.admission_failures == []
        finally:
            c.stop()


def test_partitioner_leader_election_failover_over_rest():
    """Two partitioner replicas with leader election (a coordination.k8s.io Lease over the REST
    API): one holds the lease; the leader is killed; the standby takes the lease over once it
    expires and plans the next pods."""
    from walkai_nos_amd.cmd.devcluster import fast_partitioner_config
    cfg = fast_partitioner_config()
    le = cfg.leaderElection
    le.leaderElect, le.resourceName = True, "gpu-partitioner.nos.nebuly.com"
    le.leaseDurationSeconds, le.renewDeadlineSeconds, le.retryPeriodSeconds = 3.0, 2.0, 0.5
    with tempfile.TemporaryDirectory() as d:
        c = DevCluster(d, nodes=1, gpus=2, partitioner=cfg)
        try:
            c.start()
            c._spawn("gpupartitioner-2", "walkai_nos_amd.cmd.gpupartitioner", cfg, "GpuPartitionerConfig", {})
            c.run_until(lambda: c.allocatable(NODE, "spx_nps1") == 2, 30, "the node to report")

            def holder():
                leases = c.client.list("Lease")
                return leases[0]["spec"].get("holderIdentity") if leases else None
            c.run_until(lambda: holder() is not None, 20, "a leader")
            first = holder()
            leader = next(n for n in ("gpupartitioner", "gpupartitioner-2") if first in open(c.logs[n]).read())
            for i in range(8):
                c.submit(f"c{i}", "cpx_nps1")
            c.run_until(lambda: all(c.phase(f"c{i}") == "Running" for i in range(8)), 60, "pods planned by the leader")
            c.procs[leader].kill()
            c.procs[leader].wait()
            del c.procs[leader]
            c.run_until(lambda: holder() not in (None, first), 30, "the standby to take the lease")
            for i in range(2):
                c.submit(f"d{i}", "dpx_nps1")
            c.run_until(lambda: all(c.phase(f"d{i}") == "Running" for i in range(2)), 60, "pods planned by the new leader")
        finally:
            c.stop()


def test_churn_soak_over_processes():
    """Random fractional pods (1/8, 1/2, whole GPU; 2-6 s lifetimes) arriving for 25 s on two
    2-GPU nodes, run by the binaries: flips and drains happen under kube-scheduler semantics and
    no pod is ever admitted to a partition its plugin withholds (zero admission failures); once
    arrivals stop, every waiting pod runs."""
    import random
    rng = random.Random(7)
    mix = [("cpx_nps1", 0.5), ("dpx_nps1", 0.3), ("spx_nps1", 0.2)]
    with tempfile.TemporaryDirectory() as d:
        c = DevCluster(d, nodes=2, gpus=2)
        try:
            c.start()
            c.run_until(lambda: all(c.allocatable(n, "spx_nps1") == 2 for n in c.kubelets), 30, "the nodes to report")
            seq, t_end = 0, time.time() + 25
            while time.time() < t_end:
                if rng.random() < 0.35:
                    r, acc, prof = rng.random(), 0.0, mix[-1][0]
                    for p, w in mix:
                        acc += w
                        if r < acc:
                            prof = p
                            break
                    c.submit(f"p{seq}", prof, runtime_s=rng.uniform(2, 6))
                    seq += 1
                c.step()
                time.sleep(0.2)
            c.run_until(lambda: all(ko.pod_phase(p) != "Pending" for p in c.client.list("Pod")), 150,
                        "every waiting pod to run")
            assert seq > 20
            fails = [f for k in c.kubelets.values() for f in k.admission_failures]
            assert fails == [], fails
        finally:
            c.stop()
