"""Cluster-info collector/exporter (pkg/clusterinfo/collector_test.go behaviour), telemetry exporter
(cmd/metricsexporter/metrics/metrics_test.go behaviour) and the nos device plugin over gRPC."""
import json
import os
import tempfile

import grpc
import pytest

from walkai_nos_amd.device.protos import dp
from walkai_nos_amd.device.slicing_client import MemorySliceStore
from walkai_nos_amd.deviceplugin.server import PluginManager, RegistrationServer, SliceDevicePlugin
from walkai_nos_amd.exporters.clusterinfo import Collector, Exporter, format_profiles, pod_status
from walkai_nos_amd.exporters.telemetry import Metrics, filter_labels, run
from walkai_nos_amd.kube import objects as ko
from walkai_nos_amd.kube.memory import InMemoryAPIServer
from walkai_nos_amd.models.slicing.cumask import Slice


def test_collector_inventory_from_annotations_and_pod_summaries():
    a = InMemoryAPIServer(clock=lambda: 1700000000.0)
    a.create(ko.new_node("n1", annotations_={"nos.nebuly.com/status-gpu-0-cpx_nps1-used": "3",
                                            "nos.nebuly.com/status-gpu-0-cpx_nps1-free": "5",
                                            "nos.nebuly.com/status-gpu-1-spx_nps1-free": "1"}))
    p = ko.new_pod("b", "ns2", requests={"amd.com/cpx_nps1": 2}, phase="Running")
    p["status"]["containerStatuses"] = [{"state": {"waiting": {"reason": "ContainerCreating"}}}]
    a.create(p)
    a.create(ko.new_pod("a", "ns1", requests={"amd.com/spx_nps1": 1, "amd.com/cpx_nps1": 1}, phase="Pending"))
    a.create(ko.new_pod("cpu", "ns1", requests={"cpu": "1"}))
    snap = Collector(a, clock=lambda: 1700000000.0).collect()
    assert [(g.gpu, g.allocated, g.available) for g in snap.gpus] == [("cpx_nps1", 3, 5), ("spx_nps1", 0, 1)]
    assert [(s.namespace, s.name, s.status, s.gpu) for s in snap.pods] == [
        ("ns1", "a", "Pending", "cpx_nps1, spx_nps1"), ("ns2", "b", "ContainerCreating", "cpx_nps1 x2")]
    assert snap.ts == "2023-11-14T22:13:20Z"
    assert snap.utilization["gpu_allocated_percent"] == round(100 * (3 / 8) / 2, 3)
    doc = json.loads(snap.to_json())
    assert set(doc) >= {"ts", "gpus", "pods"} and set(doc["pods"][0]) == {"name", "namespace", "status", "gpu",
                                                                         "start_time", "finish_time"}


def test_collector_capacity_fallback_caps_at_capacity():
    a = InMemoryAPIServer()
    a.create(ko.new_node("n1", allocatable={"amd.com/cpx_nps1": "8"}))
    for i in range(10):
        a.create(ko.new_pod(f"p{i}", requests={"amd.com/cpx_nps1": 1}))
    snap = Collector(a).collect()
    assert [(g.gpu, g.allocated, g.available) for g in snap.gpus] == [("cpx_nps1", 8, 0)]


def test_pod_status_and_finish_time():
    p = ko.new_pod("x", phase="Succeeded")
    p["status"]["containerStatuses"] = [
        {"state": {"terminated": {"reason": "Completed", "finishedAt": "2024-01-01T00:00:05Z"}}},
        {"state": {"terminated": {"reason": "Completed", "finishedAt": "2024-01-01T00:00:09Z"}}}]
    p["spec"]["containers"][0]["resources"] = {"requests": {"amd.com/gpu-32cu.36gb": "1"}}
    a = InMemoryAPIServer()
    a.create(p)
    s = Collector(a).collect().pods[0]
    assert s.status == "Completed" and s.finish_time == "2024-01-01T00:00:09Z"
    assert format_profiles({"b": 1, "a": 3}) == "a x3, b"
    assert pod_status({"status": {}}) == "Unknown"


def test_exporter_posts_with_bearer_and_fails_on_error_status():
    a = InMemoryAPIServer()
    sent = []

    def post(url, body, headers, timeout):
        sent.append((url, json.loads(body), headers))
        return 204 if len(sent) == 1 else 500

    ex = Exporter(Collector(a), "https://api.example/clusters", api_token="tok", post=post)
    assert ex.send_snapshot() == 204
    assert sent[0][2]["Authorization"] == "Bearer tok"
    try:
        ex.send_snapshot()
        raise AssertionError("expected failure")
    except RuntimeError:
        pass


def test_telemetry_never_fails_and_filters_labels():
    assert run("/nonexistent/metrics.yaml", "http://x") == 0
    with tempfile.NamedTemporaryFile("w", suffix=".yaml", delete=False) as f:
        f.write("installationUUID: abc\nnodes:\n- name: n1\n  labels: {amd.com/gpu.product-name: MI355X}\n"
                "components: {nosGpuPartitioner: true}\nchartValues: {x: 1}\n")
    got = []
    assert run(f.name, "http://x", post=lambda url, body: got.append(json.loads(body)) or 500) == 0
    os.unlink(f.name)
    assert got[0]["installationUUID"] == "abc" and got[0]["components"]["nosGpuPartitioner"] is True
    assert Metrics.from_yaml("{}").installationUUID == ""
    assert filter_labels({"amd.com/x": "1", "foo": "2", "node.kubernetes.io/instance-type": "t"}) == {
        "amd.com/x": "1", "node.kubernetes.io/instance-type": "t"}


def test_device_plugin_list_and_watch_allocate_and_register():
    store = MemorySliceStore()
    store.save({0: [Slice("g0::s0", "32cu.36gb", [0, 1, 2, 3], 36 * 10**9),
                    Slice("g0::s1", "32cu.36gb", [4, 5, 6, 7], 36 * 10**9),
                    Slice("g0::s2", "10gb", [], 10 * 10**9)]})
    with tempfile.TemporaryDirectory() as d:
        reg = RegistrationServer(os.path.join(d, "kubelet.sock")).start()
        mgr = PluginManager(store, {0: "/dev/dri/renderD128"}, socket_dir=d, kubelet_socket=reg.socket)
        try:
            mgr.sync()
            assert sorted(r.resource_name for r in reg.registered) == ["amd.com/gpu-10gb", "amd.com/gpu-32cu.36gb"]
            plug = mgr.plugins["amd.com/gpu-32cu.36gb"]
            with grpc.insecure_channel("unix://" + plug.socket) as ch:
                law = ch.unary_stream(f"/{dp.SERVICE}/ListAndWatch", request_serializer=dp.Empty.SerializeToString,
                                      response_deserializer=dp.ListAndWatchResponse.FromString)
                stream = law(dp.Empty(), timeout=5)
                first = next(stream)
                assert [x.ID for x in first.devices] == ["g0::s0", "g0::s1"]
                stream.cancel()
                alloc = ch.unary_unary(f"/{dp.SERVICE}/Allocate", request_serializer=dp.AllocateRequest.SerializeToString,
                                       response_deserializer=dp.AllocateResponse.FromString)
                req = dp.AllocateRequest()
                req.container_requests.add(devicesIDs=["g0::s1"])
                resp = alloc(req, timeout=5)
                envs = dict(resp.container_responses[0].envs)
                assert envs["HSA_CU_MASK"] == "0:32-63"
                assert envs["NOS_HBM_LIMIT_BYTES"] == str(36 * 10**9)
                assert envs["LD_PRELOAD"].endswith("libnos_hbmlimit.so")
                assert "GPU_MAX_HW_QUEUES" not in envs  # dedicated CUs: HIP's default queues
                assert [x.host_path for x in resp.container_responses[0].devices] == ["/dev/kfd", "/dev/dri/renderD128"]
            shared = SliceDevicePlugin("amd.com/gpu-10gb", store, {}, socket_dir=d)
            req = dp.AllocateRequest()
            req.container_requests.add(devicesIDs=["g0::s2"])
            envs = dict(shared.Allocate(req, None).container_responses[0].envs)
            assert envs["HSA_CU_MASK"] == "0:64-255"  # shared pool = rows no dedicated slice owns
            # memory-only: the queue count decides the per-pipe split (sharedSliceHwQueues auto:
            # two queues while <= 3 memory-only slices share the GPU, one beyond)
            assert envs["GPU_MAX_HW_QUEUES"] == "2"
            envs = dict(SliceDevicePlugin("amd.com/gpu-10gb", store, {}, socket_dir=d, shared_hw_queues=0)
                        .Allocate(req, None).container_responses[0].envs)
            assert "GPU_MAX_HW_QUEUES" not in envs
            envs = dict(SliceDevicePlugin("amd.com/gpu-10gb", store, {}, socket_dir=d, shared_hw_queues=3)
                        .Allocate(req, None).container_responses[0].envs)
            assert envs["GPU_MAX_HW_QUEUES"] == "3"
            many = MemorySliceStore()
            many.save({0: [Slice(f"g0::m{i}", "10gb", [], 10 * 10**9) for i in range(5)]})
            req5 = dp.AllocateRequest()
            req5.container_requests.add(devicesIDs=["g0::m4"])
            envs = dict(SliceDevicePlugin("amd.com/gpu-10gb", many, {}, socket_dir=d)
                        .Allocate(req5, None).container_responses[0].envs)
            assert envs["GPU_MAX_HW_QUEUES"] == "1"
        finally:
            mgr.stop()
            reg.stop()


def test_amdsmi_metrics_poller_publishes_activity_vram_and_mode():
    from walkai_nos_amd.device.amdsmi import FakeAmdSmi
    from walkai_nos_amd.exporters.gpu_metrics import GpuMetricsPoller
    from walkai_nos_amd.utils.metrics import REGISTRY
    smi = FakeAmdSmi(n_gpus=2)
    smi.set_processes(1, 3)
    p = GpuMetricsPoller(smi, "node-m")
    p.poll()
    text = REGISTRY.render().decode()
    assert 'nos_amdsmi_gfx_activity_percent{gpu="1",node="node-m"} 100.0' in text
    assert 'nos_amdsmi_partition_info{compute="SPX",gpu="0",memory="NPS1",node="node-m"} 1.0' in text
    smi.set_processes(0, 0)
    smi.set_compute_partition(0, "CPX")
    p.poll()
    text = REGISTRY.render().decode()
    assert 'nos_amdsmi_partition_info{compute="CPX",gpu="0",memory="NPS1",node="node-m"} 8.0' in text
    assert 'compute="SPX",gpu="0",memory="NPS1",node="node-m"' not in text  # stale mode series removed


def test_device_plugin_keeps_a_two_slice_request_on_one_gpu():
    from walkai_nos_amd.deviceplugin.server import preferred_same_gpu
    store = MemorySliceStore()
    store.save({0: [Slice("g0::s0", "32cu.36gb", [0, 1, 2, 3], 36 * 10**9),
                    Slice("g0::s1", "32cu.36gb", [4, 5, 6, 7], 36 * 10**9)],
                1: [Slice("g1::s0", "32cu.36gb", [0, 1, 2, 3], 36 * 10**9),
                    Slice("g1::s1", "32cu.36gb", [4, 5, 6, 7], 36 * 10**9),
                    Slice("g1::s2", "32cu.36gb", [8, 9, 10, 11], 36 * 10**9)]})
    plug = SliceDevicePlugin("amd.com/gpu-32cu.36gb", store, {0: "/dev/dri/renderD128", 1: "/dev/dri/renderD136"},
                             socket_dir=tempfile.gettempdir())
    req = dp.PreferredAllocationRequest()
    # g0::s0 is in use (not available): GPU 0 is the more-used GPU but has only one free slice left,
    # so a 2-slice request goes to GPU 1, never across GPUs
    req.container_requests.add(available_deviceIDs=["g0::s1", "g1::s0", "g1::s1", "g1::s2"], allocation_size=2)
    req.container_requests.add(available_deviceIDs=["g0::s1", "g1::s0", "g1::s1", "g1::s2"], allocation_size=1)
    resp = plug.GetPreferredAllocation(req, None)
    assert list(resp.container_responses[0].deviceIDs) == ["g1::s0", "g1::s1"]
    assert list(resp.container_responses[1].deviceIDs) == ["g0::s1"]  # packs onto the busier GPU
    gpu_of = {"a0": 0, "a1": 0, "b0": 1}
    assert preferred_same_gpu(["b0"], ["a0", "a1", "b0"], 2, gpu_of, {0: 2, 1: 1}) == ["b0", "a0"]  # fallback
    a = dp.AllocateRequest()
    a.container_requests.add(devicesIDs=["g0::s1", "g1::s0"])
    with pytest.raises(ValueError):
        plug.Allocate(a, None)
    a = dp.AllocateRequest()
    a.container_requests.add(devicesIDs=["g1::s0", "g1::s1"])
    r = plug.Allocate(a, None).container_responses[0]
    assert dict(r.envs)["HSA_CU_MASK"] == "0:0-63"
    assert [x.host_path for x in r.devices] == ["/dev/kfd", "/dev/dri/renderD136"]


def test_degraded_probe_withholds_the_partition_and_is_exported():
    """a partition whose probe falls below its model's expected rate is advertised
    Unhealthy with the reason, exported in the cluster-info snapshot, and the planner places new
    work on the other GPU; a target in use is never probed."""
    import json

    from walkai_nos_amd.api import v1alpha1 as api
    from walkai_nos_amd.controllers.agent.probe import ProbeRunner, device_map_targets
    from walkai_nos_amd.controllers.agent.shared import SharedState
    from walkai_nos_amd.controllers.partitioner.pod_controller import plan_cluster_pack
    from walkai_nos_amd.deviceplugin.partitions import PartitionState
    from walkai_nos_amd.device.amdsmi import FakeAmdSmi
    from walkai_nos_amd.exporters.clusterinfo import Collector
    from walkai_nos_amd.kube.memory import InMemoryAPIServer
    from walkai_nos_amd.models.xcp import node as xcp_node

    smi = FakeAmdSmi(n_gpus=2)
    smi.set_compute_partition(1, "CPX")
    m = smi.device_map()
    in_use = {m.partitions_of(1)[0].device_id}
    probed = []

    def probe(dev, cus, label):        # partition 3 of GPU 1 runs at 40% of the expected rate
        probed.append(label)
        n = 256 if label.startswith("gpu0") else 32
        return {"n_cus": n, "bf16_tflops": (0.4 if label == "gpu1.p3" else 1.0) * 6.16 * n}
    shared = SharedState()
    r = ProbeRunner(shared, "n0", probe_fn=probe, targets=device_map_targets(smi), asynchronous=False,
                    used=lambda: in_use, expected_per_cu=6.16, healthy_fraction=0.7)
    shared.record_commit(True)
    r.poll()
    assert "gpu1.p0" not in probed and len(probed) == 8                 # never under a pod
    assert set(r.degraded()) == {"gpu1.p3"} and "below 70%" in r.degraded()["gpu1.p3"]
    st = PartitionState(smi.device_map, lambda: {}, lambda: in_use, degraded=r.degraded)
    v = st.view()
    cpx = {d.partition_index: d for d in v["amd.com/cpx_nps1"]}
    assert not cpx[3].healthy and "probe" in cpx[3].reason and all(cpx[k].healthy for k in (0, 1, 2, 4))
    # exported: the status-probe annotation feeds the snapshot and the node model
    api_ = InMemoryAPIServer()
    node = ko.new_node("n0", {api.LABEL_GPU_PARTITIONING: "xcp", "amd.com/gpu.product-name": "AMD_Instinct_MI355X",
                              "amd.com/gpu.count": "2"})
    node["metadata"]["annotations"] = {api.ANNOTATION_PROBE_RESULT: json.dumps(r.results),
                                       "nos.nebuly.com/status-gpu-0-spx_nps1-free": "1",
                                       "nos.nebuly.com/status-gpu-1-cpx_nps1-used": "1",
                                       "nos.nebuly.com/status-gpu-1-cpx_nps1-free": "7"}
    api_.create(node)
    snap = Collector(api_).collect()
    bad = [p for p in snap.probes if p.degraded]
    assert [p.target for p in bad] == ["gpu1.p3"] and bad[0].gpu == 1
    assert snap.utilization["degraded_targets"] == 1.0 and snap.utilization["probed_bf16_tflops"] > 1500
    model = xcp_node.new_node(node)
    assert model.gpus[1].degraded and not model.gpus[0].degraded
    # planner: two idle GPUs, one degraded -> the healthy one is flipped for the waiting pods
    for g in model.gpus:
        g.used, g.free = {}, {"spx_nps1": 1}
    changed = plan_cluster_pack({"n0": model}, [({"cpx_nps1": 1}, 700.0)] * 6)
    flipped = [g.index for g in changed["n0"].gpus if g.geometry() != {"spx_nps1": 1}]
    assert flipped == [0]
