"""The drain, enforced outside the simulator.

The pack policy drains a busy GPU by writing its new spec while partitions are in use; the nos
partition device plugin (``deviceplugin/partitions.py``) reports every partition of a GPU being
re-partitioned Unhealthy, so kubelet's allocatable drops and neither kube-scheduler (allocatable
minus requests, no GPU knowledge) nor kubelet admission can put a new pod there.  These tests run
the real partitioner, partition agent and plugin, with a scheduler of kube-scheduler semantics.
"""
import os
import tempfile

import grpc

from walkai_nos_amd.device.amdsmi import FakeAmdSmi
from walkai_nos_amd.device.protos import dp
from walkai_nos_amd.deviceplugin.partitions import (PartitionState, draining_gpus, partition_plugin_manager,
                                                    partition_view, reconfiguring_gpus)
from walkai_nos_amd.deviceplugin.server import RegistrationServer
from walkai_nos_amd.kube import objects as ko
from walkai_nos_amd.sim.cluster import KubeScheduler, SimCluster


def test_reconfiguring_and_draining_gpus_from_annotations():
    anns = {"nos.nebuly.com/spec-gpu-0-spx_nps1": "1", "nos.nebuly.com/status-gpu-0-cpx_nps1-used": "3",
            "nos.nebuly.com/status-gpu-0-cpx_nps1-free": "5",
            "nos.nebuly.com/spec-gpu-1-dpx_nps1": "2", "nos.nebuly.com/status-gpu-1-dpx_nps1-free": "2",
            "nos.nebuly.com/spec-gpu-2-cpx_nps1": "8", "nos.nebuly.com/status-gpu-2-spx_nps1-free": "1"}
    assert reconfiguring_gpus(anns) == {0, 2}      # GPU 1's spec matches its status
    assert draining_gpus(anns) == {0}              # GPU 2 is idle: it flips, it does not drain
    smi = FakeAmdSmi(n_gpus=3)
    smi.set_compute_partition(0, "CPX")
    v = partition_view(smi.device_map(), reconfiguring_gpus(anns), used_ids=set())
    assert [d.healthy for d in v["amd.com/cpx_nps1"]] == [False] * 8    # used ones too: no race to lose
    assert [d.healthy for d in v["amd.com/spx_nps1"]] == [True, False]  # GPU 1 healthy, GPU 2 about to flip


def _node_cpx_alloc(c, node="node-0"):
    return int(ko.node_allocatable(c.api.get("Node", node)).get("amd.com/cpx_nps1", "0"))


def test_single_gpu_drains_and_flips_while_new_pods_keep_arriving():
    """A 1-GPU node full of 1/8 pods, a whole-GPU pod waiting and 1/8 pods arriving every minute:
    the partitioner drains the GPU; while it drains kubelet reports no allocatable partition and no
    pod is bound to the node — the finishing pods' partitions are not refilled although 1/8 pods are
    queued — then the agent flips it and the whole-GPU pod runs."""
    c = SimCluster(n_nodes=1, gpus_per_node=1, policy="pack", refresh_interval=5.0)
    assert isinstance(c.scheduler, KubeScheduler)
    c.run(30)
    for i in range(8):
        c.submit({"amd.com/cpx_nps1": 1}, name=f"c{i}")
    c.run(120)
    assert len(c.running_pods()) == 8
    c.submit({"amd.com/spx_nps1": 1}, name="big")
    running = {ko.name(p) for p in c.running_pods()}
    seq, drained_at, binds_while_draining = 8, None, []
    for minute in range(60):
        c.submit({"amd.com/cpx_nps1": 1}, name=f"c{seq}")   # the 1/8 queue never empties
        seq += 1
        if minute % 2 == 1 and running:                     # and a running 1/8 pod finishes now and then
            done = sorted(running)[0]
            running.discard(done)
            c.complete(done)
            c.delete_pod(done)
        nbinds = len(c.binds)
        c.run(60)
        anns = ko.annotations(c.api.get("Node", "node-0"))
        if 0 in draining_gpus(anns):
            drained_at = drained_at if drained_at is not None else minute
            assert _node_cpx_alloc(c) == 0, "a draining GPU must not offer allocatable partitions"
            binds_while_draining += [b for b in c.binds[nbinds:] if b[1] != "big"]
        if ko.pod_phase(c.api.get("Pod", "big", "default")) == "Running":
            break
        running |= {ko.name(p) for p in c.running_pods() if ko.name(p) != "big"}
    assert drained_at is not None, "the GPU was never drained"
    assert binds_while_draining == []
    assert ko.pod_phase(c.api.get("Pod", "big", "default")) == "Running"
    sn = c.nodes["node-0"]
    assert sn.smi.get_compute_partition(0) == "SPX"
    assert c.admission_failures == 0
    assert [k for k, *_ in sn.smi.set_calls] == ["compute", "compute"]  # SPX->CPX, then CPX->SPX once drained


def test_without_the_nos_plugin_the_drain_never_ends():
    """The same load with the AMD device plugin (every partition healthy): kube-scheduler keeps
    refilling the draining GPU's partitions from the 1/8 queue, so the whole-GPU pod never runs."""
    c = SimCluster(n_nodes=1, gpus_per_node=1, policy="pack", refresh_interval=5.0, device_plugin="amd")
    c.run(30)
    for i in range(8):
        c.submit({"amd.com/cpx_nps1": 1}, name=f"c{i}")
    c.run(120)
    c.submit({"amd.com/spx_nps1": 1}, name="big")
    seq = 8
    for minute in range(40):
        c.submit({"amd.com/cpx_nps1": 1}, name=f"c{seq}")
        seq += 1
        if minute % 2 == 1:
            done = sorted(ko.name(p) for p in c.running_pods() if ko.name(p) != "big")[0]
            c.complete(done)
            c.delete_pod(done)
        c.run(60)
    assert ko.pod_phase(c.api.get("Pod", "big", "default")) == "Pending"


class _Law:
    """A kubelet-side ListAndWatch client: the latest device list of a plugin."""

    def __init__(self, socket):
        self.ch = grpc.insecure_channel("unix://" + socket)
        law = self.ch.unary_stream(f"/{dp.SERVICE}/ListAndWatch", request_serializer=dp.Empty.SerializeToString,
                                   response_deserializer=dp.ListAndWatchResponse.FromString)
        self.stream = law(dp.Empty(), timeout=10)

    def next(self):
        r = next(self.stream)
        return [(d.ID, d.health) for d in r.devices]

    def close(self):
        self.stream.cancel()
        self.ch.close()


def test_grpc_partition_plugin_pushes_health_and_survives_a_kubelet_restart():
    smi = FakeAmdSmi(n_gpus=2)
    anns = {}
    used = set()
    state = PartitionState(smi.device_map, lambda: anns, lambda: used)
    with tempfile.TemporaryDirectory() as d:
        reg = RegistrationServer(os.path.join(d, "kubelet.sock")).start()
        mgr = partition_plugin_manager(state, socket_dir=d, kubelet_socket=reg.socket, register_backoff=0.01)
        try:
            mgr.sync()
            assert [r.resource_name for r in reg.registered] == ["amd.com/spx_nps1"]
            spx = mgr.plugins["amd.com/spx_nps1"]
            law = _Law(spx.socket)
            assert [h for _, h in law.next()] == [dp.HEALTHY, dp.HEALTHY]
            # the partitioner drains GPU 1 (spec CPX while its SPX partition is in use)
            ids = [i for i, _ in spx.device_states()]
            used.add(ids[1])
            anns.update({"nos.nebuly.com/spec-gpu-1-cpx_nps1": "8", "nos.nebuly.com/status-gpu-1-spx_nps1-used": "1",
                         "nos.nebuly.com/spec-gpu-0-spx_nps1": "1", "nos.nebuly.com/status-gpu-0-spx_nps1-free": "1"})
            mgr.sync()
            assert law.next() == [(ids[0], dp.HEALTHY), (ids[1], dp.UNHEALTHY)]
            # kubelet asks for the preferred allocation among what is healthy; Allocate refuses the
            # withheld partition and hands out the render node of the partition it serves
            a = dp.AllocateRequest()
            a.container_requests.add(devicesIDs=[ids[1]])
            try:
                spx.Allocate(a, None)
                raise AssertionError("a partition of a re-partitioning GPU was allocated")
            except KeyError:
                pass
            a = dp.AllocateRequest()
            a.container_requests.add(devicesIDs=[ids[0]])
            r = spx.Allocate(a, None).container_responses[0]
            dm = smi.device_map()
            assert [x.host_path for x in r.devices] == ["/dev/kfd", f"/dev/dri/renderD{dm.devices[0].render_minor}"]
            # the pod leaves, the agent flips GPU 1 and reports: a new resource registers, healthy
            used.clear()
            smi.set_compute_partition(1, "CPX")
            anns["nos.nebuly.com/status-gpu-1-cpx_nps1-free"] = "8"
            del anns["nos.nebuly.com/status-gpu-1-spx_nps1-used"]
            mgr.sync()
            assert law.next() == [(ids[0], dp.HEALTHY)]
            assert "amd.com/cpx_nps1" in {r.resource_name for r in reg.registered}
            assert all(ok for _, ok in mgr.plugins["amd.com/cpx_nps1"].device_states())
            law.close()
            # kubelet restarts: it removes every plugin socket and recreates kubelet.sock
            reg.stop()
            for f in os.listdir(d):
                os.unlink(os.path.join(d, f))
            reg2 = RegistrationServer(os.path.join(d, "kubelet.sock")).start()
            mgr.sync()
            assert sorted(r.resource_name for r in reg2.registered) == ["amd.com/cpx_nps1", "amd.com/spx_nps1"]
            assert all(p.serving() for p in mgr.plugins.values())
            law = _Law(mgr.plugins["amd.com/cpx_nps1"].socket)
            assert len(law.next()) == 8
            law.close()
            reg2.stop()
        finally:
            mgr.stop()


def test_partition_plugin_reports_a_vanished_gpu_unhealthy():
    smi = FakeAmdSmi(n_gpus=2)
    state = PartitionState(smi.device_map, lambda: {}, lambda: set())
    v = state.view()
    assert [d.healthy for d in v["amd.com/spx_nps1"]] == [True, True]
    gone = smi._gpus.pop(1)                      # the card fell off the bus
    smi.enumerate(reinit=True)                   # the agent's periodic re-enumeration
    v = state.view()
    assert [(d.id, d.healthy) for d in v["amd.com/spx_nps1"]] == [(smi._gpus[0].uuid, True), (gone.uuid, False)]
    smi._gpus.append(gone)                       # and came back
    smi.enumerate(reinit=True)
    assert [d.healthy for d in state.view()["amd.com/spx_nps1"]] == [True, True]


def test_partition_plugin_survives_a_device_map_error():
    """an amd-smi failure while building the view must not end ListAndWatch (kubelet
    would drop the resource until the plugin registers again): the last known devices are listed
    Unhealthy until the map reads again, and a pushed update carries it."""
    smi = FakeAmdSmi(n_gpus=2)
    broken = {"on": False}

    def dmap():
        if broken["on"]:
            raise RuntimeError("amdsmi_init failed")
        return smi.device_map()
    state = PartitionState(dmap, lambda: {}, lambda: set())
    assert [d.healthy for d in state.view()["amd.com/spx_nps1"]] == [True, True]
    broken["on"] = True
    v = state.view()
    assert [d.healthy for d in v["amd.com/spx_nps1"]] == [False, False]
    assert "device map unavailable" in v["amd.com/spx_nps1"][0].reason
    with tempfile.TemporaryDirectory() as d:
        reg = RegistrationServer(os.path.join(d, "kubelet.sock")).start()
        mgr = partition_plugin_manager(state, socket_dir=d, kubelet_socket=reg.socket, register_backoff=0.01)
        try:
            mgr.sync()
            law = _Law(mgr.plugins["amd.com/spx_nps1"].socket)
            assert [h for _, h in law.next()] == [dp.UNHEALTHY, dp.UNHEALTHY]
            broken["on"] = False
            mgr.sync()                      # the same stream carries the recovery
            assert [h for _, h in law.next()] == [dp.HEALTHY, dp.HEALTHY]
            law.close()
        finally:
            mgr.stop()
            reg.stop()


def test_registration_retries_with_backoff_then_succeeds():
    from walkai_nos_amd.deviceplugin.server import SliceDevicePlugin
    from walkai_nos_amd.device.slicing_client import MemorySliceStore
    with tempfile.TemporaryDirectory() as d:
        sock = os.path.join(d, "kubelet.sock")
        plug = SliceDevicePlugin("amd.com/gpu-8gb", MemorySliceStore(), {}, socket_dir=d)
        waits, reg = [], []

        def sleep(s):  # kubelet comes up during the back-off
            waits.append(s)
            if len(waits) == 2:
                reg.append(RegistrationServer(sock).start())
        plug.register(sock, timeout=0.5, attempts=5, backoff=0.1, sleep=sleep)
        assert waits == [0.1, 0.2] and plug.registrations == 1
        assert reg[0].registered[0].resource_name == "amd.com/gpu-8gb"
        reg[0].stop()
        try:
            plug.register(os.path.join(d, "nope.sock"), timeout=0.2, attempts=2, backoff=0.01, sleep=lambda s: None)
            raise AssertionError("registration without kubelet must fail")
        except RuntimeError:
            pass


def test_partition_agent_wiring_publishes_allocatable_on_a_drain():
    """``cmd/partitionagent.nos_partition_plugin``: the hook the actuator calls after a flip (and the
    controller runs on every annotation change) syncs the plugins and patches the node's
    allocatable with the healthy counts, resources no longer served going to 0."""
    from walkai_nos_amd.api.config import MigAgentConfig
    from walkai_nos_amd.cmd.partitionagent import nos_partition_plugin
    from walkai_nos_amd.device.podresources import StaticResourceClient
    from walkai_nos_amd.kube.memory import InMemoryAPIServer
    smi = FakeAmdSmi(n_gpus=2)
    api_ = InMemoryAPIServer()
    api_.create(ko.new_node("n0", allocatable={"cpu": "8", "amd.com/spx_nps1": "2"}))
    with tempfile.TemporaryDirectory() as d:
        reg = RegistrationServer(os.path.join(d, "kubelet.sock")).start()
        cfg = MigAgentConfig(devicePluginDir=d)
        hook, plugins = nos_partition_plugin(api_, "n0", smi, StaticResourceClient(lambda: [], lambda: []), cfg)
        try:
            hook.restart()
            assert ko.node_allocatable(api_.get("Node", "n0"))["amd.com/spx_nps1"] == "2"
            api_.patch("Node", "n0", {"metadata": {"annotations": {
                "nos.nebuly.com/spec-gpu-1-cpx_nps1": "8", "nos.nebuly.com/status-gpu-1-spx_nps1-used": "1"}}})
            hook.reconcile(None)
            assert ko.node_allocatable(api_.get("Node", "n0"))["amd.com/spx_nps1"] == "1"
            smi.set_compute_partition(1, "CPX")
            api_.patch("Node", "n0", {"metadata": {"annotations": {
                "nos.nebuly.com/status-gpu-1-spx_nps1-used": None, "nos.nebuly.com/status-gpu-1-cpx_nps1-free": "8"}}})
            hook.reconcile(None)
            alloc = ko.node_allocatable(api_.get("Node", "n0"))
            # the new CPX partitions are registered with kubelet, but their allocatable is kubelet's
            # to publish once it holds the devices: published first, a bound pod could fail admission
            assert alloc["amd.com/spx_nps1"] == "1" and "amd.com/cpx_nps1" not in alloc and alloc["cpu"] == "8"
            assert {r.resource_name for r in reg.registered} == {"amd.com/spx_nps1", "amd.com/cpx_nps1"}
        finally:
            plugins.stop()
            reg.stop()


def test_slice_plugin_render_nodes_health_and_kubelet_restart():
    """The CU-mask slice plugin: render node of a slice's GPU from the device map (not /dev/dri
    order), Unhealthy when its GPU leaves the map, re-served and re-registered after a kubelet
    restart (sockets wiped, kubelet.sock recreated)."""
    from walkai_nos_amd.device.slicing_client import MemorySliceStore
    from walkai_nos_amd.deviceplugin.server import PluginManager
    from walkai_nos_amd.models.slicing.cumask import Slice
    smi = FakeAmdSmi(n_gpus=2)
    dm = smi.device_map()
    b0, b1 = dm.gpus[0].bdf, dm.gpus[1].bdf
    store = MemorySliceStore()
    store.save({0: [Slice(f"{b0}::s0", "32cu.36gb", [0, 1, 2, 3], 36 * 10**9)],
                1: [Slice(f"{b1}::s0", "32cu.36gb", [0, 1, 2, 3], 36 * 10**9)]})
    with tempfile.TemporaryDirectory() as d:
        reg = RegistrationServer(os.path.join(d, "kubelet.sock")).start()
        # a wrong directory-order fallback: the device map must win
        mgr = PluginManager(store, {0: "/dev/dri/renderD999", 1: "/dev/dri/renderD998"}, socket_dir=d,
                            kubelet_socket=reg.socket, device_map=smi.device_map, register_backoff=0.01)
        try:
            mgr.sync()
            plug = mgr.plugins["amd.com/gpu-32cu.36gb"]
            a = dp.AllocateRequest()
            a.container_requests.add(devicesIDs=[f"{b1}::s0"])
            r = plug.Allocate(a, None).container_responses[0]
            assert [x.host_path for x in r.devices] == ["/dev/kfd", f"/dev/dri/renderD{dm.devices[1].render_minor}"]
            assert plug.device_states() == [(f"{b0}::s0", True), (f"{b1}::s0", True)]
            smi._gpus.pop(1)
            smi.enumerate(reinit=True)
            assert plug.device_states() == [(f"{b0}::s0", True), (f"{b1}::s0", False)]
            reg.stop()
            for f in os.listdir(d):
                os.unlink(os.path.join(d, f))
            reg2 = RegistrationServer(os.path.join(d, "kubelet.sock")).start()
            mgr.sync()
            assert [r.resource_name for r in reg2.registered] == ["amd.com/gpu-32cu.36gb"] and plug.serving()
            reg2.stop()
        finally:
            mgr.stop()
