"""The public test helpers (walkai_nos_amd.testing): builders feed the real planners/agents, and the
recording fakes capture interactions (reference pkg/test/factory, pkg/test/mocks)."""
import pytest

from walkai_nos_amd.api import v1alpha1 as api
from walkai_nos_amd.controllers.agent.actuator import Actuator
from walkai_nos_amd.controllers.agent.shared import SharedState
from walkai_nos_amd.kube import objects as ko
from walkai_nos_amd.kube.memory import InMemoryAPIServer
from walkai_nos_amd.kube.runtime import Request
from walkai_nos_amd.models.device import DeviceList, GpuDevice
from walkai_nos_amd.models.errors import GpuError
from walkai_nos_amd.models.resource import compute_pod_request
from walkai_nos_amd.testing import (MockDevicePluginClient, MockPartitionClient, NodeBuilder, PodBuilder,
                                    RecordingBarrier)
from walkai_nos_amd.utils import pod as podutil


def test_builders_produce_valid_objects():
    node = NodeBuilder("n0").with_mi355x(8, "xcp").with_allocatable({"amd.com/gpu": 8}).build()
    assert ko.labels(node)[api.LABEL_GPU_PARTITIONING] == "xcp" and node["status"]["allocatable"]["amd.com/gpu"] == "8"
    pod = (PodBuilder("p", "ns").with_container(requests={"amd.com/cpx_nps1": 1, "cpu": "500m"})
           .with_container(requests={"amd.com/cpx_nps1": 1}).with_init_container({"amd.com/cpx_nps1": 3})
           .with_overhead({"cpu": "100m"}).unschedulable().with_priority(5).build())
    assert podutil.is_unschedulable(pod) and pod["spec"]["priority"] == 5
    req = compute_pod_request(pod)
    assert req["amd.com/cpx_nps1"] == 3  # max(sum of containers, max init container)


def _dev(i, gpu, profile, status):
    return GpuDevice(f"d{i}", f"amd.com/{profile}", status, gpu)


def test_mocks_record_actuator_interactions_and_inject_failures():
    api_ = InMemoryAPIServer()
    api_.create(NodeBuilder("node-a").with_mi355x(2, "xcp").build())
    pc = MockPartitionClient(DeviceList([_dev(0, 0, "spx_nps1", "free"), _dev(1, 1, "spx_nps1", "free")]),
                             profiles={0: "spx_nps1", 1: "spx_nps1"})
    dp = MockDevicePluginClient()
    bar = RecordingBarrier()
    shared = SharedState()
    act = Actuator(api_, pc, shared, "node-a", dp, barrier_factory=lambda n: bar)
    api_.patch("Node", "node-a", {"metadata": {"annotations": {"nos.nebuly.com/spec-gpu-1-cpx_nps1": "8",
                                                               api.ANNOTATION_PARTITIONING_PLAN: "1"}}})
    shared.on_report_done()
    act.reconcile(Request("node-a"))
    assert ("set_profile", (1, "cpx_nps1")) in pc.calls and pc.profiles[1] == "cpx_nps1"
    assert bar.votes == [True] and dp.counts["restart"] == 1
    pc.fail_next("get_partition_devices")
    with pytest.raises(GpuError):
        pc.get_partition_devices()
