"""End-to-end on the in-process cluster (SURVEY §7.4 minimum slice and churn scenarios)."""
import pytest

from walkai_nos_amd.api import v1alpha1 as api
from walkai_nos_amd.kube import objects as ko
from walkai_nos_amd.sim.cluster import SimCluster


def anns(c, node="node-0"):
    return ko.annotations(c.api.get("Node", node))


def test_minimum_slice_spx_to_cpx_eight_pods():
    c = SimCluster(n_nodes=1, gpus_per_node=1)
    c.run(30)
    a = anns(c)
    assert a["nos.nebuly.com/spec-gpu-0-spx_nps1"] == "1"
    assert a["nos.nebuly.com/status-gpu-0-spx_nps1-free"] == "1"
    assert a[api.ANNOTATION_REPORTED_PARTITIONING_PLAN] == a[api.ANNOTATION_PARTITIONING_PLAN]
    for i in range(8):
        c.submit({"amd.com/cpx_nps1": 1}, name=f"w{i}")
    c.run(60)
    a = anns(c)
    assert a["nos.nebuly.com/spec-gpu-0-cpx_nps1"] == "8"
    assert a["nos.nebuly.com/status-gpu-0-cpx_nps1-used"] == "8"
    assert a[api.ANNOTATION_REPORTED_PARTITIONING_PLAN] == a[api.ANNOTATION_PARTITIONING_PLAN]
    assert a[api.ANNOTATION_COMMIT_STATUS] == "ok"
    assert len(c.running_pods()) == 8 and not c.pending_pods()
    assert c.utilization() == 100.0
    assert c.nodes["node-0"].smi.set_calls == [("compute", 0, "CPX")]


def test_gpu_returns_to_spx_after_partitions_drain():
    c = SimCluster(n_nodes=1, gpus_per_node=1)
    c.run(30)
    for i in range(3):
        c.submit({"amd.com/cpx_nps1": 1}, name=f"w{i}")
    c.run(60)
    c.submit({"amd.com/spx_nps1": 1}, name="big")
    c.run(60)
    assert [ko.name(p) for p in c.pending_pods()] == ["big"]  # CPX pinned by running partitions
    for i in range(3):
        c.complete(f"w{i}")
    c.run(120)
    assert [ko.name(p) for p in c.running_pods()] == ["big"]
    assert anns(c)["nos.nebuly.com/status-gpu-0-spx_nps1-used"] == "1"


def test_mixed_fractions_across_gpus_and_nodes():
    c = SimCluster(n_nodes=2, gpus_per_node=2)
    c.run(30)
    reqs = [{"amd.com/spx_nps1": 1}, {"amd.com/dpx_nps1": 1}, {"amd.com/dpx_nps1": 1}] + \
           [{"amd.com/cpx_nps1": 1}] * 8 + [{"amd.com/qpx_nps1": 1}] * 4
    for i, r in enumerate(reqs):
        c.submit(r, name=f"w{i}")
    c.run(120)
    assert len(c.running_pods()) == len(reqs)
    assert c.utilization() == 100.0  # 1 + 2x1/2 + 8x1/8 + 4x1/4 = 4 GPUs exactly


def test_permission_denied_agent_keeps_pods_pending_and_reports_failure():
    c = SimCluster(n_nodes=1, gpus_per_node=1)
    c.run(30)
    c.nodes["node-0"].smi.is_root = False
    c.submit({"amd.com/cpx_nps1": 1}, name="w")
    c.run(60)
    assert [ko.name(p) for p in c.pending_pods()] == ["w"]
    assert anns(c)[api.ANNOTATION_COMMIT_STATUS] == "failed"
    # the operator fixes permissions: the agent's retry (back-off) applies the plan
    c.nodes["node-0"].smi.is_root = True
    c.run(600)
    assert [ko.name(p) for p in c.running_pods()] == ["w"]


def test_partial_failure_rolls_back_whole_plan():
    c = SimCluster(n_nodes=1, gpus_per_node=2)
    c.run(30)
    c.nodes["node-0"].smi.fail_next = 1  # the next amd-smi set fails once
    for i in range(9):
        c.submit({"amd.com/cpx_nps1": 1}, name=f"w{i}")
    c.run(300)
    assert len(c.running_pods()) == 9


@pytest.mark.slow
def test_churn_keeps_utilisation_high_on_eight_gpus():
    from walkai_nos_amd.bench_core import BenchConfig, NodeBench
    nb = NodeBench(BenchConfig(gpus=8), gpu_data_plane=False)
    for _ in range(100):
        nb.control_step()
        nb.end_step()
    # effective allocation (flipped GPUs dark for flip_cost_s) of the flip-aware pack policy
    assert sum(nb.util_samples[60:]) / len(nb.util_samples[60:]) > 95.0
    assert max(nb.pods_samples) > 8
