"""Partition agent: node-side plan, actuator (rollback, commit barrier, handshake) and reporter.

Mirrors the reference's actuator unit/integration scenarios (internal/controllers/migagent/
actuator_test.go:31-212, actuator_int_test.go:64-256, reporter_int_test.go:56-100) on the
MI355X compute-partition model.
"""
import pytest

from walkai_nos_amd.api import v1alpha1 as api
from walkai_nos_amd.controllers.agent.actuator import Actuator
from walkai_nos_amd.controllers.agent.plan import ModeChange, XcpState, new_xcp_config_plan
from walkai_nos_amd.controllers.agent.reporter import Reporter
from walkai_nos_amd.controllers.agent.shared import SharedState
from walkai_nos_amd.device.amdsmi import FakeAmdSmi
from walkai_nos_amd.device.partition_client import PartitionClient
from walkai_nos_amd.device.podresources import StaticResourceClient
from walkai_nos_amd.kube import objects as ko
from walkai_nos_amd.kube.memory import InMemoryAPIServer
from walkai_nos_amd.kube.runtime import Request
from walkai_nos_amd.models.annotation import SpecAnnotation
from walkai_nos_amd.models.device import GpuDevice
from walkai_nos_amd.parallel.barrier import CommitBarrier


def dev(profile, gpu, k, status):
    return GpuDevice(f"amd.com/{profile}", f"g{gpu}/xcp{k}", status, gpu)


# -- plan ---------------------------------------------------------------------------------
def test_plan_flips_only_idle_gpus_named_in_spec():
    state = XcpState([dev("spx_nps1", 0, 0, "free"), dev("cpx_nps1", 1, 0, "used")] +
                     [dev("cpx_nps1", 1, k, "free") for k in range(1, 8)] + [dev("spx_nps1", 2, 0, "free")])
    current = {0: "spx_nps1", 1: "cpx_nps1", 2: "spx_nps1"}
    spec = [SpecAnnotation("cpx_nps1", 0, 8), SpecAnnotation("spx_nps1", 1, 1)]
    plan = new_xcp_config_plan(state, current, spec)
    assert plan.changes == [ModeChange(0, "spx_nps1", "cpx_nps1")]
    assert [g for g, _ in plan.blocked] == [1]  # GPU 1 has a partition in use
    assert not plan.is_empty()


def test_plan_rejects_invalid_spec_and_noop_when_matching():
    state = XcpState([dev("spx_nps1", 0, 0, "free")])
    plan = new_xcp_config_plan(state, {0: "spx_nps1"}, [SpecAnnotation("cpx_nps1", 0, 3)])
    assert plan.is_empty() and plan.invalid
    plan = new_xcp_config_plan(state, {0: "spx_nps1"}, [SpecAnnotation("cpx_nps1", 0, 8),
                                                         SpecAnnotation("spx_nps1", 0, 1)])
    assert plan.is_empty() and plan.invalid
    assert new_xcp_config_plan(state, {0: "spx_nps1"}, [SpecAnnotation("spx_nps1", 0, 1)]).is_empty()
    assert state.matches([SpecAnnotation("spx_nps1", 0, 1)])


def test_plan_memory_partition_change_needs_idle_node():
    idle = XcpState([dev("spx_nps1", 0, 0, "free"), dev("spx_nps1", 1, 0, "free")])
    plan = new_xcp_config_plan(idle, {0: "spx_nps1", 1: "spx_nps1"},
                               [SpecAnnotation("dpx_nps2", 0, 2), SpecAnnotation("dpx_nps2", 1, 2)],
                               spec_nps=None, current_nps="nps1")
    assert plan.memory_partition == "nps2"
    busy = XcpState([dev("spx_nps1", 0, 0, "used"), dev("spx_nps1", 1, 0, "free")])
    plan = new_xcp_config_plan(busy, {0: "spx_nps1", 1: "spx_nps1"},
                               [SpecAnnotation("dpx_nps2", 1, 2)], spec_nps="nps2", current_nps="nps1")
    assert plan.memory_partition is None and plan.blocked


# -- actuator / reporter fixtures ----------------------------------------------------------
class Env:
    def __init__(self, n_gpus=2, used=()):
        self.api = InMemoryAPIServer()
        self.smi = FakeAmdSmi(n_gpus=n_gpus)
        self.used = set(used)
        self.api.create(ko.new_node("node-a", {api.LABEL_GPU_PARTITIONING: "xcp"}))
        rc = StaticResourceClient(
            lambda: [(r, i) for r, i in self.alloc() if i in self.used],
            lambda: self.alloc())
        self.pc = PartitionClient(rc, self.smi)
        self.shared = SharedState()
        self.restarts = 0
        me = self

        class DP:
            def restart(self, node, timeout=60):
                me.restarts += 1

        self.votes = []

        class Bar(CommitBarrier):
            def __init__(self, veto=False):
                self.veto = veto

            def vote(self, ok):
                me.votes.append(ok)
                return ok and not self.veto

        self.veto = False
        self.actuator = Actuator(self.api, self.pc, self.shared, "node-a", DP(),
                                 barrier_factory=lambda n: Bar(self.veto))
        self.reporter = Reporter(self.api, self.pc, self.shared, refresh_interval=10)

    def alloc(self):
        return [(f"amd.com/{d.compute_mode.lower()}_{d.memory_mode.lower()}", d.device_id)
                for d in self.smi.logical_devices()]

    def spec(self, anns):
        self.api.patch("Node", "node-a", {"metadata": {"annotations": anns}})

    def annotations(self):
        return ko.annotations(self.api.get("Node", "node-a"))


def test_actuator_waits_for_a_report_then_applies_and_reregisters():
    e = Env()
    e.spec({"nos.nebuly.com/spec-gpu-0-cpx_nps1": "8", api.ANNOTATION_PARTITIONING_PLAN: "42"})
    res = e.actuator.reconcile(Request("node-a"))
    assert res.requeue_after == 1.0 and e.smi.set_calls == []  # no report since last apply
    e.reporter.reconcile(Request("node-a"))
    e.actuator.reconcile(Request("node-a"))
    assert e.smi.get_compute_partition(0) == "CPX" and e.smi.get_compute_partition(1) == "SPX"
    assert e.restarts == 1 and e.votes == [True] and e.shared.last_commit == "ok"
    e.reporter.reconcile(Request("node-a"))
    a = e.annotations()
    assert a["nos.nebuly.com/status-gpu-0-cpx_nps1-free"] == "8"
    assert a["nos.nebuly.com/status-gpu-1-spx_nps1-free"] == "1"
    assert a[api.ANNOTATION_REPORTED_PARTITIONING_PLAN] == "42"
    assert a[api.ANNOTATION_COMMIT_STATUS] == "ok"
    # spec == status now: a second pass is a no-op (no flip, no restart)
    e.actuator.reconcile(Request("node-a"))
    assert len(e.smi.set_calls) == 1 and e.restarts == 1


def test_actuator_rolls_back_when_a_flip_fails():
    e = Env(n_gpus=3)
    e.smi.fail_set = {2}
    e.reporter.reconcile(Request("node-a"))
    e.spec({"nos.nebuly.com/spec-gpu-0-cpx_nps1": "8", "nos.nebuly.com/spec-gpu-1-qpx_nps1": "4",
            "nos.nebuly.com/spec-gpu-2-dpx_nps1": "2"})
    with pytest.raises(Exception):
        e.actuator.reconcile(Request("node-a"))
    # GPUs 0 and 1 were flipped, GPU 2 failed -> 0 and 1 restored to SPX (node-atomic)
    assert [e.smi.get_compute_partition(i) for i in range(3)] == ["SPX", "SPX", "SPX"]
    assert e.shared.last_commit == "failed"


def test_actuator_rolls_back_on_barrier_veto():
    e = Env()
    e.veto = True
    e.reporter.reconcile(Request("node-a"))
    e.spec({"nos.nebuly.com/spec-gpu-0-cpx_nps1": "8"})
    with pytest.raises(Exception):
        e.actuator.reconcile(Request("node-a"))
    assert e.smi.get_compute_partition(0) == "SPX"


def test_plugin_registration_failure_after_a_commit_does_not_leave_the_journal():
    """kubelet restarting during an apply (the plugin sync raising) must not escape
    apply(): the flip is committed, the journal cleared and the commit recorded."""
    e = Env()

    class FailingHook:
        def restart(self, node, timeout=60):
            raise RuntimeError("unable to register amd.com/cpx_nps1 with kubelet")
    e.actuator.device_plugin = FailingHook()
    e.reporter.reconcile(Request("node-a"))
    e.spec({"nos.nebuly.com/spec-gpu-0-cpx_nps1": "8", api.ANNOTATION_PARTITIONING_PLAN: "7"})
    e.actuator.reconcile(Request("node-a"))
    assert e.smi.get_compute_partition(0) == "CPX" and e.shared.last_commit == "ok"
    assert api.ANNOTATION_INFLIGHT_PLAN not in e.annotations()


def test_barrier_that_cannot_start_is_a_veto_and_rolls_back():
    """a commit barrier whose construction fails (native helper missing) after the
    switch vetoes the plan: the GPU is flipped back and the journal cleared."""
    e = Env()

    def broken(n):
        raise RuntimeError("native helper nos-gpuhelper is not built")
    e.actuator.barrier_factory = broken
    e.reporter.reconcile(Request("node-a"))
    e.spec({"nos.nebuly.com/spec-gpu-0-cpx_nps1": "8"})
    with pytest.raises(Exception):
        e.actuator.reconcile(Request("node-a"))
    assert e.smi.get_compute_partition(0) == "SPX" and e.shared.last_commit == "failed"
    assert api.ANNOTATION_INFLIGHT_PLAN not in e.annotations()


def test_actuator_never_flips_a_gpu_with_used_partitions():
    e = Env()
    e.smi.set_compute_partition(0, "CPX")
    e.used = {e.alloc()[0][1]}  # one CPX partition of GPU 0 in use
    e.reporter.reconcile(Request("node-a"))
    e.spec({"nos.nebuly.com/spec-gpu-0-spx_nps1": "1"})
    e.actuator.reconcile(Request("node-a"))
    assert e.smi.get_compute_partition(0) == "CPX" and e.restarts == 0


def test_actuator_permission_denied_surfaces_error_and_keeps_modes():
    e = Env()
    e.smi.is_root = False
    e.reporter.reconcile(Request("node-a"))
    e.spec({"nos.nebuly.com/spec-gpu-0-cpx_nps1": "8"})
    with pytest.raises(Exception) as ei:
        e.actuator.reconcile(Request("node-a"))
    assert "PERMISSION" in str(ei.value)
    assert e.smi.get_compute_partition(0) == "SPX"


def test_failed_plan_is_retried_but_applied_plan_is_not_repeated():
    e = Env()
    e.smi.fail_next = 1
    e.reporter.reconcile(Request("node-a"))
    e.spec({"nos.nebuly.com/spec-gpu-0-cpx_nps1": "8"})
    with pytest.raises(Exception):
        e.actuator.reconcile(Request("node-a"))
    assert e.smi.get_compute_partition(0) == "SPX"
    e.reporter.reconcile(Request("node-a"))
    e.actuator.reconcile(Request("node-a"))  # retry succeeds
    assert e.smi.get_compute_partition(0) == "CPX"
    restarts = e.restarts
    e.actuator.last_applied_status = None  # force the dedup path below to rely on the plan only
    e.reporter.reconcile(Request("node-a"))
    e.actuator.reconcile(Request("node-a"))  # spec now matches status -> nothing to do
    assert e.restarts == restarts


def test_deleted_node_is_ignored():
    e = Env()
    e.reporter.reconcile(Request("node-a"))
    e.api.delete("Node", "node-a")
    assert e.actuator.reconcile(Request("node-a")).requeue_after == 0
    assert e.reporter.reconcile(Request("node-a")).requeue_after == 0


def test_reporter_only_patches_on_change_and_echoes_plan_id():
    e = Env()
    e.shared.last_parsed_plan_id = "7"
    e.reporter.reconcile(Request("node-a"))
    rv = e.api.get("Node", "node-a")["metadata"]["resourceVersion"]
    res = e.reporter.reconcile(Request("node-a"))
    assert res.requeue_after == 10
    assert e.api.get("Node", "node-a")["metadata"]["resourceVersion"] == rv
    a = e.annotations()
    assert a[api.ANNOTATION_REPORTED_PARTITIONING_PLAN] == "7"
    assert a[api.ANNOTATION_MEMORY_PARTITION_STATUS] == "nps1"
    # stale status keys are stripped on the next report
    e.api.patch("Node", "node-a", {"metadata": {"annotations": {"nos.nebuly.com/status-gpu-9-cpx_nps1-free": "1"}}})
    e.reporter.reconcile(Request("node-a"))
    assert "nos.nebuly.com/status-gpu-9-cpx_nps1-free" not in e.annotations()


def test_shared_state_token_semantics():
    s = SharedState()
    assert not s.at_least_one_report_since_last_apply()
    s.on_report_done()
    s.on_report_done()
    assert s.at_least_one_report_since_last_apply()
    assert not s.at_least_one_report_since_last_apply()  # consumed
    s.on_report_done()
    s.on_apply_done()
    assert not s.at_least_one_report_since_last_apply()


def test_probe_on_commit_publishes_status_probe_annotation():
    import json

    from walkai_nos_amd.controllers.agent.probe import ProbeRunner
    e = Env()
    calls = []

    def fake_probe(dev, cus, label):
        calls.append(label)
        n = 32 if e.smi.get_compute_partition(0) == "CPX" else 256
        return {"n_cus": n, "bf16_tflops": 5.0 * n, "fp32_tflops": 0.5 * n, "hbm_gbps": 600.0}

    runner = ProbeRunner(e.shared, "node-a", probe_fn=fake_probe,
                         targets=lambda: [(i, None, f"dev{i}") for i in range(2)], asynchronous=False)
    e.reporter.extra = runner.annotations
    e.reporter.reconcile(Request("node-a"))
    doc = json.loads(e.annotations()[api.ANNOTATION_PROBE_RESULT])  # startup baseline of the current layout
    assert doc["commit"] == 0 and doc["slices"]["dev0"]["fp32_tflops"] == 128.0
    e.spec({"nos.nebuly.com/spec-gpu-0-cpx_nps1": "8", api.ANNOTATION_PARTITIONING_PLAN: "1"})
    e.actuator.reconcile(Request("node-a"))
    e.reporter.reconcile(Request("node-a"))
    doc = json.loads(e.annotations()[api.ANNOTATION_PROBE_RESULT])
    assert doc["commit"] == 1 and set(doc["slices"]) == {"dev0", "dev1"}
    assert doc["slices"]["dev0"]["fp32_tflops"] == 16.0
    e.reporter.reconcile(Request("node-a"))
    assert calls == ["dev0", "dev1"] * 2  # one probe round per commit, not per report


def test_probe_runner_survives_a_failing_slice():
    from walkai_nos_amd.controllers.agent.probe import ProbeRunner
    s = SharedState()

    def probe(dev, cus, label):
        if dev == 1:
            raise RuntimeError("device lost")
        return {"n_cus": 64, "bf16_tflops": 300.0}

    r = ProbeRunner(s, "n", probe_fn=probe, targets=lambda: [(0, None, "a"), (1, None, "b")], asynchronous=False)
    s.record_commit(True)
    r.poll()
    assert r.results["slices"]["a"]["bf16_tflops"] == 300.0 and "error" in r.results["slices"]["b"]
    s.record_commit(False)  # a vetoed commit does not trigger a new round
    r.poll()
    assert r.results["commit"] == 1
