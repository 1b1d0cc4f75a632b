"""CU-mask slicing: B.7 geometry update (reference pkg/gpu/slicing/gpu_test.go:122-343 vectors),
2-D budgets, XCD-symmetric CU placement, the slice agent plan and the cumask end-to-end path."""
import pytest

from walkai_nos_amd.controllers.sliceagent.agent import plan_slices
from walkai_nos_amd.kube import objects as ko
from walkai_nos_amd.models.annotation import SpecAnnotation
from walkai_nos_amd.models.errors import GpuError
from walkai_nos_amd.models.slicing.cumask import Slice, cus_of, hsa_cu_mask, mask_hex, place
from walkai_nos_amd.models.slicing.gpu import SlicingGPU, SlicingNode
from walkai_nos_amd.models.slicing.profile import (SliceProfile, extract_gpu_id, extract_profile_name, new_profile,
                                                   parse_profile)
from walkai_nos_amd.sim.cluster import SimCluster


def sg(mem, used=None, free=None, cus=256):
    g = SlicingGPU("MI355X", 0, mem, cus, dict(used or {}), dict(free or {}))
    g.validate()
    return g


@pytest.mark.parametrize("gpu,required,expected,updated", [
    (sg(40, {"10gb": 2}, {"20gb": 1}), {}, {"10gb": 2, "20gb": 1}, False),
    (sg(40, {}, {"20gb": 2}), {"20gb": 2}, {"20gb": 2}, False),
    (sg(40, {"20gb": 2}), {"10gb": 1, "20gb": 1}, {"20gb": 2}, False),                      # full GPU
    (sg(60, {"10gb": 1}), {"10gb": 1, "20gb": 2}, {"10gb": 2, "20gb": 2}, True),           # spare capacity
    (sg(40), {"10gb": 5}, {"10gb": 4}, True),                                              # capped by memory
    (sg(40), {"20gb": 2, "10gb": 2, "5gb": 2}, {"5gb": 2, "10gb": 2}, True),                # smaller first
    (sg(40, {"20gb": 1}, {"10gb": 2}), {"20gb": 1}, {"20gb": 2}, True),                     # delete free to fit
])
def test_update_geometry_for_reference_vectors(gpu, required, expected, updated):
    assert gpu.update_geometry_for(required) is updated
    assert gpu.geometry() == expected


def test_free_slices_kept_when_spare_capacity_suffices():
    g = sg(40, {"10gb": 2}, {"5gb": 1})
    assert g.update_geometry_for({"10gb": 1})
    assert g.geometry() == {"10gb": 3, "5gb": 1}


def test_validation_and_cu_budget():
    with pytest.raises(ValueError):
        sg(40, {"30gb": 2})
    with pytest.raises(ValueError):
        SlicingGPU("MI355X", 0, 288, 256, {"48cu.10gb": 1}).validate()  # not a multiple of 32 CUs
    g = SlicingGPU.full("MI355X", 0, 288, 256)
    assert g.update_geometry_for({"128cu.100gb": 3})
    assert g.geometry() == {"128cu.100gb": 2}  # 256 dedicated CUs max
    g2 = SlicingGPU.full("MI355X", 0, 288, 256)
    g2.create_slices("10gb", 1)  # a shared slice reserves one 32-CU row group for the shared pool
    assert not g2.create_slices("256cu.10gb", 1)
    assert g2.create_slices("224cu.10gb", 1)


def test_profiles():
    assert parse_profile("32cu.36gb") == SliceProfile(36, 32)
    assert parse_profile("10gb") == SliceProfile(10, 0) and not parse_profile("10gb").dedicated
    assert new_profile(36, 32) == "32cu.36gb"
    assert extract_profile_name("amd.com/gpu-32cu.36gb") == "32cu.36gb"
    assert extract_profile_name("amd.com/gpu") is None and extract_profile_name("amd.com/cpx_nps1") is None
    assert extract_gpu_id("0000:a4:00.0::s3") == "0000:a4:00.0"
    assert parse_profile("32cu.36gb") < parse_profile("32cu.40gb") < parse_profile("8cu.64gb")


def test_cumask_rows_are_xcd_symmetric_and_used_slices_stay():
    keep = [Slice("g::s0", "128cu.144gb", list(range(16)))]
    placed = place(keep, [("g::s1", "32cu.36gb"), ("g::s2", "64cu.72gb")], 256)
    by = {s.id: s for s in placed}
    assert by["g::s2"].rows == [16, 17, 18, 19, 20, 21, 22, 23]  # largest first, contiguous
    assert by["g::s1"].rows == [24, 25, 26, 27]
    for s in placed:
        assert {c % 8 for c in s.cus} == set(range(8))  # every XCD
    assert hsa_cu_mask(by["g::s1"].cus) == "0:192-223"
    assert mask_hex(range(32)) == "ffffffff," + ",".join(["00000000"] * 7)
    shared = Slice("g::s3", "10gb")
    assert len(cus_of(shared, keep + placed + [shared], 256)) == 256 - 128 - 32 - 64
    with pytest.raises(ValueError):
        place(keep + placed, [("g::s4", "128cu.10gb")], 256)


def test_slice_plan_deletes_free_keeps_used_and_checks_budgets():
    cur = {0: [Slice("g::s0", "256cu.288gb", list(range(32)))]}
    plan = plan_slices(cur, set(), [SpecAnnotation("32cu.36gb", 0, 3)], {0: "g"}, 288, 256)
    assert plan.deleted == ["g::s0"] and len(plan.created) == 3
    assert [s.profile for s in plan.new[0]] == ["32cu.36gb"] * 3
    # a used slice is never deleted even if the spec drops it
    cur = {0: [Slice("g::s0", "64cu.72gb", list(range(8)))]}
    plan = plan_slices(cur, {"g::s0"}, [SpecAnnotation("32cu.36gb", 0, 1)], {0: "g"}, 288, 256)
    assert plan.deleted == [] and plan.blocked and len(plan.new[0]) == 2
    with pytest.raises(GpuError):
        plan_slices({}, set(), [SpecAnnotation("32cu.100gb", 0, 3)], {0: "g"}, 288, 256)


def test_cumask_end_to_end_heterogeneous_slices_on_one_gpu():
    c = SimCluster(n_nodes=1, gpus_per_node=1, kind="cumask")
    c.run(30)
    a = ko.annotations(c.api.get("Node", "node-0"))
    assert a["nos.nebuly.com/status-gpu-0-256cu.288gb-free"] == "1"
    for _ in range(4):
        c.submit({"amd.com/gpu-32cu.36gb": 1})
    c.submit({"amd.com/gpu-128cu.144gb": 1})
    c.run(60)
    assert len(c.running_pods()) == 5 and c.utilization() == 100.0
    slices = c.nodes["node-0"].plugin.store.load()[0]
    rows = [r for s in slices for r in s.rows]
    assert len(rows) == len(set(rows)) == 32  # disjoint, every CU owned once


def test_slicing_node_greedy():
    n = SlicingNode("n", [SlicingGPU.full("MI355X", 0, 288), SlicingGPU.full("MI355X", 1, 288)])
    assert n.update_geometry_for({"32cu.36gb": 10})
    assert n.gpus[0].geometry() == {"32cu.36gb": 8} and n.gpus[1].geometry() == {"32cu.36gb": 2}
    assert n.allocatable["amd.com/gpu-32cu.36gb"] == 10


def test_row_groups_keep_slices_shader_engine_balanced():
    from walkai_nos_amd.models.slicing.cumask import GROUP_ROWS, allocate_rows
    placed = place([], [("g::a", "32cu.36gb"), ("g::b", "96cu.108gb"), ("g::c", "64cu.72gb")], 256)
    for s_ in placed:
        # every slice owns each shader engine (row mod 4) of every XCD equally often
        per_se = [sum(1 for r in s_.rows if r % GROUP_ROWS == se) for se in range(GROUP_ROWS)]
        assert len(set(per_se)) == 1, (s_.profile, s_.rows)
    # a stale unaligned slice blocks its whole group, never splits a new slice over SEs unevenly
    rows = allocate_rows(4, [5], 32)
    assert rows == [0, 1, 2, 3]
    assert allocate_rows(8, [5], 32) == [8, 9, 10, 11, 12, 13, 14, 15]


def test_slice_probe_targets_cover_each_live_slice_cu_set():
    from walkai_nos_amd.controllers.sliceagent.agent import slice_probe_targets
    from walkai_nos_amd.device.slicing_client import MemorySliceStore
    store = MemorySliceStore()
    store.save({0: place([], [("g::s0", "32cu.36gb"), ("g::s1", "64cu.72gb")], 256), 1: [Slice("h::s0", "10gb")]})
    t = {label: (gpu, cus) for gpu, cus, label in slice_probe_targets(store)()}
    assert set(t) == {"g::s0", "g::s1", "h::s0"}
    assert len(t["g::s0"][1]) == 32 and len(t["g::s1"][1]) == 64 and t["g::s1"][0] == 0
    assert t["h::s0"][0] == 1 and len(t["h::s0"][1]) == 256  # memory-only slice runs on the shared pool


# -- slice-agent reporter (reference internal/controllers/gpuagent/reporter_int_test.go:61-177) --
class _SliceDevices:
    """Slicing client stub: the reporter only calls ``get_partition_devices``."""

    def __init__(self, devs):
        self.devs = devs

    def get_partition_devices(self):
        from walkai_nos_amd.models.device import devices
        return devices(self.devs)


def _slice_reporter(devs):
    from walkai_nos_amd.api import v1alpha1 as api
    from walkai_nos_amd.controllers.agent.reporter import Reporter
    from walkai_nos_amd.controllers.agent.shared import SharedState
    from walkai_nos_amd.kube.memory import InMemoryAPIServer
    srv = InMemoryAPIServer()
    srv.create(ko.new_node("node-s", {api.LABEL_GPU_PARTITIONING: "cumask"}))
    rep = Reporter(srv, _SliceDevices(devs), SharedState(), refresh_interval=5,
                   profile_extractor=extract_profile_name)
    return srv, rep


def _status(srv):
    from walkai_nos_amd.api import v1alpha1 as api
    return {k: v for k, v in ko.annotations(srv.get("Node", "node-s")).items()
            if k.startswith(api.ANNOTATION_GPU_STATUS_PREFIX)}


def test_slice_reporter_without_gpus_writes_no_status_annotations():
    from walkai_nos_amd.kube.runtime import Request
    srv, rep = _slice_reporter([])
    assert rep.reconcile(Request("node-s")).requeue_after == 5
    assert _status(srv) == {}


def test_slice_reporter_groups_slices_and_excludes_whole_gpu_resource():
    from walkai_nos_amd.kube.runtime import Request
    from walkai_nos_amd.models.device import GpuDevice
    devs = [GpuDevice("amd.com/gpu-32cu.36gb", "g0/s0", "used", 0),
            GpuDevice("amd.com/gpu-32cu.36gb", "g0/s1", "used", 0),
            GpuDevice("amd.com/gpu-64cu.72gb", "g0/s2", "free", 0),
            GpuDevice("amd.com/gpu-128cu.144gb", "g1/s0", "free", 1),
            GpuDevice("amd.com/gpu", "g2", "used", 2)]  # plain whole-GPU resource: never reported
    srv, rep = _slice_reporter(devs)
    rep.reconcile(Request("node-s"))
    assert _status(srv) == {"nos.nebuly.com/status-gpu-0-32cu.36gb-used": "2",
                            "nos.nebuly.com/status-gpu-0-64cu.72gb-free": "1",
                            "nos.nebuly.com/status-gpu-1-128cu.144gb-free": "1"}
    # unchanged devices: the next report does not patch the node again
    rv = srv.get("Node", "node-s")["metadata"]["resourceVersion"]
    rep.reconcile(Request("node-s"))
    assert srv.get("Node", "node-s")["metadata"]["resourceVersion"] == rv


def test_pack_policy_plans_cumask_nodes_oldest_first():
    """The partitioner's default policy is ``pack`` (compute partitions); on a cumask node it must
    still plan slices (found by the process-level test: the pack planner assumed partition GPUs)."""
    from walkai_nos_amd.controllers.partitioner.setup import policy_for
    assert policy_for("cumask", "pack") == "fifo" and policy_for("xcp", "pack") == "pack"
    c = SimCluster(n_nodes=1, gpus_per_node=1, kind="cumask", policy="pack")
    c.run(30)
    c.submit({"amd.com/gpu-64cu.72gb": 1}, name="s0")
    c.submit({"amd.com/gpu-36gb": 1}, name="m0")
    c.run(120)
    assert {ko.name(p) for p in c.running_pods()} == {"s0", "m0"}


def test_at_most_eight_slices_per_gpu_unless_the_node_allows_more():
    """Each slice serves one pod process, and beyond 8 processes per GPU the hardware scheduler
    time-slices them (profiles/procs_cap_r4.json): the planner carves at most 8 slices per GPU;
    the node label nos.nebuly.com/max-slices-per-gpu raises (or lowers) it."""
    g = SlicingGPU.full("MI355X", 0, 288)
    assert g.create_slices("8gb", 8) and not g.create_slices("8gb", 1)
    assert not g.can_create_more_slices() and g.spare_memory_gb() == 288 - 64
    n = SlicingNode("n", [SlicingGPU.full("MI355X", 0, 288), SlicingGPU.full("MI355X", 1, 288)])
    n.update_geometry_for({"16gb": 12})
    assert n.gpus[0].geometry() == {"16gb": 8} and n.gpus[1].geometry() == {"16gb": 4}
    wide = SlicingGPU.full("MI355X", 0, 288, max_slices=16)
    assert wide.create_slices("8gb", 16) and not wide.create_slices("8gb", 1)
    assert wide.clone().max_slices == 16


@pytest.mark.parametrize("label,running", [(None, 8), ("10", 10), ("bogus", 8)])
def test_cumask_node_serves_at_most_its_slice_cap(label, running):
    c = SimCluster(n_nodes=1, gpus_per_node=1, kind="cumask")
    if label is not None:
        c.api.patch("Node", "node-0", {"metadata": {"labels": {"nos.nebuly.com/max-slices-per-gpu": label}}})
    c.run(30)
    for i in range(12):
        c.submit({"amd.com/gpu-8gb": 1}, name=f"m{i}")
    c.run(120)
    assert len(c.running_pods()) == running and len(c.pending_pods()) == 12 - running


@pytest.mark.parametrize("failure", ["factory", "vote", "veto"])
def test_slice_agent_commit_failure_restores_the_layout_and_finishes_the_apply(failure):
    """a barrier that cannot be built, raises or vetoes leaves the old layout in
    the store, the plugin re-read and the apply recorded (ref ``actuator.go:181-184`` rollback)."""
    from walkai_nos_amd.controllers.agent.shared import SharedState
    from walkai_nos_amd.controllers.sliceagent.agent import SliceActuator
    from walkai_nos_amd.device.amdsmi import FakeAmdSmi
    from walkai_nos_amd.device.podresources import StaticResourceClient
    from walkai_nos_amd.device.slicing_client import MemorySliceStore, SlicingClient
    from walkai_nos_amd.kube.memory import InMemoryAPIServer
    from walkai_nos_amd.kube.runtime import Request

    class Barrier:
        def vote_all(self, votes):
            if failure == "vote":
                raise RuntimeError("helper died")
            return failure != "veto"

        def close(self):
            pass

    def factory(n):
        if failure == "factory":
            raise FileNotFoundError("nos-gpuhelper not built")
        return Barrier()

    class Plugin:
        restarts = 0

        def restart(self, node, timeout=60.0):
            Plugin.restarts += 1

    smi = FakeAmdSmi(n_gpus=1)
    bdf = smi.list_gpus()[0].bdf
    store = MemorySliceStore()
    old = {0: [Slice(f"{bdf}::s0", "256cu.288gb", list(range(32)))]}
    store.save(old)
    api_ = InMemoryAPIServer()
    node = ko.new_node("n0", {})
    node["metadata"]["annotations"] = {"nos.nebuly.com/spec-gpu-0-32cu.36gb": "2",
                                       "nos.nebuly.com/status-gpu-0-256cu.288gb-free": "1",
                                       "nos.nebuly.com/spec-partitioning-plan": "7"}
    api_.create(node)
    shared = SharedState()
    shared.on_report_done()
    sc = SlicingClient(StaticResourceClient(lambda: [], lambda: []), smi)
    act = SliceActuator(api_, sc, store, shared, "n0", device_plugin=Plugin(), barrier_factory=factory)
    with pytest.raises(GpuError):
        act.reconcile(Request("n0"))
    assert store.load() == old                                 # the old layout is back
    assert Plugin.restarts == 1                                # the plugin re-read it
    assert shared.last_commit and not shared.at_least_one_report_since_last_apply()   # apply recorded
