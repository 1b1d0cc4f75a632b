"""Sliced MI355X GPUs (``models/xcp/slices.py``): mixed per-GPU geometries — SPX + CU-mask slices of
the partition sizes — planned per pod, re-carved without a drain, served by the nos partition
plugin (VERDICT r3 "next round" #1; the MIG behaviour of ref ``pkg/gpu/mig/known_configs.go:41-90``
and ``internal/controllers/migagent/actuator.go:225-229``)."""
import collections

import pytest

from walkai_nos_amd.api import v1alpha1 as api
from walkai_nos_amd.controllers.agent.plan import XcpState, new_xcp_config_plan
from walkai_nos_amd.controllers.partitioner.pod_controller import PackParams, plan_cluster_pack
from walkai_nos_amd.device.amdsmi import FakeAmdSmi
from walkai_nos_amd.device.protos import dp
from walkai_nos_amd.deviceplugin.partitions import PartitionDevicePlugin, PartitionState
from walkai_nos_amd.kube import objects as ko
from walkai_nos_amd.models.annotation import SpecAnnotation
from walkai_nos_amd.models.device import GpuDevice
from walkai_nos_amd.models.partitioned import PartitionedNode
from walkai_nos_amd.models.slicing.cumask import Slice
from walkai_nos_amd.models.xcp import node as xcp_node
from walkai_nos_amd.models.xcp.slices import (GROUP_ROWS, all_slice_geometries, apply_recarve, new_sliced_gpu,
                                              place_slices, recarve, slice_groups)
from walkai_nos_amd.sim.cluster import SimCluster


def _slice(sid, profile, groups):
    return Slice(sid, profile, [GROUP_ROWS * g + i for g in groups for i in range(GROUP_ROWS)], 36 * 10**9 * len(groups))


# -- model ---------------------------------------------------------------------------------
def test_sliced_gpu_allows_mixed_geometries_and_never_drops_used_slices():
    g = new_sliced_gpu("MI355X", 0, used={"dpx_nps1": 1}, free={"cpx_nps1": 4})
    assert g.allows_geometry({"dpx_nps1": 1, "qpx_nps1": 1, "cpx_nps1": 2})
    assert not g.allows_geometry({"dpx_nps1": 2, "cpx_nps1": 1})            # 9 groups
    assert not g.allows_geometry({"cpx_nps2": 1})                           # slices are NPS1
    assert not g.can_apply_geometry({"qpx_nps1": 4})[0]                     # drops the used dpx
    assert len(all_slice_geometries()) == 10 and all(g.allows_geometry(x) for x in all_slice_geometries())
    # a qpx pod re-carves two free cpx slices; the used dpx is untouched
    g.claim("qpx_nps1")
    assert g.used == {"dpx_nps1": 1, "qpx_nps1": 1} and g.free == {"cpx_nps1": 2}
    g.claim("cpx_nps1")
    g.claim("cpx_nps1")
    assert g.room() == 0
    with pytest.raises(ValueError):
        g.claim("cpx_nps1")


def test_sliced_gpu_fill_and_update_geometry_for():
    g = new_sliced_gpu("MI355X", 0, used={"cpx_nps1": 3})
    g.fill()
    assert g.free == {"cpx_nps1": 5}
    assert g.update_geometry_for({"dpx_nps1": 1})
    assert g.free == {"dpx_nps1": 1, "cpx_nps1": 1} and g.used == {"cpx_nps1": 3}
    assert not g.update_geometry_for({"spx_nps1": 1})                       # cannot fit next to used slices


def test_recarve_is_deterministic_and_keeps_used_slices():
    ss = [_slice("b::x0", "cpx_nps1", [0]), _slice("b::x1", "cpx_nps1", [1]), _slice("b::x2", "cpx_nps1", [2]),
          _slice("b::x3", "dpx_nps1", [4, 5, 6, 7])]
    rc = recarve(ss, {"b::x1"}, {"cpx_nps1": 1, "qpx_nps1": 1})
    assert [s.id for s in rc.keep] == ["b::x1"]                              # the used one, not the lowest id
    assert sorted(s.id for s in rc.delete) == ["b::x0", "b::x2", "b::x3"] and rc.create == ["qpx_nps1"]
    assert rc.achievable
    new = apply_recarve(ss, rc, "b", 288 * 10**9)
    assert [s.id for s in new] == ["b::x1", "b::x4"]                        # serials never reused
    assert slice_groups(new[1]) in ([2, 3], [6, 7], [4, 5])                  # buddy-aligned 2-group block
    # a spec the used slices leave no room for: a drain target, only deletions apply
    rc2 = recarve(new, {"b::x1"}, {"cpx_nps1": 1, "spx_nps1": 1})
    assert not rc2.achievable and [s.id for s in rc2.delete] == ["b::x4"]
    assert [s.id for s in apply_recarve(new, rc2, "b", 288 * 10**9)] == ["b::x1"]


def test_placement_prefers_aligned_blocks_in_used_halves():
    existing = [_slice("b::x0", "cpx_nps1", [0])]
    new = place_slices(existing, ["qpx_nps1", "cpx_nps1", "dpx_nps1"], "b", 288 * 10**9)
    groups = {s.profile: slice_groups(s) for s in new}
    assert groups["dpx_nps1"] == [4, 5, 6, 7]        # the empty half stays whole for the dpx
    assert groups["qpx_nps1"] == [2, 3]              # aligned, in the half already in use
    assert groups["cpx_nps1"] == [1]                 # the cpx buddy of the used group
    with pytest.raises(ValueError):
        place_slices(existing + new, ["cpx_nps1"], "b", 288 * 10**9)


def test_node_model_reads_the_layout_label_and_sliced_status():
    n = ko.new_node("n", {api.LABEL_GPU_PARTITIONING: "xcp", api.LABEL_XCP_LAYOUT: "slices",
                          "amd.com/gpu.product-name": "AMD_Instinct_MI355X", "amd.com/gpu.count": "2"})
    n["metadata"]["annotations"] = {
        "nos.nebuly.com/status-gpu-0-dpx_nps1-used": "1", "nos.nebuly.com/status-gpu-0-cpx_nps1-free": "4",
        "nos.nebuly.com/status-gpu-1-cpx_nps1-used": "8", api.ANNOTATION_SLICED_GPUS_STATUS: "0"}
    m = xcp_node.new_node(n)
    assert m.layout == "slices"
    assert m.gpus[0].sliced and not m.gpus[1].sliced          # GPU 1 is still a hardware CPX GPU
    assert m.gpus[0].geometry() == {"dpx_nps1": 1, "cpx_nps1": 4}
    n["metadata"]["labels"][api.LABEL_XCP_LAYOUT] = "bogus"
    assert xcp_node.new_node(n).layout == "partitions"


# -- planner ---------------------------------------------------------------------------------
def _sliced_node(*gpus):
    return PartitionedNode("n", list(gpus), layout="slices", weight=xcp_node.fraction_weight,
                           is_resource=lambda r: r.startswith("amd.com/"), as_resource=lambda p: "amd.com/" + p)


def test_pack_backfills_a_sliced_gpu_without_a_flip():
    g = new_sliced_gpu("MI355X", 0, used={"dpx_nps1": 1}, free={"cpx_nps1": 4})
    changed = plan_cluster_pack({"n": _sliced_node(g)}, [({"qpx_nps1": 1}, 30.0), ({"cpx_nps1": 1}, 10.0)])
    out = changed["n"].gpus[0]
    assert out.sliced and out.target is None
    assert out.geometry() == {"dpx_nps1": 1, "qpx_nps1": 1, "cpx_nps1": 2}


def test_reservation_drains_one_gpu_for_an_old_whole_gpu_pod_and_is_recomputed():
    p = PackParams(slice_reserve_after=900.0)
    g = new_sliced_gpu("MI355X", 0, used={"cpx_nps1": 3}, free={"cpx_nps1": 5})
    # young: the whole-GPU pod waits, the cpx behind it is backfilled
    ch = plan_cluster_pack({"n": _sliced_node(g.clone())}, [({"spx_nps1": 1}, 100.0), ({"cpx_nps1": 1}, 5.0)], params=p)
    assert "n" not in ch or ch["n"].gpus[0].target is None
    # overdue: the GPU's spec becomes "in use + the pod" (no room yet), so the plugin withholds it
    ch = plan_cluster_pack({"n": _sliced_node(g.clone())}, [({"spx_nps1": 1}, 1000.0), ({"cpx_nps1": 1}, 5.0)],
                           params=p)
    out = ch["n"].gpus[0]
    assert out.target == {"cpx_nps1": 3, "spx_nps1": 1} and out.target_sliced
    # the GPU empties: the pod is placed and the reservation disappears
    empty = new_sliced_gpu("MI355X", 0, free={"cpx_nps1": 8})
    empty.target, empty.target_sliced = {"cpx_nps1": 3, "spx_nps1": 1}, True
    ch = plan_cluster_pack({"n": _sliced_node(empty)}, [({"spx_nps1": 1}, 1200.0), ({"cpx_nps1": 1}, 300.0)],
                           params=p)
    out = ch["n"].gpus[0]
    assert out.target is None and out.geometry() == {"spx_nps1": 1}


def test_a_younger_pod_never_drains_a_gpu_an_older_pod_just_took():
    """Regression: the GPU empties, the overdue whole-GPU pod takes it; an overdue cpx pod behind
    it must not turn that GPU into its own reservation (which dropped the placement)."""
    p = PackParams(slice_reserve_after=900.0)
    g = new_sliced_gpu("MI355X", 0, free={"dpx_nps1": 2})
    ch = plan_cluster_pack({"n": _sliced_node(g)}, [({"spx_nps1": 1}, 1100.0), ({"cpx_nps1": 1}, 1000.0)], params=p)
    out = ch["n"].gpus[0]
    assert out.target is None and out.geometry() == {"spx_nps1": 1}


# -- agent plan ------------------------------------------------------------------------------
def test_agent_plan_recarves_a_sliced_gpu_and_slices_an_idle_partitioned_one():
    smi = FakeAmdSmi(n_gpus=2)
    smi.set_compute_partition(1, "CPX")
    m = smi.device_map()
    bdf0 = m.gpus[0].bdf
    slices = {0: [_slice(f"{bdf0}::x0", "dpx_nps1", [0, 1, 2, 3]), _slice(f"{bdf0}::x1", "dpx_nps1", [4, 5, 6, 7])]}
    used = {f"{bdf0}::x0"}
    devs = [GpuDevice("amd.com/dpx_nps1", f"{bdf0}::x0", "used", 0), GpuDevice("amd.com/dpx_nps1", f"{bdf0}::x1", "free", 0)]
    devs += [GpuDevice("amd.com/cpx_nps1", d.device_id, "free", 1) for d in m.partitions_of(1)]
    spec = [SpecAnnotation("dpx_nps1", 0, 1), SpecAnnotation("cpx_nps1", 0, 4),
            SpecAnnotation("qpx_nps1", 1, 1), SpecAnnotation("cpx_nps1", 1, 6)]
    plan = new_xcp_config_plan(XcpState(devs), smi.device_map().modes(), spec, sliced={0, 1}, slices=slices,
                               used_ids=used, gpu_ids={g.index: g.bdf for g in m.gpus},
                               vram_bytes={g.index: g.vram_bytes for g in m.gpus})
    # GPU 0: no flip, the used dpx kept, the free one re-carved into 4 cpx
    assert [(c.gpu_index, c.to_profile) for c in plan.changes] == [(1, "spx_nps1")]
    assert collections.Counter(s.profile for s in plan.slices[0]) == {"dpx_nps1": 1, "cpx_nps1": 4}
    assert f"{bdf0}::x0" in {s.id for s in plan.slices[0]}
    # GPU 1: an idle CPX GPU flips to SPX once and is sliced
    assert collections.Counter(s.profile for s in plan.slices[1]) == {"qpx_nps1": 1, "cpx_nps1": 6}


def test_agent_plan_leaves_a_busy_partitioned_gpu_until_it_drains():
    smi = FakeAmdSmi(n_gpus=1)
    smi.set_compute_partition(0, "CPX")
    m = smi.device_map()
    devs = [GpuDevice("amd.com/cpx_nps1", d.device_id, "used" if d.partition_index == 0 else "free", 0)
            for d in m.partitions_of(0)]
    plan = new_xcp_config_plan(XcpState(devs), m.modes(), [SpecAnnotation("dpx_nps1", 0, 1)], sliced={0},
                               slices={}, used_ids={devs[0].device_id}, gpu_ids={0: m.gpus[0].bdf})
    assert not plan.changes and not plan.slices and plan.blocked


# -- plugin ----------------------------------------------------------------------------------
def _plugin_state(smi, anns, used, store):
    return PartitionState(smi.device_map, lambda: anns, lambda: used, slices=lambda: store)


def test_plugin_serves_slices_and_withholds_only_what_a_recarve_deletes():
    smi = FakeAmdSmi(n_gpus=1)
    bdf = smi.device_map().gpus[0].bdf
    store = {0: [_slice(f"{bdf}::x0", "dpx_nps1", [0, 1, 2, 3]), _slice(f"{bdf}::x1", "cpx_nps1", [4]),
                 _slice(f"{bdf}::x2", "cpx_nps1", [5]), _slice(f"{bdf}::x3", "qpx_nps1", [6, 7])]}
    used = {f"{bdf}::x0", f"{bdf}::x1"}
    anns = {"nos.nebuly.com/status-gpu-0-dpx_nps1-used": "1", "nos.nebuly.com/status-gpu-0-cpx_nps1-used": "1",
            "nos.nebuly.com/status-gpu-0-cpx_nps1-free": "1", "nos.nebuly.com/status-gpu-0-qpx_nps1-free": "1",
            "nos.nebuly.com/spec-gpu-0-dpx_nps1": "1", "nos.nebuly.com/spec-gpu-0-cpx_nps1": "2",
            "nos.nebuly.com/spec-gpu-0-qpx_nps1": "1",
            api.ANNOTATION_SLICED_GPUS_SPEC: "0", api.ANNOTATION_SLICED_GPUS_STATUS: "0"}
    st = _plugin_state(smi, anns, used, store)
    v = st.view()
    assert sorted(v) == ["amd.com/cpx_nps1", "amd.com/dpx_nps1", "amd.com/qpx_nps1"]
    assert all(d.healthy for ds in v.values() for d in ds)
    # the planner re-carves the free qpx into 2 cpx: only the qpx is withheld meanwhile
    anns["nos.nebuly.com/spec-gpu-0-cpx_nps1"] = "4"
    del anns["nos.nebuly.com/spec-gpu-0-qpx_nps1"]
    v = st.view()
    assert [d.healthy for d in v["amd.com/qpx_nps1"]] == [False]
    assert all(d.healthy for d in v["amd.com/cpx_nps1"] + v["amd.com/dpx_nps1"])
    # a drain (a whole-GPU pod waiting): every slice of the GPU is withheld
    anns.update({"nos.nebuly.com/spec-gpu-0-spx_nps1": "1"})
    v = st.view()
    assert not any(d.healthy for ds in v.values() for d in ds)
    # Allocate of a slice: its GPU's render node, its CU mask and HBM budget, the limiter preloaded
    del anns["nos.nebuly.com/spec-gpu-0-spx_nps1"]
    plug = PartitionDevicePlugin("amd.com/cpx_nps1", st, socket_dir="/tmp", shim_path="/opt/nos/shim.so")
    req = dp.AllocateRequest()
    req.container_requests.add(devicesIDs=[f"{bdf}::x2"])
    r = plug.Allocate(req, None).container_responses[0]
    assert r.envs["HSA_CU_MASK"] == "0:160-191" and r.envs["NOS_HBM_LIMIT_BYTES"] == str(36 * 10**9)
    assert r.envs["LD_PRELOAD"] == "/opt/nos/shim.so"
    render = smi.device_map().devices[0].render_minor
    assert [x.host_path for x in r.devices] == ["/dev/kfd", f"/dev/dri/renderD{render}"]


# -- simulated cluster -----------------------------------------------------------------------
def test_one_gpu_serves_cpx_and_dpx_pods_at_once_without_a_flip():
    c = SimCluster(n_nodes=1, gpus_per_node=1, policy="pack", xcp_layout="slices", refresh_interval=5.0)
    c.run(30)
    sn = c.nodes["node-0"]
    c.submit({"amd.com/dpx_nps1": 1}, name="d0")
    for i in range(3):
        c.submit({"amd.com/cpx_nps1": 1}, name=f"c{i}")
    c.run(60)
    assert {ko.name(p) for p in c.running_pods()} == {"d0", "c0", "c1", "c2"}
    assert sn.smi.set_calls == []                                  # no amd-smi switch, ever
    cus = {}
    slices = {s.id: s for s in sn.xcp_slices.load()[0]}
    for (_, name), devs in sn.kubelet.allocations.items():
        cus[name] = set(slices[devs[0][1]].cus)
    assert len(cus["d0"]) == 128 and all(len(cus[f"c{i}"]) == 32 for i in range(3))
    assert not any(cus[a] & cus[b] for a in cus for b in cus if a < b)   # disjoint CU sets
    # one cpx pod leaves; a qpx pod gets the two free groups, re-carved around the running pods
    c.complete("c2")
    c.delete_pod("c2")
    c.submit({"amd.com/qpx_nps1": 1}, name="q0")
    c.run(60)
    assert {ko.name(p) for p in c.running_pods()} == {"d0", "c0", "c1", "q0"}
    assert c.utilization() == pytest.approx(100.0)
    assert c.admission_failures == 0 and sn.smi.set_calls == []


def test_whole_gpu_pod_gets_the_sliced_gpu_through_a_reservation():
    c = SimCluster(n_nodes=1, gpus_per_node=1, policy="pack", xcp_layout="slices", refresh_interval=5.0,
                   pack=PackParams(slice_reserve_after=120.0))
    c.run(30)
    for i in range(4):
        c.submit({"amd.com/cpx_nps1": 1}, name=f"c{i}")
    c.run(60)
    c.submit({"amd.com/spx_nps1": 1}, name="big")
    c.run(200)                                                    # overdue: the GPU is reserved
    c.submit({"amd.com/cpx_nps1": 1}, name="late")
    c.run(60)
    assert {ko.name(p) for p in c.pending_pods()} == {"big", "late"}   # nothing new lands on it
    for i in range(4):
        c.complete(f"c{i}")
        c.delete_pod(f"c{i}")
    c.run(60)
    assert ko.pod_node_name(c.api.get("Pod", "big", "default")) == "node-0"
    assert [ko.name(p) for p in c.running_pods()] == ["big"]
    assert c.nodes["node-0"].smi.set_calls == [] and c.admission_failures == 0
    # the pod the GPU drained for was told so, once (then "late", overdue behind it, reserves it next)
    ev = [e for e in c.api.list("Event") if e.get("reason") == "SlicedGPUReserved"]
    assert [e["involvedObject"]["name"] for e in ev] == ["big", "late"]
    assert "GPU 0 of node node-0 is draining for this pod's spx_nps1 slice: 4 pods still run" in ev[0]["message"]


def test_slices_node_turns_an_idle_hardware_gpu_into_a_sliced_one():
    c = SimCluster(n_nodes=1, gpus_per_node=1, policy="pack", xcp_layout="slices", refresh_interval=5.0)
    sn = c.nodes["node-0"]
    sn.smi.set_compute_partition(0, "CPX")        # left in CPX by a previous layout
    sn.smi.set_calls.clear()
    c.run(30)
    c.submit({"amd.com/dpx_nps1": 1}, name="d0")
    c.submit({"amd.com/cpx_nps1": 1}, name="c0")
    c.run(120)
    assert {ko.name(p) for p in c.running_pods()} == {"d0", "c0"}
    assert [(k, g, m) for k, g, m in sn.smi.set_calls] == [("compute", 0, "SPX")]
    assert ko.annotations(c.api.get("Node", "node-0"))[api.ANNOTATION_SLICED_GPUS_STATUS] == "0"


class _BusyGpuClient:
    """A partition client whose GPUs 0 (CPX, processes on it) and 1 (already SPX) are planned sliced."""

    def __init__(self):
        self.modes = {0: "cpx_nps1", 1: "spx_nps1"}
        self.set_calls = []

    def current_profiles(self):
        return dict(self.modes)

    def gpu_busy(self, gpu):
        return gpu == 0

    def set_profile(self, gpu, profile):
        self.set_calls.append((gpu, profile))
        self.modes[gpu] = profile


def test_actuator_keeps_no_slice_layout_for_a_gpu_whose_spx_flip_was_skipped_as_busy():
    """a skipped (busy) flip to SPX must not save the GPU's new slice layout — the reporter
    would publish a CPX GPU as sliced and the plugin would stop withholding it."""
    from walkai_nos_amd.controllers.agent.actuator import Actuator
    from walkai_nos_amd.controllers.agent.plan import ModeChange, XcpConfigPlan
    from walkai_nos_amd.controllers.agent.shared import SharedState
    from walkai_nos_amd.device.slicing_client import MemorySliceStore
    from walkai_nos_amd.kube.memory import InMemoryAPIServer
    store = MemorySliceStore()
    pc = _BusyGpuClient()
    act = Actuator(InMemoryAPIServer(), pc, SharedState(), "node-a", journal=False, slice_store=store)
    act._votes = lambda applied: [True]
    plan = XcpConfigPlan(changes=[ModeChange(0, "cpx_nps1", "spx_nps1")],
                         slices={0: [_slice("g0::x0", "dpx_nps1", [0, 1, 2, 3])],
                                 1: [_slice("g1::x0", "cpx_nps1", [0])]})
    err = act.apply(plan, "p1")
    assert err is not None and pc.set_calls == []                    # busy: not flipped, retried later
    assert set(store.load()) == {1}                                  # GPU 1 (SPX) re-carved; GPU 0 untouched
    assert [s.id for s in store.load()[1]] == ["g1::x0"]


def test_default_layout_of_unlabelled_nodes_comes_from_the_partitioner_config():
    """the chart default is the layout the bench measures (slices)."""
    from walkai_nos_amd.api.config import GpuPartitionerConfig
    cfg = GpuPartitionerConfig()
    assert cfg.defaultXcpLayout == "slices"
    cfg.defaultXcpLayout = "mig"
    with pytest.raises(ValueError):
        cfg.validate()
    n = ko.new_node("n", {api.LABEL_GPU_PARTITIONING: "xcp", "amd.com/gpu.product-name": "AMD_Instinct_MI355X",
                          "amd.com/gpu.count": "1"})
    assert xcp_node.get_layout(n) == "partitions"          # library default: unchanged
    assert xcp_node.get_layout(n, "slices") == "slices"    # the planner's default, passed explicitly
    n["metadata"]["labels"][api.LABEL_XCP_LAYOUT] = "partitions"
    assert xcp_node.get_layout(n, "slices") == "partitions"  # the label wins
    import os

    import yaml
    vals = yaml.safe_load(open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                            "helm-charts", "nos", "values.yaml")))
    import bench as _bench  # noqa: F401  (bench.py's --layout default, read from its parser)
    import inspect
    src = inspect.getsource(_bench.main)
    assert 'ap.add_argument("--layout", default="slices"' in src
    assert vals["gpuPartitioner"]["defaultXcpLayout"] == "slices"


def test_a_held_reservation_lapses_on_bigger_clusters():
    """``slice_reserve_hold_max_gpus``: a drain in progress keeps its target until a pod of its profile
    is placed while the cluster has at most that many sliced GPUs (default 2); with more, it is
    re-decided each pass (here: the whole-GPU pod is not overdue, so the draining GPU takes the small
    pod again). 0 holds at any cluster size."""
    assert PackParams().slice_reserve_hold_max_gpus == 2
    p = PackParams(slice_reserve_after=900.0)

    def draining():
        g = new_sliced_gpu("MI355X", 0, used={"cpx_nps1": 3})
        g.target, g.target_sliced = {"cpx_nps1": 3, "spx_nps1": 1}, True
        return g

    pending = [({"spx_nps1": 1}, 100.0), ({"cpx_nps1": 1}, 5.0)]
    ch = plan_cluster_pack({"n": _sliced_node(draining())}, list(pending), params=p)
    out = (ch.get("n") or _sliced_node(draining())).gpus[0]
    assert out.target == {"cpx_nps1": 3, "spx_nps1": 1}          # held on one GPU
    full = [new_sliced_gpu("MI355X", i, used={"cpx_nps1": 8}) for i in (1, 2)]
    ch = plan_cluster_pack({"n": _sliced_node(draining(), *full)}, list(pending), params=p)
    out = ch["n"].gpus[0]
    assert out.target is None and out.used.get("cpx_nps1", 0) + out.free.get("cpx_nps1", 0) >= 4
    p0 = PackParams(slice_reserve_after=900.0, slice_reserve_hold_max_gpus=0)
    ch = plan_cluster_pack({"n": _sliced_node(draining(), *full)}, list(pending), params=p0)
    out = (ch.get("n") or _sliced_node(draining(), *full)).gpus[0]
    assert out.target == {"cpx_nps1": 3, "spx_nps1": 1}          # 0: held at any cluster size


def test_free_drain_reserves_room_no_waiting_pod_fits():
    """Every waiting pod is bigger than the GPU's unused room (one group): that room idles whatever
    the planner does, so the oldest waiting pod reserves the GPU without waiting for its threshold."""
    def run(free_drain):
        g = new_sliced_gpu("MI355X", 0, used={"cpx_nps1": 7}, free={"cpx_nps1": 1})
        p = PackParams(slice_reserve_after=900.0, slice_free_drain=free_drain)
        ch = plan_cluster_pack({"n": _sliced_node(g)}, [({"dpx_nps1": 1}, 10.0)], params=p)
        return ch["n"].gpus[0].target if "n" in ch else None
    assert run(True) == {"cpx_nps1": 7, "dpx_nps1": 1}
    assert run(False) is None


def test_free_drain_is_held_on_small_clusters_and_lapses_on_bigger_ones():
    """a free drain made on a one-GPU cluster is held like any reservation until a pod of
    its profile is placed (a smaller pod arriving meanwhile waits — letting it lapse there measured
    worse, sliced.py 3b); on a cluster of more sliced GPUs than ``slice_reserve_hold_max_gpus`` it is
    re-decided each pass and lapses once the room fits a waiting pod."""
    p = PackParams(slice_reserve_after=900.0)
    g = new_sliced_gpu("MI355X", 0, used={"cpx_nps1": 7}, free={"cpx_nps1": 1})
    ch = plan_cluster_pack({"n": _sliced_node(g)}, [({"dpx_nps1": 1}, 10.0)], params=p)
    assert ch["n"].gpus[0].target == {"cpx_nps1": 7, "dpx_nps1": 1}     # the free drain

    def held(i=0):
        h = new_sliced_gpu("MI355X", i, used={"cpx_nps1": 7})
        h.target, h.target_sliced = {"cpx_nps1": 7, "dpx_nps1": 1}, True
        return h
    pending = [({"dpx_nps1": 1}, 20.0), ({"cpx_nps1": 1}, 1.0)]
    ch = plan_cluster_pack({"n": _sliced_node(held())}, list(pending), params=p)
    out = (ch.get("n") or _sliced_node(held())).gpus[0]
    assert out.target == {"cpx_nps1": 7, "dpx_nps1": 1}                  # held: the 1/8 pod waits
    full = [new_sliced_gpu("MI355X", i, used={"cpx_nps1": 8}) for i in (1, 2)]
    ch = plan_cluster_pack({"n": _sliced_node(held(), *full)}, list(pending), params=p)
    out = ch["n"].gpus[0]
    assert out.target is None and out.used.get("cpx_nps1", 0) + out.free.get("cpx_nps1", 0) == 8


def test_reservation_threshold_in_learned_lifetimes():
    from walkai_nos_amd.controllers.partitioner.lifetimes import LifetimeModel
    life = LifetimeModel(min_samples=1)
    for _ in range(8):
        life.observe(100.0)
    p = PackParams(slice_reserve_after=900.0, slice_reserve_lifetimes=3.75, slice_reserve_backlog=0.0,
                   slice_free_drain=False)

    def target(age, learned):
        g = new_sliced_gpu("MI355X", 0, used={"cpx_nps1": 3}, free={"cpx_nps1": 5})
        ch = plan_cluster_pack({"n": _sliced_node(g)}, [({"spx_nps1": 1}, age)], params=p,
                               pods_of=lambda n, i: [(1, 50.0)] * 3, life=life if learned else None)
        return ch["n"].gpus[0].target if "n" in ch else None
    assert target(400.0, True) is not None        # 3.75 x the 100 s median = 375 s
    assert target(300.0, True) is None
    assert target(400.0, False) is None           # not learned: the 900 s constant


def test_no_reservation_that_only_its_own_profile_blocks():
    """A whole-GPU pod never reserves a GPU another whole-GPU pod runs on: nothing idles while that
    pod runs and its slice goes to the next whole-GPU pod anyway, but the plugin would withhold the
    slice in use, and kube-scheduler (its request counted, the device not) would stop seeing the
    node's other free whole-GPU slices. With learned lifetimes that GPU is the cheapest drain (no
    group idles), so it was the one picked; a held reservation of it lapses too."""
    from walkai_nos_amd.controllers.partitioner.lifetimes import LifetimeModel
    life = LifetimeModel(min_samples=1)
    for _ in range(8):
        life.observe(240.0)
    p = PackParams(slice_reserve_after=900.0, slice_reserve_lifetimes=0.0, slice_free_drain=False)
    pods = {0: [(8, 200.0)], 1: [(1, 10.0)] * 3}
    pending = [({"spx_nps1": 1}, 1000.0)]

    def node(held=False):
        g0 = new_sliced_gpu("MI355X", 0, used={"spx_nps1": 1})
        if held:
            g0.target, g0.target_sliced = {"spx_nps1": 2}, True
        return _sliced_node(g0, new_sliced_gpu("MI355X", 1, used={"cpx_nps1": 3}, free={"cpx_nps1": 5}))

    for held in (False, True):
        ch = plan_cluster_pack({"n": node(held)}, list(pending), params=p, pods_of=lambda n, g: pods[g], life=life)
        targets = [g.target for g in ch["n"].gpus]
        assert targets[0] is None and targets[1] == {"cpx_nps1": 3, "spx_nps1": 1}
    # a half-GPU pod may still reserve the other half of a GPU a half-GPU pod runs on
    g = new_sliced_gpu("MI355X", 0, used={"dpx_nps1": 1, "cpx_nps1": 2}, free={"cpx_nps1": 2})
    ch = plan_cluster_pack({"n": _sliced_node(g)}, [({"dpx_nps1": 1}, 1000.0)], params=p)
    assert ch["n"].gpus[0].target == {"dpx_nps1": 2, "cpx_nps1": 2}


def test_free_drain_wait_grows_with_the_gpus_up_to_a_cap():
    """The wait before a free drain is ``sliceFreeDrainAfterLifetimes`` per other sliced GPU (with more
    GPUs one empties on its own sooner), capped at ``sliceFreeDrainCapLifetimes``: eight GPUs whose
    one free group no waiting pod fits idle 1/8 of the cluster until a drain starts."""
    from walkai_nos_amd.controllers.partitioner.lifetimes import LifetimeModel
    life = LifetimeModel(min_samples=1)
    for _ in range(8):
        life.observe(100.0)

    def drains(cap, age):
        gpus = [new_sliced_gpu("MI355X", i, used={"cpx_nps1": 7}, free={"cpx_nps1": 1}) for i in range(8)]
        p = PackParams(slice_reserve_after=900.0, slice_reserve_lifetimes=0.0, slice_free_drain_cap=cap)
        ch = plan_cluster_pack({"n": _sliced_node(*gpus)}, [({"dpx_nps1": 1}, age)], params=p,
                               pods_of=lambda n, g: [(1, 50.0)] * 7, life=life)
        return sum(1 for g in ch["n"].gpus if g.target is not None) if "n" in ch else 0
    assert drains(0.75, 80.0) == 1          # 0.5 x 7 = 3.5 lifetimes, capped at 0.75 = 75 s
    assert drains(0.75, 70.0) == 0
    assert drains(0.0, 80.0) == 0           # uncapped: 350 s
    assert drains(0.0, 360.0) == 1



def test_a_pod_of_several_slices_may_reserve_a_gpu_its_profile_fills():
    """Two cpx slices for one pod on a GPU full of one-slice cpx pods: each slice those pods free goes
    to a one-slice pod unless the GPU is reserved, so the reservation is kept."""
    p = PackParams(slice_reserve_after=900.0, slice_free_drain=False)
    g = new_sliced_gpu("MI355X", 0, used={"cpx_nps1": 8})
    ch = plan_cluster_pack({"n": _sliced_node(g)}, [({"cpx_nps1": 2}, 1000.0)], params=p)
    assert ch["n"].gpus[0].target == {"cpx_nps1": 10}


def test_reservation_threshold_stretches_up_to_four_times_under_backlog():
    """``sliceReserveStretch`` (4): with a long queue the threshold grows with the backlog (GPUs of
    waiting work per sliced GPU over ``sliceReserveBacklog``), at most 4x — so under sustained
    overload drains stay rare."""
    assert PackParams().slice_reserve_stretch == 4.0
    p = PackParams(slice_reserve_after=100.0, slice_reserve_backlog=1.0, slice_free_drain=False)

    def target(age):
        g = new_sliced_gpu("MI355X", 0, used={"cpx_nps1": 8})
        backlog = [({"cpx_nps1": 1}, 1.0)] * 80        # 10 GPUs of waiting work on one GPU
        ch = plan_cluster_pack({"n": _sliced_node(g)}, [({"spx_nps1": 1}, age)] + backlog, params=p)
        return ch["n"].gpus[0].target if "n" in ch else None
    assert target(350.0) is None                      # under 4 x 100 s
    assert target(410.0) == {"cpx_nps1": 8, "spx_nps1": 1}
