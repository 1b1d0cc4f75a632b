"""Cluster-side partitioner: pod controller (B1), node initialiser (B2), spec writer (C4)."""
import pytest

from walkai_nos_amd import constant
from walkai_nos_amd.api import v1alpha1 as api
from walkai_nos_amd.controllers.partitioner.node_controller import NodeController
from walkai_nos_amd.controllers.partitioner.pod_controller import PodController, plan_cluster, plan_cluster_fifo
from walkai_nos_amd.kube import objects as ko
from walkai_nos_amd.kube.memory import InMemoryAPIServer
from walkai_nos_amd.kube.runtime import Request, SimClock
from walkai_nos_amd.models.xcp import node as xcp_node
from walkai_nos_amd.partitioning.planner import (NodeInitializer, Partitioner, build_node_partitioning, new_plan_id,
                                                 spec_annotations)


def xnode(name="n0", gpus=2, anns=None):
    return ko.new_node(name, {api.LABEL_GPU_PARTITIONING: "xcp", constant.LABEL_AMD_GPU_PRODUCT: "AMD_Instinct_MI355X",
                              constant.LABEL_AMD_GPU_COUNT: str(gpus)}, anns or {})


def unschedulable_pod(name, req, ns="default"):
    p = ko.new_pod(name, ns, requests=req)
    ko.set_condition(p, "PodScheduled", "False", "Unschedulable")
    return p


def test_plan_ids_are_unique_and_increasing():
    clock = SimClock(5)
    a, b = new_plan_id(clock), new_plan_id(clock)
    assert int(b) > int(a)


def test_partitioner_replaces_spec_family_and_sets_plan():
    api_ = InMemoryAPIServer()
    api_.create(xnode(anns={"nos.nebuly.com/spec-gpu-5-cpx_nps1": "8", "keep": "me"}))
    model = xcp_node.new_node(api_.get("Node", "n0"))
    for g in model.gpus:
        g.init_geometry()
    Partitioner(api_).apply_partitioning(api_.get("Node", "n0"), "99", build_node_partitioning(model))
    a = ko.annotations(api_.get("Node", "n0"))
    assert a["nos.nebuly.com/spec-gpu-0-spx_nps1"] == "1" and a["nos.nebuly.com/spec-gpu-1-spx_nps1"] == "1"
    assert "nos.nebuly.com/spec-gpu-5-cpx_nps1" not in a and a["keep"] == "me"
    assert a[api.ANNOTATION_PARTITIONING_PLAN] == "99"


def test_node_controller_initialises_once_and_requires_labels():
    api_ = InMemoryAPIServer()
    api_.create(xnode())
    nc = NodeController(api_, NodeInitializer(api_))
    nc.reconcile(Request("n0"))
    n = api_.get("Node", "n0")
    assert NodeController.is_initialized(n)
    plan = ko.annotations(n)[api.ANNOTATION_PARTITIONING_PLAN]
    nc.reconcile(Request("n0"))
    assert ko.annotations(api_.get("Node", "n0"))[api.ANNOTATION_PARTITIONING_PLAN] == plan
    bare = ko.new_node("bare", {api.LABEL_GPU_PARTITIONING: "xcp"})
    api_.create(bare)
    nc.reconcile(Request("bare"))
    assert api.ANNOTATION_PARTITIONING_PLAN not in ko.annotations(api_.get("Node", "bare"))


def _settled(api_, status):
    anns = dict(status)
    anns[api.ANNOTATION_PARTITIONING_PLAN] = "1"
    anns[api.ANNOTATION_REPORTED_PARTITIONING_PLAN] = "1"
    api_.patch("Node", "n0", {"metadata": {"annotations": anns}})


def test_pod_controller_ignores_schedulable_or_unrelated_pods():
    api_ = InMemoryAPIServer()
    api_.create(xnode())
    pc = PodController(api_)
    api_.create(ko.new_pod("plain", requests={"amd.com/cpx_nps1": 1}))  # not marked unschedulable
    api_.create(unschedulable_pod("cpu-only", {"cpu": "1"}))
    assert pc.map_pod(api_.get("Pod", "plain", "default")) == []
    assert pc.map_pod(api_.get("Pod", "cpu-only", "default")) == []
    pc.reconcile(Request("plain", "default"))
    pc.reconcile(Request("cpu-only", "default"))
    assert pc.plans_written == 0


def test_pod_controller_flips_free_gpu_and_skips_when_free_capacity_exists():
    api_ = InMemoryAPIServer()
    api_.create(xnode())
    _settled(api_, {"nos.nebuly.com/status-gpu-0-spx_nps1-free": "1", "nos.nebuly.com/status-gpu-1-spx_nps1-used": "1"})
    pc = PodController(api_)
    api_.create(unschedulable_pod("p", {"amd.com/cpx_nps1": 1}))
    pc.reconcile(pc.plan_key)
    a = ko.annotations(api_.get("Node", "n0"))
    assert a["nos.nebuly.com/spec-gpu-0-cpx_nps1"] == "8" and a["nos.nebuly.com/spec-gpu-1-spx_nps1"] == "1"
    assert pc.plans_written == 1
    # a plan is in flight (spec plan != status plan): no re-planning, capacity counted as incoming
    api_.create(unschedulable_pod("p2", {"amd.com/cpx_nps1": 1}))
    pc.reconcile(Request("p2", "default"))
    assert pc.plans_written == 1


def test_q1_fix_repartitions_when_every_partition_of_the_profile_is_used():
    # reference bug Q1: "profile exists somewhere (free or used)" suppressed repartitioning
    api_ = InMemoryAPIServer()
    api_.create(xnode())
    _settled(api_, {"nos.nebuly.com/status-gpu-0-cpx_nps1-used": "8", "nos.nebuly.com/status-gpu-1-spx_nps1-free": "1"})
    pc = PodController(api_)
    api_.create(unschedulable_pod("p", {"amd.com/cpx_nps1": 1}))
    pc.reconcile(pc.plan_key)
    a = ko.annotations(api_.get("Node", "n0"))
    assert a["nos.nebuly.com/spec-gpu-1-cpx_nps1"] == "8"


def test_q14_requeue_when_nothing_can_help():
    api_ = InMemoryAPIServer()
    api_.create(xnode(gpus=1))
    _settled(api_, {"nos.nebuly.com/status-gpu-0-cpx_nps1-used": "8"})
    pc = PodController(api_, retry_after=7)
    api_.create(unschedulable_pod("p", {"amd.com/spx_nps1": 1}))
    res = pc.reconcile(pc.plan_key)
    assert res.requeue_after == 7 and pc.plans_written == 0


def test_batch_window_defers_planning():
    api_ = InMemoryAPIServer()
    clock = SimClock(0)
    api_.create(xnode())
    pc = PodController(api_, clock=clock, batch_timeout=10, batch_idle=3)
    api_.create(unschedulable_pod("p", {"amd.com/cpx_nps1": 1}))
    res = pc.reconcile(pc.plan_key)
    assert 0 < res.requeue_after <= 3 and pc.plans_written == 0
    clock.advance(3)
    pc.reconcile(pc.plan_key)
    assert pc.plans_written == 1


def test_plan_cluster_scores_nodes_and_fifo_is_head_of_line():
    api_ = InMemoryAPIServer()
    for n in ("a", "b"):
        api_.create(xnode(n, gpus=1, anns={"nos.nebuly.com/status-gpu-0-spx_nps1-free": "1"}))
    models = {n: xcp_node.new_node(api_.get("Node", n)) for n in ("a", "b")}
    changed = plan_cluster(models, {"cpx_nps1": 9})
    assert set(changed) == {"a", "b"}  # 8 + 1 partitions need both GPUs
    # head pod reserves a free SPX GPU; the 1/8 pod behind it flips the *other* GPU
    changed = plan_cluster_fifo(models, [{"spx_nps1": 1}, {"cpx_nps1": 1}])
    assert list(changed) == ["b"] and changed["b"].gpus[0].geometry() == {"cpx_nps1": 8}
    # two SPX pods take both GPUs: a 1/8 pod cannot be helped
    assert plan_cluster_fifo(models, [{"spx_nps1": 1}, {"spx_nps1": 1}, {"cpx_nps1": 1}]) == {}
    # one GPU flipped to CPX serves both 1/8 pods, the other stays SPX for the whole-GPU pod
    changed = plan_cluster_fifo(models, [{"cpx_nps1": 1}, {"cpx_nps1": 1}, {"spx_nps1": 1}])
    assert len(changed) == 1
    (name, model), = changed.items()
    assert model.gpus[0].geometry() == {"cpx_nps1": 8}


def test_spec_annotations_sum_per_gpu_profile():
    from walkai_nos_amd.partitioning.state import GPUPartitioning, NodePartitioning
    np_ = NodePartitioning([GPUPartitioning(0, {"amd.com/cpx_nps1": 8}), GPUPartitioning(1, {"amd.com/gpu-8cu.4gb": 2})])
    assert spec_annotations(np_) == {"nos.nebuly.com/spec-gpu-0-cpx_nps1": "8", "nos.nebuly.com/spec-gpu-1-8cu.4gb": "2"}


def test_simulate_policy_picks_the_plan_that_schedules_most_pods():
    from walkai_nos_amd.controllers.partitioner.pod_controller import (plan_cluster_simulate, planned_state,
                                                                       simulate_schedule)
    api_ = InMemoryAPIServer()
    api_.create(xnode("a", gpus=1, anns={"nos.nebuly.com/status-gpu-0-spx_nps1-free": "1"}))
    models = {"a": xcp_node.new_node(api_.get("Node", "a"))}
    pending = [{"spx_nps1": 1}] + [{"cpx_nps1": 1}] * 6
    # FIFO serves the head-of-line whole-GPU pod (1 pod scheduled) ...
    fifo = plan_cluster_fifo(models, pending)
    assert simulate_schedule(planned_state(models, fifo), pending)[0] == 1
    # ... the simulation planner picks the CPX layout that schedules 6 of them
    sim = plan_cluster_simulate(models, pending)
    assert sim["a"].gpus[0].geometry() == {"cpx_nps1": 8}
    assert simulate_schedule(planned_state(models, sim), pending) == (6, 0.75)


def test_simulate_policy_end_to_end_on_the_in_memory_cluster():
    from walkai_nos_amd.sim.cluster import SimCluster
    c = SimCluster(n_nodes=1, gpus_per_node=2, policy="simulate")
    c.run(30)
    for i in range(10):
        c.submit({"amd.com/cpx_nps1": 1}, name=f"c{i}")
    c.submit({"amd.com/dpx_nps1": 1}, name="d0")
    c.run(120)
    # partitions are homogeneous per GPU: 10 x 1/8 + 1 x 1/2 cannot all fit on 2 GPUs; the
    # simulation keeps the layout that runs the most pods (both GPUs CPX)
    assert len(c.running_pods()) == 10 and [ko.name(p) for p in c.pending_pods()] == ["d0"]


def test_read_only_plan_pass_is_reused_until_the_api_changes():
    """A requeued plan key on an unchanged cluster reuses the last read-only answer; any write
    (here: the blocking pods finish) makes the next pass plan again."""
    import walkai_nos_amd.controllers.partitioner.pod_controller as pcm
    api_ = InMemoryAPIServer()
    api_.create(xnode(gpus=1))
    _settled(api_, {"nos.nebuly.com/status-gpu-0-cpx_nps1-used": "8"})
    pc = PodController(api_, retry_after=7)
    api_.create(unschedulable_pod("p", {"amd.com/spx_nps1": 1}))
    calls = []
    orig = pcm.plan_cluster_fifo
    pcm.plan_cluster_fifo = lambda *a, **k: calls.append(1) or orig(*a, **k)
    try:
        assert pc.reconcile(pc.plan_key).requeue_after == 7
        assert pc.reconcile(pc.plan_key).requeue_after == 7
        assert len(calls) == 1 and pc.plans_written == 0
        _settled(api_, {"nos.nebuly.com/status-gpu-0-cpx_nps1-used": "0",
                        "nos.nebuly.com/status-gpu-0-cpx_nps1-free": "8"})
        pc.reconcile(pc.plan_key)
        assert len(calls) == 2 and pc.plans_written == 1
    finally:
        pcm.plan_cluster_fifo = orig


def test_pod_controller_plan_memo_skips_replanning_until_the_api_changes():
    from walkai_nos_amd.controllers.partitioner import pod_controller as pcm
    from walkai_nos_amd.sim.cluster import SimCluster
    c = SimCluster(n_nodes=1, gpus_per_node=1)
    c.run(30)
    ctl = c.pod_controllers[0] if isinstance(c.pod_controllers, list) else c.pod_controllers
    calls = []
    orig = pcm.plan_cluster_fifo

    def counting(*a, **k):
        calls.append(1)
        return orig(*a, **k)
    pcm.plan_cluster_fifo = counting
    try:
        # an unsatisfiable pod keeps the plan key requeued with nothing to change
        c.submit({"amd.com/spx_nps1": 2}, name="big")
        c.run(5)
        n = len(calls)
        assert n >= 1
        for _ in range(5):
            ctl.reconcile(ctl.plan_key)
        assert len(calls) == n                       # same revision: memoised answer
        c.api.patch("Node", "node-0", {"metadata": {"annotations": {"touch": "1"}}})
        ctl.reconcile(ctl.plan_key)
        assert len(calls) == n + 1                   # a node write forces a re-plan
    finally:
        pcm.plan_cluster_fifo = orig


def test_packing_config_maps_to_pack_params():
    from walkai_nos_amd.api.config import GpuPartitionerConfig
    cfg = GpuPartitionerConfig(packing={"minFill": 0.25, "drainGainAfterSeconds": 120, "spxReserve": False})
    cfg.validate()
    p = cfg.pack_params()
    assert (p.min_fill, p.drain_gain_after, p.spx_reserve) == (0.25, 120.0, False)
    assert p.drain_gain == 0.3 and p.min_stint == 120.0  # untouched knobs keep their defaults
    with pytest.raises(ValueError):
        GpuPartitionerConfig(packing={"minFil": 0.2}).validate()
    with pytest.raises(ValueError):
        GpuPartitionerConfig(packing={"drainGain": -1}).validate()


def test_every_packing_key_names_a_pack_param():
    """Each ``packing`` key of the config (and so of the chart) maps to a ``PackParams`` field, and a
    value set through it reaches the planner (booleans stay booleans)."""
    import dataclasses

    from walkai_nos_amd.api.config import GpuPartitionerConfig
    from walkai_nos_amd.controllers.partitioner.pod_controller import PackParams
    fields = {f.name for f in dataclasses.fields(PackParams)}
    assert set(GpuPartitionerConfig.PACKING_KEYS.values()) <= fields
    for key, name in GpuPartitionerConfig.PACKING_KEYS.items():
        boolean = key in GpuPartitionerConfig.BOOL_PACKING_KEYS
        value = False if boolean else 3.0
        cfg = GpuPartitionerConfig(packing={key: value})
        cfg.validate()
        assert getattr(cfg.pack_params(), name) == value, key
    p = GpuPartitionerConfig(packing={"sliceStrandWeight": 0, "sliceFreeDrainCapLifetimes": 0}).pack_params()
    assert (p.slice_strand_weight, p.slice_free_drain_cap) == (0.0, 0.0)


def test_pack_gain_drain_rotates_an_underused_gpu():
    # one GPU in CPX mode holding a single 1/8 pod, SPX pods waiting past drain_gain_after: the GPU
    # is drained for SPX (target set, no new CPX pods), which it would never be by the backlog rule
    from walkai_nos_amd.controllers.partitioner.pod_controller import PackParams, new_node_model, plan_cluster_pack
    node = xnode("n0", gpus=1, anns={"nos.nebuly.com/status-gpu-0-cpx_nps1-used": "1",
                                     "nos.nebuly.com/status-gpu-0-cpx_nps1-free": "7"})
    models = {"n0": new_node_model("xcp", node)}
    pending = [({"spx_nps1": 1}, 700.0)]
    changed = plan_cluster_pack(models, pending, params=PackParams())
    assert changed["n0"].gpus[0].target == {"spx_nps1": 1}
    assert plan_cluster_pack(models, pending, params=PackParams(drain_gain_after=0, unserved_after=0)) == {}
    assert plan_cluster_pack(models, [({"spx_nps1": 1}, 100.0)], params=PackParams()) == {}


def test_pack_fairness_drains_a_full_gpu_for_an_unserved_profile_after_its_stint():
    # one GPU in CPX mode with all 8 partitions in use: the gain rule never drains it (the SPX queue
    # would fill it no better), but no GPU serves SPX at all — after unserved_after x 1 GPU of
    # waiting, and once the GPU has held CPX for min_stint, it is drained for SPX
    from walkai_nos_amd.controllers.partitioner.pod_controller import PackParams, new_node_model, plan_cluster_pack
    node = xnode("n0", gpus=1, anns={"nos.nebuly.com/status-gpu-0-cpx_nps1-used": "8"})
    models = {"n0": new_node_model("xcp", node)}
    waited = [({"spx_nps1": 1}, 400.0)]
    p = PackParams()
    assert plan_cluster_pack(models, [({"spx_nps1": 1}, 200.0)], params=p) == {}          # not long enough
    assert plan_cluster_pack(models, waited, params=p, mode_age=lambda n, g: 60.0) == {}  # stint not over
    changed = plan_cluster_pack(models, waited, params=p, mode_age=lambda n, g: 600.0)
    assert changed["n0"].gpus[0].target == {"spx_nps1": 1}
    assert plan_cluster_pack(models, waited, params=PackParams(unserved_after=0), mode_age=lambda n, g: 600.0) == {}


def test_multi_node_cluster_bench_tracks_flips_per_node():
    # the bench's control plane + outage model on a 3-node cluster (nos-simulate --nodes): every
    # flip darkens its own (node, GPU); the planner keeps the cluster allocated
    from walkai_nos_amd.bench_core import BenchConfig, NodeBench
    nb = NodeBench(BenchConfig(gpus=2, nodes=3, flip_cost_s=1.0, quantum_s=0.5, seed=3), gpu_data_plane=False)
    assert len(nb.cluster.nodes) == 3
    for _ in range(40):
        nb.control_step()
        assert all(isinstance(k, tuple) and k[0] in nb.cluster.nodes for k in nb.outage)
        nb.end_step()
    assert nb.flips > 0 and max(nb.util_samples) > 50.0
    assert nb.gpu_quanta == 40 * 6


def test_pack_reserve_break_flips_a_reserved_idle_spx_gpu_for_a_full_queue():
    # GPU 0 serves a whole-GPU pod, GPU 1 is an idle SPX GPU held as the whole-GPU reserve
    # (spx_demand 2): a DPX queue of 1.5 GPUs leaves it reserved, 2 GPUs' worth takes it
    from walkai_nos_amd.controllers.partitioner.pod_controller import PackParams, new_node_model, plan_cluster_pack
    node = xnode("n0", gpus=2, anns={"nos.nebuly.com/status-gpu-0-spx_nps1-used": "1",
                                     "nos.nebuly.com/status-gpu-1-spx_nps1-free": "1"})
    models = {"n0": new_node_model("xcp", node)}
    three = [({"dpx_nps1": 1}, 60.0)] * 3
    assert plan_cluster_pack(models, three, params=PackParams(), spx_demand=2.0) == {}
    changed = plan_cluster_pack(models, three + [({"dpx_nps1": 1}, 60.0)], params=PackParams(), spx_demand=2.0)
    assert changed["n0"].gpus[1].geometry() == {"dpx_nps1": 2}
    assert changed["n0"].gpus[0].geometry() == {"spx_nps1": 1}  # the busy GPU is never touched
    # without a reserve the idle GPU flips for a half-GPU queue already (min_fill)
    assert "n0" in plan_cluster_pack(models, three[:1], params=PackParams(), spx_demand=0.0)


def test_pack_switches_an_idle_node_to_another_memory_partition_mode_and_back():
    """``*_nps2`` pods on an NPS1 node: the memory mode is node-wide, so the planner switches a
    whole idle node (``spec-memory-partition``) with the waiting profile's mode on as many GPUs as
    the demand starts and the fewest-partition NPS2 geometry (DPX: SPX needs NPS1) on the rest; a
    whole-GPU NPS1 pod arriving meanwhile waits, and the node switches back once it is idle."""
    from walkai_nos_amd.sim.cluster import SimCluster
    c = SimCluster(n_nodes=1, gpus_per_node=2, policy="pack")
    c.run(30)
    for i in range(5):
        c.submit({"amd.com/cpx_nps2": 1}, name=f"m{i}")
    c.run(120)
    anns = ko.annotations(c.api.get("Node", "node-0"))
    assert anns["nos.nebuly.com/spec-memory-partition"] == "nps2"
    assert anns["nos.nebuly.com/status-memory-partition"] == "nps2"
    assert anns["nos.nebuly.com/spec-gpu-0-cpx_nps2"] == "8" and anns["nos.nebuly.com/spec-gpu-1-dpx_nps2"] == "2"
    assert all(ko.pod_phase(c.api.get("Pod", f"m{i}", "default")) == "Running" for i in range(5))
    c.submit({"amd.com/spx_nps1": 1}, name="w")
    c.run(200)
    assert ko.pod_phase(c.api.get("Pod", "w", "default")) == "Pending"
    for i in range(5):
        c.complete(f"m{i}")
        c.delete_pod(f"m{i}")
    c.run(600)
    anns = ko.annotations(c.api.get("Node", "node-0"))
    assert anns["nos.nebuly.com/status-memory-partition"] == "nps1"
    assert ko.pod_phase(c.api.get("Pod", "w", "default")) == "Running"


def test_pack_drains_a_whole_node_for_an_unserved_memory_partition_mode():
    """No idle node: once an NPS2 pod has waited unserved_after x GPUs, the least-used node is
    drained as a whole — every GPU's spec changes at once (idle ones included), none takes new
    pods — and the agent switches the node when its last pod leaves."""
    from walkai_nos_amd.controllers.partitioner.pod_controller import PackParams, plan_cluster_pack
    from walkai_nos_amd.models.xcp import node as xn
    n = ko.new_node("node-0", {"nos.nebuly.com/gpu-partitioning": "xcp",
                               "amd.com/gpu.product-name": "AMD_Instinct_MI355X", "amd.com/gpu.count": "2"},
                    {"nos.nebuly.com/status-gpu-0-spx_nps1-used": "1", "nos.nebuly.com/status-gpu-1-spx_nps1-free": "1",
                     "nos.nebuly.com/status-memory-partition": "nps1"})
    m = xn.new_node(n)
    p = PackParams(unserved_after=300)
    assert plan_cluster_pack({"node-0": m}, [({"cpx_nps2": 1}, 500.0)], None, p) == {}   # not yet: 500 < 300 x 2
    ch = plan_cluster_pack({"node-0": m}, [({"cpx_nps2": 1}, 700.0)], None, p)
    out = ch["node-0"]
    assert out.memory_target == "nps2"
    assert [g.target for g in out.gpus] == [{"cpx_nps2": 8}, {"dpx_nps2": 2}]
    # the next pass reads the written spec: every GPU withheld, the idle one included
    from walkai_nos_amd.partitioning.planner import build_node_partitioning, spec_annotations
    anns = dict(ko.annotations(n))
    anns.update(spec_annotations(build_node_partitioning(out, out.memory_target)))
    anns["nos.nebuly.com/spec-memory-partition"] = "nps2"
    m2 = xn.new_node(ko.new_node("node-0", ko.labels(n), anns))
    assert m2.memory_target == "nps2" and all(g.target is not None for g in m2.gpus)
    with pytest.raises(ValueError):
        m2.gpus[1].add_pod({"spx_nps1": 1})


def test_agent_blocks_every_gpu_while_a_memory_partition_change_waits_for_an_idle_node():
    from walkai_nos_amd.controllers.agent.plan import XcpState, new_xcp_config_plan
    from walkai_nos_amd.models.annotation import SpecAnnotation
    from walkai_nos_amd.models.device import GpuDevice
    state = XcpState([GpuDevice("amd.com/spx_nps1", "g0", "used", 0), GpuDevice("amd.com/spx_nps1", "g1", "free", 1)])
    spec = [SpecAnnotation("cpx_nps2", 0, 8), SpecAnnotation("dpx_nps2", 1, 2)]
    plan = new_xcp_config_plan(state, {0: "spx_nps1", 1: "spx_nps1"}, spec, "nps2", "nps1")
    assert plan.memory_partition is None and plan.changes == []
    assert sorted(g for g, _ in plan.blocked) == [0, 1]


def test_two_planners_with_different_defaults_in_one_process():
    """defaultXcpLayout / sharedSliceSkipCounts are passed to each planner's node
    models, not set as module globals — two planners in one process each see their own."""
    from walkai_nos_amd.api.config import GpuPartitionerConfig
    from walkai_nos_amd.controllers.partitioner.pod_controller import new_node_model
    from walkai_nos_amd.models.defaults import ModelDefaults
    api_ = InMemoryAPIServer()
    api_.create(xnode())                       # no xcp-layout label
    sliced = ModelDefaults.from_config(GpuPartitionerConfig())          # chart default: slices
    parts = ModelDefaults.from_config(GpuPartitionerConfig(defaultXcpLayout="partitions", sharedSliceSkipCounts=[]))
    pa, pb = PodController(api_, defaults=sliced), PodController(api_, defaults=parts)
    n = api_.get("Node", "n0")
    assert new_node_model("xcp", n, defaults=pa.defaults).layout == "slices"
    assert new_node_model("xcp", n, defaults=pb.defaults).layout == "partitions"
    assert new_node_model("xcp", n).layout == "partitions"             # library default
    # interleaved: building one planner's models never changes the other's
    assert pa._models([n])["n0"].layout == "slices"
    assert pb._models([n])["n0"].layout == "partitions"
    assert pa._models([n])["n0"].layout == "slices"
    assert sliced.shared_skip_counts == (5, 7) and parts.shared_skip_counts == ()
    # the node initialiser of each planner uses its own defaults too
    assert NodeInitializer(api_, defaults=sliced).defaults is sliced
