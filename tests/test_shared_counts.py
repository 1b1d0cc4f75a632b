"""Memory-only slice counts the planner skips (``models/slicing/profile.py`` SKIP_SHARED_COUNTS):
odd counts from five up split memory-only pods into two rate classes by start order
(``profiles/fair_probe_r5.json``), so the cumask model never leaves 5 or 7 memory-only slices on a
GPU — it carves two at once past them when two pods wait, else the odd pod waits."""
from __future__ import annotations

import pytest

from walkai_nos_amd.api.config import GpuPartitionerConfig
from walkai_nos_amd.controllers.partitioner.pod_controller import plan_cluster_fifo
from walkai_nos_amd.models.slicing import gpu as sg
from walkai_nos_amd.models.slicing import profile as sp


def _gpu(shared_used=4, dedicated_used=0, skip=None):
    used = {"16gb": shared_used} if shared_used else {}
    if dedicated_used:
        used["32cu.24gb"] = dedicated_used
    return sg.SlicingGPU("MI355X", 0, 288, 256, used, {}, skip_shared=skip)


def test_default_skips_five_and_seven():
    assert sp.SKIP_SHARED_COUNTS == (5, 7)
    assert GpuPartitionerConfig().sharedSliceSkipCounts == [5, 7]


def test_a_fifth_memory_only_slice_alone_is_not_carved():
    g = _gpu(4)
    assert not g.update_geometry_for({"16gb": 1})
    assert g.shared_count() == 4 and g.free == {}


def test_two_waiting_pods_pass_the_skipped_count_together():
    g = _gpu(4)
    assert g.update_geometry_for({"16gb": 2})
    assert g.shared_count() == 6 and g.free == {"16gb": 2}
    # from six, the seventh alone is skipped too, two make eight
    g2 = _gpu(6)
    assert not g2.update_geometry_for({"16gb": 1})
    assert g2.update_geometry_for({"16gb": 2}) and g2.shared_count() == 8


def test_counts_below_five_and_dedicated_slices_are_unaffected():
    g = _gpu(0)
    assert g.update_geometry_for({"16gb": 3}) and g.shared_count() == 3
    g = _gpu(4)
    assert g.update_geometry_for({"32cu.24gb": 1}) and g.free == {"32cu.24gb": 1}


def test_skip_list_can_be_disabled_per_gpu_and_per_planner():
    g = _gpu(4, skip=())
    assert g.update_geometry_for({"16gb": 1}) and g.shared_count() == 5
    assert g.clone().skip_shared == ()
    # a planner's ModelDefaults reach every GPU of the node models it builds
    from walkai_nos_amd.kube import objects as ko
    from walkai_nos_amd.api import v1alpha1 as api
    from walkai_nos_amd.models.defaults import ModelDefaults
    node = ko.new_node("n", {api.LABEL_GPU_PARTITIONING: "cumask", "amd.com/gpu.product-name": "AMD_Instinct_MI355X",
                             "amd.com/gpu.count": "2", "amd.com/gpu.vram": "288G"})
    assert [g.skip_shared for g in sg.new_node(node).gpus] == [(5, 7), (5, 7)]
    assert [g.skip_shared for g in sg.new_node(node, ModelDefaults(shared_skip_counts=())).gpus] == [(), ()]


def test_config_rejects_bad_skip_counts():
    with pytest.raises(ValueError):
        GpuPartitionerConfig(sharedSliceSkipCounts=[1]).validate()
    GpuPartitionerConfig(sharedSliceSkipCounts=[]).validate()


def _node(shared_used):
    return sg.SlicingNode("n0", [_gpu(shared_used)])


@pytest.mark.parametrize("waiting,placed", [(1, 0), (2, 2), (3, 2)])
def test_fifo_planner_pairs_pods_past_the_skipped_count(waiting, placed):
    models = {"n0": _node(4)}
    changed = plan_cluster_fifo(models, [{"16gb": 1}] * waiting)
    if not placed:
        assert changed == {}
        return
    g = changed["n0"].gpus[0]
    # the pods the pass placed are "used" in the model; the third waits (7 would split again)
    assert g.used.get("16gb", 0) - 4 == placed and g.shared_count() == 6


def _events(c, reason):
    return [e for e in c.api.list("Event") if e.get("reason") == reason]


def test_a_lone_fifth_memory_only_pod_waits_with_an_event_and_a_sixth_releases_both():
    """End to end on the simulated cumask node: four memory-only pods run, a fifth waits with one
    ``SharedSliceCountSkipped`` event on it (not one per pass), and a sixth arriving lets the planner
    carve both slices at once."""
    from walkai_nos_amd.sim.cluster import SimCluster
    c = SimCluster(n_nodes=1, gpus_per_node=1, kind="cumask")
    c.run(30)
    for i in range(4):
        c.submit({"amd.com/gpu-16gb": 1}, name=f"m{i}")
    c.run(60)
    assert len(c.running_pods()) == 4
    c.submit({"amd.com/gpu-16gb": 1}, name="m4")
    c.run(120)
    assert len(c.running_pods()) == 4 and len(c.pending_pods()) == 1
    ev = _events(c, "SharedSliceCountSkipped")
    assert len(ev) == 1 and ev[0]["involvedObject"]["name"] == "m4" and "5 memory-only pods" in ev[0]["message"]
    c.submit({"amd.com/gpu-16gb": 1}, name="m5")
    c.run(120)
    assert len(c.running_pods()) == 6 and not c.pending_pods()


def test_slice_cap_wait_is_explained_once_per_pod():
    from walkai_nos_amd.sim.cluster import SimCluster
    c = SimCluster(n_nodes=1, gpus_per_node=1, kind="cumask")
    c.run(30)
    for i in range(9):
        c.submit({"amd.com/gpu-8gb": 1}, name=f"m{i}")
    c.run(240)
    assert len(c.running_pods()) == 8
    ev = _events(c, "SliceCapReached")
    assert [e["involvedObject"]["name"] for e in ev] == ["m8"]
