"""The planner's pod-lifetime model (``controllers/partitioner/lifetimes.py``): run times learned from
the pods that finished, conditional residuals of running pods, the Monte Carlo cost of draining a
GPU, the tracker's bookkeeping, and the sliced planner choosing its drain victim by that cost."""
from __future__ import annotations

import random

import pytest

from walkai_nos_amd.controllers.partitioner.lifetimes import LifetimeModel, LifetimeTracker, drain_cost
from walkai_nos_amd.kube import objects as ko


def _model(values, window=256, min_samples=8):
    m = LifetimeModel(window=window, min_samples=min_samples)
    for v in values:
        m.observe(v)
    return m


def test_model_quantiles_readiness_and_window():
    m = _model([100.0, 200.0, 300.0, 400.0], min_samples=8)
    assert not m.ready() and m.n == 4 and m.median() == 300.0 and m.quantile(0.0) == 100.0
    m.observe(-5.0)                       # a non-positive run time is ignored
    assert m.n == 4
    m = _model(range(1, 11), window=4)    # the window keeps the last four observations
    assert m.n == 4 and m.quantile(0.0) == 7 and m.quantile(1.0) == 10
    assert LifetimeModel().median() is None


def test_residuals_are_conditional_on_the_age():
    m = _model([100.0, 200.0, 300.0, 400.0])
    rng = random.Random(0)
    # a pod that ran 250 s finishes at 300 or 400: its residual is 50 or 150, never negative
    draws = {m.sample_residual(250.0, rng) for _ in range(200)}
    assert draws == {50.0, 150.0}
    assert m.expected_residual(250.0) == pytest.approx(100.0)
    assert m.expected_residual(0.0) == pytest.approx(250.0)
    # older than every observation: its age again (at least a second) — a pod that outlived every
    # finished one is evidence of a long tail, not of an imminent end
    assert m.sample_residual(1000.0, rng) == 1000.0 and m.expected_residual(1.0 + 400.0) == pytest.approx(401.0)


def test_drain_cost_basics():
    m = _model([240.0] * 16)
    assert drain_cost([(4, 10.0)], capacity=8, need=4, model=m) == (0.0, 0.0)   # room already there
    # one pod of 8 groups, 100 s into a 240 s run: 140 s with nothing free
    cost, wait = drain_cost([(8, 100.0)], capacity=8, need=8, model=m)
    assert wait == pytest.approx(140.0) and cost == pytest.approx(0.0)
    # two pods of 4: the first frees 4 groups that idle until the second ends
    cost, wait = drain_cost([(4, 200.0), (4, 40.0)], capacity=8, need=8, model=m)
    assert wait == pytest.approx(200.0) and cost == pytest.approx(4 * (200.0 - 40.0))
    # deterministic for a seed, and a bigger need never costs less
    m2 = _model([60.0, 120.0, 240.0, 360.0, 480.0] * 4)
    pods = [(1, 30.0), (2, 100.0), (4, 10.0)]
    assert drain_cost(pods, 8, 4, m2) == drain_cost(pods, 8, 4, m2)
    assert drain_cost(pods, 8, 8, m2)[0] >= drain_cost(pods, 8, 4, m2)[0]


def _pod(name, phase, start=None, finished=None, uid=None):
    p = {"metadata": {"name": name, "namespace": "default", "uid": uid or name},
         "status": {"phase": phase}}
    if start is not None:
        p["status"]["startTime"] = ko.now_rfc3339(start)
    if finished is not None:
        p["status"]["containerStatuses"] = [{"state": {"terminated": {"finishedAt": ko.now_rfc3339(finished)}}}]
    return p


def test_tracker_learns_run_times_from_finished_and_vanished_pods():
    t = LifetimeTracker(_model([], min_samples=1))
    ages = t.update([_pod("a", "Running", start=1000.0), _pod("b", "Running", start=1100.0)], now=1200.0)
    assert ages == {"default/a": pytest.approx(200.0), "default/b": pytest.approx(100.0)}
    # a finishes with a recorded finish time; b vanishes (deleted): its last-seen time counts
    t.update([_pod("a", "Succeeded", start=1000.0, finished=1250.0)], now=1300.0)
    assert sorted(t.model._sorted) == [pytest.approx(100.0), pytest.approx(250.0)]
    assert t.update([], now=1400.0) == {} and t.model.n == 2


def test_terminal_pod_seen_only_after_it_finished_is_learned_once():
    # a pod that starts and finishes between two passes is still a run time (its own
    # startTime to finishedAt), counted once however many passes list it before it is deleted
    t = LifetimeTracker(_model([], min_samples=1))
    done = _pod("c", "Succeeded", start=1000.0, finished=1030.0)
    t.update([done], now=1100.0)
    t.update([done], now=1200.0)
    assert t.model._sorted == [pytest.approx(30.0)]


def test_running_pods_are_censored_observations():
    """30% of the pods never end (long-running inference Deployments). Learning from
    finished pods alone gives the median of the short ones; with the running pods as right-censored
    observations (Kaplan-Meier) the learned median tracks the whole population's, and so do the
    reservation thresholds built on it."""
    rng = random.Random(7)
    t = LifetimeTracker(LifetimeModel(window=4096, min_samples=8))
    pods, now, seq = {}, 0.0, 0
    life = {}
    for step in range(600):                       # one pass every 5 s for 50 minutes
        now = step * 5.0
        for _ in range(2):                        # two pods arrive per pass
            seq += 1
            name = f"p{seq}"
            life[name] = float("inf") if rng.random() < 0.3 else rng.uniform(10.0, 50.0)
            pods[name] = now
        seen = []
        for name, start in list(pods.items()):
            if now - start >= life[name]:
                seen.append(_pod(name, "Succeeded", start=start, finished=start + life[name]))
                del pods[name]
            else:
                seen.append(_pod(name, "Running", start=start))
        t.update(seen, now)
    # the population: 70% uniform(10, 50) s, 30% never end -> median = 10 + 40 * 0.5 / 0.7
    true_median = 10.0 + 40.0 * 0.5 / 0.7
    assert t.model.median() == pytest.approx(true_median, rel=0.06)
    finished_only = LifetimeModel(window=4096)
    for v in t.model._sorted:
        finished_only.observe(v)
    assert finished_only.median() == pytest.approx(30.0, rel=0.06)    # the survival-biased estimate
    # a pod that outlived every finished one is expected to run on (not to end within seconds)
    assert t.model.expected_residual(60.0) >= 60.0
    # the sliced planner's threshold (slice_reserve_lifetimes x the learned median) follows
    from walkai_nos_amd.controllers.partitioner.pod_controller import PackParams
    p = PackParams()
    assert p.slice_reserve_lifetimes * t.model.median() > p.slice_reserve_lifetimes * finished_only.median() * 1.2


def test_drain_cost_counts_groups_the_pod_list_misses():
    # a stale or empty status-pods annotation must not make a busy GPU look free
    m = _model([240.0] * 16)
    assert drain_cost([], capacity=8, need=8, model=m) == (0.0, 0.0)               # no model of use
    cost, wait = drain_cost([], capacity=8, need=8, model=m, used=8)                # all 8 groups in use
    assert wait > 0.0
    # partly listed: the unlisted 4 groups count as a pod that has just started
    _, w_listed = drain_cost([(4, 230.0)], capacity=8, need=8, model=m, used=8)
    assert w_listed == pytest.approx(240.0)


def test_sliced_planner_drains_the_gpu_whose_pods_end_soonest():
    """Two sliced GPUs, neither with room for a whole-GPU pod past its threshold. GPU 0 has fewer
    groups in use but young pods; GPU 1 has more groups in use, all near the end of their run:
    learned lifetimes make GPU 1 the cheaper drain (without them the planner would pick GPU 0)."""
    from walkai_nos_amd.controllers.partitioner.pod_controller import PackParams, plan_cluster_pack
    from walkai_nos_amd.models.partitioned import PartitionedNode
    from walkai_nos_amd.models.xcp import node as xcp_node
    from walkai_nos_amd.models.xcp.slices import new_sliced_gpu

    def node():
        g0 = new_sliced_gpu("MI355X", 0, used={"qpx_nps1": 2}, free={"qpx_nps1": 2})
        g1 = new_sliced_gpu("MI355X", 1, used={"qpx_nps1": 3}, free={"qpx_nps1": 1})
        return PartitionedNode("n", [g0, g1], layout="slices", weight=xcp_node.fraction_weight,
                               is_resource=lambda r: r.startswith("amd.com/"), as_resource=lambda p: "amd.com/" + p)

    pods = {0: [(2, 10.0), (2, 20.0)], 1: [(2, 230.0), (2, 235.0), (2, 225.0)]}
    life = _model([240.0] * 16)
    p = PackParams(slice_reserve_after=900.0, slice_reserve_lifetimes=0.0, slice_free_drain=False)
    pending = [({"spx_nps1": 1}, 1000.0)]
    ch = plan_cluster_pack({"n": node()}, list(pending), params=p, pods_of=lambda n, g: pods[g], life=life)
    targets = [g.target for g in ch["n"].gpus]
    assert targets[1] is not None and targets[0] is None
    ch = plan_cluster_pack({"n": node()}, list(pending), params=p)          # no lifetimes: fewest groups
    targets = [g.target for g in ch["n"].gpus]
    assert targets[0] is not None and targets[1] is None


def test_drain_victim_avoids_hiding_slices_pods_wait_for():
    """On a node of several sliced GPUs a drain withholds its slices in use, and kube-scheduler, which
    still counts their pods, sees as many fewer free slices of those profiles on the node. GPU 0's
    eight 1/8 pods end sooner than GPU 1's four 1/4 pods, but 1/8 pods are waiting: with the strand
    weight the drain goes to GPU 1 (whose profile nobody waits for)."""
    from walkai_nos_amd.controllers.partitioner.pod_controller import PackParams, plan_cluster_pack
    from walkai_nos_amd.models.partitioned import PartitionedNode
    from walkai_nos_amd.models.xcp import node as xcp_node
    from walkai_nos_amd.models.xcp.slices import new_sliced_gpu

    def node():
        g0 = new_sliced_gpu("MI355X", 0, used={"cpx_nps1": 8})
        g1 = new_sliced_gpu("MI355X", 1, used={"qpx_nps1": 4})
        return PartitionedNode("n", [g0, g1], layout="slices", weight=xcp_node.fraction_weight,
                               is_resource=lambda r: r.startswith("amd.com/"), as_resource=lambda p: "amd.com/" + p)

    pods = {0: [(1, 200.0)] * 8, 1: [(2, 150.0)] * 4}
    life = _model([240.0] * 16)
    pending = [({"spx_nps1": 1}, 1000.0), ({"cpx_nps1": 1}, 10.0)]
    for w, want in ((0.0, [True, False]), (1.0, [False, True])):
        p = PackParams(slice_reserve_after=900.0, slice_reserve_lifetimes=0.0, slice_free_drain=False,
                       slice_strand_weight=w)
        ch = plan_cluster_pack({"n": node()}, list(pending), params=p, pods_of=lambda n, g: pods[g], life=life)
        assert [g.target is not None for g in ch["n"].gpus] == want


def test_declared_bounds_cap_the_residuals_of_a_drain():
    # spec.activeDeadlineSeconds: kubelet ends the pod that long after its start, so a pod near its
    # deadline frees its groups soon whatever the learned run times say
    from walkai_nos_amd.controllers.partitioner.lifetimes import declared_bound
    m = _model([600.0] * 32)
    free = drain_cost([(4, 100.0), (4, 100.0)], capacity=8, need=8, model=m)
    near = drain_cost([(4, 100.0, 130.0), (4, 100.0, 160.0)], capacity=8, need=8, model=m)
    assert free[1] == pytest.approx(500.0) and near[1] == pytest.approx(60.0)
    assert near[0] == pytest.approx(4 * 30.0)      # one pod's 4 groups idle from its deadline to the other's
    # a bound already passed: the pod is as good as gone; a loose bound changes nothing
    assert drain_cost([(8, 100.0, 90.0)], capacity=8, need=8, model=m)[1] == 0.0
    assert drain_cost([(4, 100.0, 10_000.0), (4, 100.0)], capacity=8, need=8, model=m) == free
    assert declared_bound({"spec": {"activeDeadlineSeconds": 360}}) == 360.0
    assert declared_bound({"spec": {}}) is None and declared_bound({"spec": {"activeDeadlineSeconds": "x"}}) is None


def test_the_pod_controller_reads_declared_bounds():
    # the sim's pods carry the bound the bench gives them; _gpu_pods hands it to drain_cost
    from walkai_nos_amd.bench_core import BenchConfig, NodeBench
    nb = NodeBench(BenchConfig(gpus=1, layout="slices", declared_bound_quanta=6.0, data_plane=False),
                   gpu_data_plane=False)
    for _ in range(6):
        nb.control_step()
        nb.end_step()
    pods = [p for p in nb.cluster.api.list("Pod") if (p.get("spec") or {}).get("activeDeadlineSeconds")]
    assert pods and all(p["spec"]["activeDeadlineSeconds"] >= 360 for p in pods)
