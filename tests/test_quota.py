"""Elastic Resource Quota: calculator, fair-share arithmetic (key-concepts.md worked example),
operator status/labels, and the nos-scheduler borrowing + preemption across 8 simulated MI355X."""
import pytest

from walkai_nos_amd.api import v1alpha1 as api
from walkai_nos_amd.kube import objects as ko
from walkai_nos_amd.kube.memory import InMemoryAPIServer
from walkai_nos_amd.kube.runtime import Request
from walkai_nos_amd.quota.elasticquota import QuotaInfo, QuotaSet, capacity_labels, validate_cluster, validate_quota
from walkai_nos_amd.quota.gpu_memory import GpuMemoryCalculator
from walkai_nos_amd.quota.operator import QuotaOperator
from walkai_nos_amd.sim.cluster import SimCluster

GM = api.RESOURCE_GPU_MEMORY


def eq(name, ns, mn, mx=None, kind=api.KIND_ELASTIC_QUOTA, namespaces=None):
    spec = {"min": {k: str(v) for k, v in mn.items()}}
    if mx is not None:
        spec["max"] = {k: str(v) for k, v in mx.items()}
    if namespaces is not None:
        spec["namespaces"] = namespaces
    return {"apiVersion": api.API_VERSION, "kind": kind, "metadata": {"name": name, "namespace": ns}, "spec": spec}


def test_gpu_memory_calculator():
    c = GpuMemoryCalculator(gpu_resource_memory_gb=288)
    assert c.required_gb({"amd.com/gpu": 1}) == 288
    assert c.required_gb({"amd.com/cpx_nps1": 2}) == 72
    assert c.required_gb({"amd.com/dpx_nps1": 1, "amd.com/gpu-32cu.36gb": 1, "amd.com/gpu-10gb": 2}) == 144 + 36 + 20
    # the reference docs' example: 1g.10gb + 1 nvidia.com/gpu (32 GB) = 42
    assert c.required_gb({"nvidia.com/mig-1g.10gb": 1, "nvidia.com/gpu": 1}) == 42
    pod = ko.new_pod("p", requests={"amd.com/cpx_nps1": 1, "cpu": "2"})
    assert c.pod_request(pod)[GM] == 36


def test_fair_share_worked_example():
    qa = QuotaInfo("a", "a", {"a"}, {GM: 40}, None, {GM: 40})
    qb = QuotaInfo("b", "b", {"b"}, {GM: 10}, None, {GM: 40})
    qc = QuotaInfo("c", "c", {"c"}, {GM: 30}, None, {GM: 0})
    qs = QuotaSet([qa, qb, qc])
    assert qs.available_over_quota(GM) == 30
    assert qs.guaranteed_over_quota(qa, GM) == pytest.approx(15)
    assert qs.guaranteed_over_quota(qb, GM) == pytest.approx(3.75)  # 10/80*30 (docs round to 3)
    assert qs.may_preempt(qa, {GM: 10}, qb)          # 40+10 <= 40+15 and 30 > 3.75
    assert not qs.may_preempt(qa, {GM: 20}, qb)      # 40+20 > 55
    assert not qs.may_preempt(qb, {GM: 10}, qa)      # A is not over its guaranteed share
    assert qs.can_borrow(qc, {GM: 10})               # within min
    assert not qs.can_borrow(qb, {GM: 10})           # B already over min, and 80+10 > 80


def test_validation():
    assert validate_quota(eq("q", "ns", {GM: 10}, {GM: 5}))
    assert not validate_quota(eq("q", "ns", {GM: 10}, {GM: 20}))
    a = QuotaInfo.from_object(eq("a", "ns1", {GM: 1}))
    c = QuotaInfo.from_object(eq("c", "x", {GM: 1}, kind=api.KIND_COMPOSITE_ELASTIC_QUOTA, namespaces=["ns1", "ns2"]))
    assert validate_cluster([a, c]) and not validate_cluster([a])


def test_capacity_labels_creation_order_then_smaller_request():
    q = QuotaInfo("q", "ns", {"ns"}, {GM: 50}, None)
    pods = []
    for name, ts, gm in (("old", "2024-01-01T00:00:00Z", 36), ("tie-big", "2024-01-02T00:00:00Z", 36),
                         ("tie-small", "2024-01-02T00:00:00Z", 10), ("pending", "2024-01-03T00:00:00Z", 10)):
        p = ko.new_pod(name, "ns", requests={GM: gm}, phase="Running" if name != "pending" else "Pending")
        p["metadata"]["creationTimestamp"] = ts
        pods.append(p)
    labels = capacity_labels(pods, q, lambda p: {GM: int(p["spec"]["containers"][0]["resources"]["requests"][GM])})
    assert labels == {"ns/old": "in-quota", "ns/tie-small": "in-quota", "ns/tie-big": "over-quota"}


def test_operator_updates_used_and_labels():
    a = InMemoryAPIServer()
    a.create(eq("qa", "team-a", {GM: 36}))
    for i, phase in enumerate(("Running", "Running", "Pending")):
        a.create(ko.new_pod(f"p{i}", "team-a", requests={"amd.com/cpx_nps1": 1}, phase=phase))
    op = QuotaOperator(a)
    op.reconcile(Request(f"{api.KIND_ELASTIC_QUOTA}|qa", "team-a"))
    q = a.get(api.KIND_ELASTIC_QUOTA, "qa", "team-a")
    assert q["status"]["used"] == {GM: "72"}
    assert q["status"]["conditions"][0]["status"] == "True"
    lbl = {ko.name(p): ko.labels(p).get(api.LABEL_CAPACITY_INFO) for p in a.list("Pod", namespace="team-a")}
    assert lbl == {"p0": "in-quota", "p1": "over-quota", "p2": None}


def test_two_namespaces_borrow_and_reclaim_on_eight_gpus():
    c = SimCluster(n_nodes=1, gpus_per_node=8, kind="cumask", elastic_quota=True)
    c.run(30)
    # each team is guaranteed half of the node's 8 x 288 GB of HBM
    for team in ("team-a", "team-b"):
        c.api.create(eq(f"q-{team}", team, {GM: 4 * 288}))
    c.run(10)
    slice_ = {"amd.com/gpu-128cu.144gb": 1}  # half a GPU
    for i in range(16):  # team-a fills the whole node: 8 slices in quota, 8 borrowed
        c.submit(slice_, name=f"a{i}", namespace="team-a", scheduler_name="nos-scheduler")
    c.run(300)
    running_a = [p for p in c.running_pods() if ko.namespace(p) == "team-a"]
    assert len(running_a) == 16
    over = [p for p in running_a if ko.labels(p).get(api.LABEL_CAPACITY_INFO) == "over-quota"]
    assert len(over) == 8
    qa = c.api.get(api.KIND_ELASTIC_QUOTA, "q-team-a", "team-a")
    assert qa["status"]["used"][GM] == str(16 * 144)
    # team-b claims back its guaranteed share: over-quota pods of team-a are preempted
    for i in range(4):
        c.submit(slice_, name=f"b{i}", namespace="team-b", scheduler_name="nos-scheduler")
    c.run(300)
    running_b = [p for p in c.running_pods() if ko.namespace(p) == "team-b"]
    assert len(running_b) == 4
    assert c.nos_scheduler.preempted >= 4
    assert len([p for p in c.running_pods() if ko.namespace(p) == "team-a"]) == 12
    assert c.utilization() == 100.0


# -- default filter plugins (ref docs/en/docs/elastic-resource-quota/configuration.md:19-42) ----
def _node(name, labels=None, taints=None, unschedulable=False):
    n = ko.new_node(name, labels or {}, allocatable={"cpu": "8", "memory": "8Gi", "pods": "10",
                                                     "amd.com/cpx_nps1": "8"})
    if taints:
        n.setdefault("spec", {})["taints"] = taints
    if unschedulable:
        n.setdefault("spec", {})["unschedulable"] = True
    return n


def test_filters_taints_selectors_affinity():
    from walkai_nos_amd.quota.filters import filter_node, tolerates
    pod = ko.new_pod("p", "default", requests={"amd.com/cpx_nps1": 1})
    gpu_taint = {"key": "amd.com/gpu", "value": "present", "effect": "NoSchedule"}
    assert filter_node(pod, _node("a"))[0]
    assert not filter_node(pod, _node("a", taints=[gpu_taint]))[0]
    assert filter_node(pod, _node("a", taints=[dict(gpu_taint, effect="PreferNoSchedule")]))[0]
    pod["spec"]["tolerations"] = [{"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}]
    assert filter_node(pod, _node("a", taints=[gpu_taint]))[0]
    assert tolerates({"operator": "Exists"}, gpu_taint)                          # tolerate-everything
    assert not tolerates({"key": "amd.com/gpu", "value": "absent"}, gpu_taint)   # Equal needs the value
    assert not filter_node(pod, _node("a", unschedulable=True))[0]
    pod["spec"]["nodeSelector"] = {"pool": "mi355x"}
    assert not filter_node(pod, _node("a"))[0]
    assert filter_node(pod, _node("a", {"pool": "mi355x"}))[0]
    del pod["spec"]["nodeSelector"]
    pod["spec"]["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
        "nodeSelectorTerms": [
            {"matchExpressions": [{"key": "zone", "operator": "In", "values": ["z1", "z2"]},
                                  {"key": "gpus", "operator": "Gt", "values": ["4"]}]},
            {"matchFields": [{"key": "metadata.name", "operator": "In", "values": ["special"]}]}]}}}
    assert filter_node(pod, _node("a", {"zone": "z2", "gpus": "8"}))[0]
    assert not filter_node(pod, _node("a", {"zone": "z2", "gpus": "2"}))[0]
    assert not filter_node(pod, _node("a", {"zone": "z3", "gpus": "8"}))[0]
    assert filter_node(pod, _node("special"))[0]                                 # second term (OR)


def test_nos_scheduler_respects_taints_and_selectors():
    from walkai_nos_amd.quota.scheduler import SCHEDULER_NAME, NosScheduler
    api = InMemoryAPIServer()
    api.create(_node("tainted", {"pool": "a"}, taints=[{"key": "dedicated", "value": "x", "effect": "NoSchedule"}]))
    api.create(_node("plain", {"pool": "b"}))
    s = NosScheduler(api)
    p = ko.new_pod("sel", "default", requests={"amd.com/cpx_nps1": 1}, scheduler_name=SCHEDULER_NAME)
    p["spec"]["nodeSelector"] = {"pool": "a"}
    api.create(p)
    s.reconcile(NosScheduler.KEY)
    pod = api.get("Pod", "sel", "default")
    assert not ko.pod_node_name(pod)                      # only the tainted node matches the selector
    assert "untolerated taint" in pod["status"]["conditions"][0]["message"]
    api.patch("Pod", "sel", {"spec": {"tolerations": [{"key": "dedicated", "operator": "Equal", "value": "x",
                                                       "effect": "NoSchedule"}]}}, "default")
    s.reconcile(NosScheduler.KEY)
    assert ko.pod_node_name(api.get("Pod", "sel", "default")) == "tainted"


def test_erq_on_partitioned_nodes_borrow_reclaim_under_churn():
    """ERQ on the main path — an xcp node under churn, quota ``used`` in
    gpu-memory of partitions; team A borrows all of B's idle share, B reclaims it through
    preemption, and the reclaim latency is measured."""
    from walkai_nos_amd.sim.erq import run_erq_churn
    r = run_erq_churn(gpus=8, epochs=40, b_start=15, seed=3)
    share = r["min_gb_per_team"]
    assert share == 4 * 288
    before = [x for x in r["samples"] if x["epoch"] < 15]
    assert max(x["used_gb"]["team-a"] for x in before) > share          # A borrowed beyond its min
    assert r["preemptions"] > 0 and r["reclaim_latency_s"]["n"] > 0
    assert r["reclaim_latency_s"]["p50"] <= 120.0                        # reclaimed within two minutes
    late = [x for x in r["samples"] if x["epoch"] >= 30]
    assert all(x["used_gb"]["team-a"] <= 2 * share for x in late)
    assert sum(x["used_gb"]["team-b"] for x in late) / len(late) >= 0.6 * share


def test_erq_on_a_sliced_node_under_churn():
    """The same churn on an 8-GPU node of sliced GPUs: B's reclaims evict only the pods on the row
    groups they need and never wait for a flip (profiles/erq_churn_r4_layouts.json: median wait of
    B's pods 12 s vs 180 s on hardware modes, seeds 1-5)."""
    from walkai_nos_amd.sim.erq import run_erq_churn
    r = run_erq_churn(gpus=8, epochs=40, b_start=15, seed=3, layout="slices")
    share = r["min_gb_per_team"]
    before = [x for x in r["samples"] if x["epoch"] < 15]
    assert max(x["used_gb"]["team-a"] for x in before) > share
    assert r["preemptions"] > 0
    assert r["team_b_wait_s"]["p50"] <= 60.0
    late = [x for x in r["samples"] if x["epoch"] >= 30]
    assert sum(x["used_gb"]["team-b"] for x in late) / len(late) >= 0.6 * share


def test_nos_scheduler_frees_a_whole_gpu_for_a_profile_no_node_offers():
    """A reclaiming spx pod on a node whose GPUs are all CPX: the scheduler evicts the pods of the
    GPU the partitioner is draining for spx (all over-quota), not those of a GPU holding an
    in-quota pod, marks the pod quota-reclaim and holds its request against its quota."""
    import json
    from walkai_nos_amd.api import v1alpha1 as v1
    from walkai_nos_amd.quota.scheduler import SCHEDULER_NAME, NosScheduler
    api = InMemoryAPIServer()
    n = _node("n0")
    n["status"]["allocatable"].update({"amd.com/cpx_nps1": "16"})
    anns = {"nos.nebuly.com/status-gpu-0-cpx_nps1-used": "8", "nos.nebuly.com/status-gpu-1-cpx_nps1-used": "8",
            "nos.nebuly.com/status-gpu-2-cpx_nps1-used": "8",
            "nos.nebuly.com/spec-gpu-0-cpx_nps1": "8", "nos.nebuly.com/spec-gpu-1-cpx_nps1": "8",
            "nos.nebuly.com/spec-gpu-2-spx_nps1": "1",
            v1.ANNOTATION_MEMORY_PARTITION_STATUS: "nps1"}
    gpus = {0: [f"team-a/a{i}" for i in range(8)], 1: [f"team-a/a{i}" for i in range(8, 15)] + ["team-c/c0"],
            2: [f"team-a/a{i}" for i in range(15, 23)]}
    anns[v1.ANNOTATION_GPU_PODS_STATUS] = json.dumps({str(g): v for g, v in gpus.items()})
    n["metadata"]["annotations"] = anns
    n["status"]["allocatable"]["amd.com/cpx_nps1"] = "24"
    api.create(n)
    for ns, gb in (("team-a", 288), ("team-b", 288), ("team-c", 288)):
        api.create({"apiVersion": v1.API_VERSION, "kind": v1.KIND_ELASTIC_QUOTA, "metadata": {"name": f"q-{ns}", "namespace": ns},
                    "spec": {"min": {v1.RESOURCE_GPU_MEMORY: str(gb)}}})
    t = 0
    for g, keys in gpus.items():
        for k in keys:
            ns, name = k.split("/")
            p = ko.new_pod(name, ns, requests={"amd.com/cpx_nps1": 1}, scheduler_name=SCHEDULER_NAME)
            p["spec"]["nodeName"] = "n0"
            p["status"]["phase"] = "Running"
            p["metadata"]["creationTimestamp"] = f"2026-01-01T00:00:{t:02d}Z"
            t += 1
            api.create(p)
    s = NosScheduler(api)
    b = ko.new_pod("b0", "team-b", requests={"amd.com/spx_nps1": 1}, scheduler_name=SCHEDULER_NAME)
    api.create(b)
    s.reconcile(NosScheduler.KEY)
    left = {ko.name(p) for p in api.list("Pod", "team-a")}
    assert left == {f"a{i}" for i in range(15)}            # GPU 2 (draining for spx) was freed
    b = api.get("Pod", "b0", "team-b")
    assert ko.annotations(b).get(v1.ANNOTATION_QUOTA_RECLAIM) == "n0" and not ko.pod_node_name(b)
    # a second cycle before the agent reports: GPU 2's pods are gone, so nothing more is evicted,
    # and a new team-A pod cannot borrow the held share
    api.create(ko.new_pod("a99", "team-a", requests={"amd.com/cpx_nps1": 1}, scheduler_name=SCHEDULER_NAME))
    s.reconcile(NosScheduler.KEY)
    assert len(api.list("Pod", "team-a")) == 16 and not ko.pod_node_name(api.get("Pod", "a99", "team-a"))
    assert s.preempted == 8


def test_preemptor_reclaim_timer_dropped_when_the_pod_leaves_the_queue():
    # a preemptor deleted before it binds stops being timed (no unbounded growth of the timer map,
    # no reclaim latency recorded for it)
    from walkai_nos_amd.quota.scheduler import SCHEDULER_NAME, NosScheduler
    api = InMemoryAPIServer()
    api.create(_node("n1", {"pool": "a"}))
    s = NosScheduler(api)
    p = ko.new_pod("waiting", "default", requests={"amd.com/cpx_nps1": 1}, scheduler_name=SCHEDULER_NAME)
    p["spec"]["nodeSelector"] = {"pool": "none"}
    api.create(p)
    s._preempted_for["default/waiting"] = 0.0
    s._preempted_for["default/gone"] = 0.0
    s.reconcile(NosScheduler.KEY)
    assert "default/gone" not in s._preempted_for and not s.reclaim_latency_s
    assert list(s._preempted_for) == ["default/waiting"]
    api.delete("Pod", "waiting", "default")
    s.reconcile(NosScheduler.KEY)
    assert not s._preempted_for


class _GracefulAPI:
    """An API server whose pod deletes are graceful: ``delete`` only sets
    ``metadata.deletionTimestamp``; ``finish()`` removes the terminating pods (kubelet done)."""

    def __init__(self, api):
        self.api = api
        self.deletes = 0

    def __getattr__(self, k):
        return getattr(self.api, k)

    def delete(self, kind, name, namespace=None):
        if kind != "Pod":
            return self.api.delete(kind, name, namespace)
        self.deletes += 1
        self.api.patch("Pod", name, {"metadata": {"deletionTimestamp": "2026-01-01T00:01:00Z"}}, namespace)

    def finish(self):
        for p in self.api.list("Pod"):
            if p["metadata"].get("deletionTimestamp"):
                self.api.delete("Pod", ko.name(p), ko.namespace(p))


def test_preemption_waits_for_terminating_victims():
    """with graceful deletion, victims stay (terminating) for a while; a preemptor must
    not evict more pods while its victims shut down, and no other preemptor may count them."""
    from walkai_nos_amd.quota.scheduler import SCHEDULER_NAME, NosScheduler
    mem = InMemoryAPIServer()
    mem.create(_node("n0"))
    mem.create(eq("qa", "team-a", {GM: 36}))
    mem.create(eq("qb", "team-b", {GM: 7 * 36}))
    for i in range(8):
        p = ko.new_pod(f"a{i}", "team-a", requests={"amd.com/cpx_nps1": 1}, scheduler_name=SCHEDULER_NAME)
        p["spec"]["nodeName"] = "n0"
        p["status"]["phase"] = "Running"
        p["metadata"]["creationTimestamp"] = f"2026-01-01T00:00:{i:02d}Z"
        mem.create(p)
    api = _GracefulAPI(mem)
    s = NosScheduler(api)
    for i in range(2):
        mem.create(ko.new_pod(f"b{i}", "team-b", requests={"amd.com/cpx_nps1": 1}, scheduler_name=SCHEDULER_NAME))
    s.reconcile(NosScheduler.KEY)
    assert api.deletes == 2                                   # one victim per preemptor
    terminating = {ko.name(p) for p in mem.list("Pod", "team-a") if p["metadata"].get("deletionTimestamp")}
    assert len(terminating) == 2
    for _ in range(3):                                        # victims still shutting down
        s.reconcile(NosScheduler.KEY)
    assert api.deletes == 2
    assert not any(ko.pod_node_name(mem.get("Pod", f"b{i}", "team-b")) for i in range(2))
    api.finish()
    s.reconcile(NosScheduler.KEY)
    assert all(ko.pod_node_name(mem.get("Pod", f"b{i}", "team-b")) == "n0" for i in range(2))
    assert api.deletes == 2


def test_erq_bench_mode_reclaims_on_a_sliced_gpu_without_a_flip():
    """VERDICT r3 #7 (control path of ``bench.py --erq``): team A borrows team B's half of a sliced
    GPU with 1/8 pods; B's 1/2 pod reclaims it through 4 evictions of A's over-quota pods and a
    re-carve — no mode flip — within the first reclaim quantum. On hardware partitions the same GPU
    cannot be reclaimed without taking A's guaranteed pods, so B waits (the case slices fix)."""
    from walkai_nos_amd.bench_core import BenchConfig
    from walkai_nos_amd.bench_erq import run_erq
    r = run_erq(BenchConfig(gpus=1, layout="slices"))
    assert r["team_a_borrowed_gb"] == 144 and r["preemptions"] == 4 and r["team_b_bound"]
    assert r["reclaim_quanta"] == 1 and r["flips"] == 0 and r["reclaim_latency_s"]["max"] <= 60
    last = r["samples"][-1]
    assert last["used_gb"] == {"team-a": 144, "team-b": 144} and last["running"] == {"team-a": 4, "team-b": 1}
    p = run_erq(BenchConfig(gpus=1, layout="partitions"), max_reclaim_quanta=3, after_quanta=1)
    assert not p["team_b_bound"] and p["preemptions"] == 0
