"""Elastic Resource Quota with real serving (BASELINE config 5 on the GPUs of one node; ``bench.py
--erq``; ref ``docs/en/docs/elastic-resource-quota/key-concepts.md:30-78``).

Two namespaces hold an ``ElasticQuota`` each whose ``min`` is half the node's HBM in
``nos.nebuly.com/gpu-memory``. Everything runs through the real control plane on the virtual clock
— quota operator, nos-scheduler (CapacityScheduling: borrow while the other team is under its
``min``, preempt over-quota pods to reclaim), partitioner, partition agents and the nos partition
plugin — while every running pod of this rank's GPU serves YOLOS-small inferences on its partition
or CU-mask slice, one at a time, as in the headline bench:

1. **borrow** — team A alone fills the node with 1/8-GPU pods: twice its ``min``, half of it
   borrowed from team B's idle share (the pods beyond A's ``min`` are labelled over-quota);
2. **reclaim** — team B submits its guaranteed share (by default one 1/2-GPU pod per GPU): nos-scheduler
   preempts A's over-quota pods, and the node re-partitions for B — on a sliced GPU the freed
   groups are re-carved into B's slice without a flip;
3. **after** — both teams serve their guaranteed shares.

Reported: inferences/s per namespace in each phase, and the **reclaim latency**, from the
preemption to the preemptor being bound (cluster seconds) — with the number of quanta B waited.
"""
from __future__ import annotations

import collections
import time
from typing import Any, Dict, List, Optional

from .api import v1alpha1 as api
from .bench_core import BenchConfig, DataPlane, pod_keys
from .kube import objects as ko

TEAMS = ("team-a", "team-b")


def _quota(name: str, ns: str, gb: int) -> Dict[str, Any]:
    return {"apiVersion": api.API_VERSION, "kind": api.KIND_ELASTIC_QUOTA, "metadata": {"name": name, "namespace": ns},
            "spec": {"min": {api.RESOURCE_GPU_MEMORY: str(gb)}}}


def run_erq(cfg: BenchConfig, data: Optional[DataPlane] = None, borrow_quanta: int = 4, after_quanta: int = 4,
            max_reclaim_quanta: int = 12, b_profile: str = "dpx_nps1", memory_gb: int = 288) -> Dict[str, Any]:
    """The three phases on ``cfg.gpus`` GPUs of one node; ``data`` (this rank's GPU) serves the pods
    of GPU ``cfg.rank`` — without it only the control plane runs (tests)."""
    from .sim.cluster import SimCluster
    c = SimCluster(n_nodes=1, gpus_per_node=cfg.gpus, refresh_interval=5.0, policy=cfg.policy, elastic_quota=True,
                   xcp_layout=cfg.layout)
    c.run(30)
    share = cfg.gpus * memory_gb // 2
    for team in TEAMS:
        c.api.create(_quota(f"q-{team}", team, share))
    c.run(10)
    sn = next(iter(c.nodes.values()))
    served: Dict[str, Dict[str, int]] = collections.defaultdict(lambda: collections.defaultdict(int))
    wall: Dict[str, float] = collections.defaultdict(float)
    samples: List[Dict[str, Any]] = []
    b_pods = [f"b{i}" for i in range(cfg.gpus)]

    def quantum(phase: str) -> None:
        c.run(cfg.cluster_s)
        keys = pod_keys(sn, cfg.rank)
        t0 = time.perf_counter()
        if data is not None:
            n = data.serve(sorted(set(keys.values())), t0 + cfg.quantum_s)
            data.drain_all()
            for (ns, _), k in keys.items():
                served[phase][ns] += n.get(k, 0) // max(1, sum(1 for v in keys.values() if v == k))
        wall[phase] += time.perf_counter() - t0 if data is not None else cfg.quantum_s
        used = {}
        for team in TEAMS:
            q = c.api.get(api.KIND_ELASTIC_QUOTA, f"q-{team}", team)
            used[team] = int((q.get("status", {}).get("used") or {}).get(api.RESOURCE_GPU_MEMORY, "0"))
        samples.append({"phase": phase, "t": round(c.clock(), 1), "used_gb": used,
                        "running": {t: sum(1 for p in c.running_pods() if ko.namespace(p) == t) for t in TEAMS},
                        "pending": {t: sum(1 for p in c.pending_pods() if ko.namespace(p) == t) for t in TEAMS}})

    # 1. borrow: team A fills every GPU with 1/8 pods (twice its min)
    for i in range(8 * cfg.gpus):
        c.submit({"amd.com/cpx_nps1": 1}, name=f"a{i}", namespace="team-a", scheduler_name="nos-scheduler")
    for _ in range(borrow_quanta):
        quantum("borrow")
    borrowed = samples[-1]["used_gb"]["team-a"] - share
    # 2. reclaim: team B asks for its guaranteed share
    t_submit = c.clock()
    for name in b_pods:
        c.submit({f"amd.com/{b_profile}": 1}, name=name, namespace="team-b", scheduler_name="nos-scheduler")
    reclaim_quanta = 0
    while reclaim_quanta < max_reclaim_quanta:
        quantum("reclaim")
        reclaim_quanta += 1
        if all(ko.pod_node_name(c.api.get("Pod", n, "team-b")) for n in b_pods):
            break
    bound_at = {name: t for t, name, _ in c.binds if name in b_pods}
    # 3. after
    for _ in range(after_quanta):
        quantum("after")
    rates = {ph: {ns: round(v / max(1e-9, wall[ph]), 1) for ns, v in served[ph].items()} for ph in served}
    lat = sorted(c.nos_scheduler.reclaim_latency_s)
    return {
        "mode": "erq", "gpus": cfg.gpus, "layout": cfg.layout, "team_b_profile": b_profile,
        "min_gb_per_team": share, "team_a_borrowed_gb": borrowed,
        "preemptions": c.nos_scheduler.preempted,
        "reclaim_latency_s": {"n": len(lat), "p50": lat[len(lat) // 2] if lat else None,
                              "max": lat[-1] if lat else None},
        "team_b_bound": len(bound_at) == len(b_pods),
        "team_b_wait_s": {n: round(t - t_submit, 1) for n, t in sorted(bound_at.items())},
        "reclaim_quanta": reclaim_quanta, "flips": len(sn.smi.set_calls),
        "inf_per_s": rates, "samples": samples,
        "window": {"cluster_s_per_quantum": cfg.cluster_s, "wall_s_per_quantum": cfg.quantum_s},
    }
