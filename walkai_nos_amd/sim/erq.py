"""Elastic Resource Quota on compute-partitioned (xcp) nodes under pod churn (ref
``docs/en/docs/elastic-resource-quota/key-concepts.md:30-78``).

Two namespaces each hold an ``ElasticQuota`` whose ``min`` is half of the node's HBM in
``nos.nebuly.com/gpu-memory`` (partition pods are charged their partition's HBM: a CPX pod 36 GB,
DPX 144 GB, SPX 288 GB).  Team A starts alone and offers the whole node's worth of mixed 1/8,
1/2 and 1/1 pods — it borrows team B's idle guaranteed share; from ``b_start`` on team B offers
its own share.  Everything runs through the real control plane on the virtual clock: the quota
operator (``used``, in/over-quota labels), nos-scheduler (CapacityScheduling: borrow while others
are under ``min``, preempt over-quota pods to reclaim), the partitioner and the partition agents.

Reported per quantum and summarised: each team's ``used`` against its ``min``, the node's
allocation, and the **reclaim latency** — from the preemption nos-scheduler makes for a
reclaiming pod to that pod being bound.  A reclaiming pod whose profile no node offers has a whole
GPU freed for it (every pod of one GPU evicted, quota/scheduler.py) and waits for the partitioner
to flip it: every team-B pod's wait (creation -> bound) is reported as ``team_b_wait_s``.
"""
from __future__ import annotations

import math
import random
from typing import Any, Dict, List

from ..api import v1alpha1 as api
from ..kube import objects as ko
from .cluster import SimCluster

MIX = (("cpx_nps1", 0.5), ("dpx_nps1", 0.3), ("spx_nps1", 0.2))
FRACTION = {"cpx_nps1": 1 / 8, "dpx_nps1": 1 / 2, "spx_nps1": 1.0}


def _quota(name: str, ns: str, gb: int) -> Dict[str, Any]:
    return {"apiVersion": api.API_VERSION, "kind": api.KIND_ELASTIC_QUOTA, "metadata": {"name": name, "namespace": ns},
            "spec": {"min": {api.RESOURCE_GPU_MEMORY: str(gb)}}}


def _stats(v: List[float]) -> Dict[str, float]:
    if not v:
        return {"n": 0}
    v = sorted(v)
    return {"n": len(v), "p50": round(v[len(v) // 2], 1), "p99": round(v[min(len(v) - 1, int(0.99 * len(v)))], 1),
            "max": round(v[-1], 1)}


def run_erq_churn(gpus: int = 8, epochs: int = 60, b_start: int = 20, seed: int = 1, cluster_s: float = 60.0,
                  lifetime=(2, 6), load_a: float = 1.0, load_b: float = 0.5, memory_gb: int = 288,
                  layout: str = "partitions") -> Dict[str, Any]:
    """``layout``: the node's ``xcp-layout`` (partitions: hardware modes, a reclaim may need a flip;
    slices: sliced GPUs, a reclaim evicts only the pods on the row groups it needs)."""
    rng = random.Random(seed)
    c = SimCluster(n_nodes=1, gpus_per_node=gpus, kind=api.PARTITIONING_KIND_XCP, elastic_quota=True, policy="pack",
                   xcp_layout=layout)
    c.run(30)
    share = gpus * memory_gb // 2
    for team in ("team-a", "team-b"):
        c.api.create(_quota(f"q-{team}", team, share))
    c.run(10)
    mean_frac = sum(FRACTION[p] * w for p, w in MIX)
    mean_life = (lifetime[0] + lifetime[1]) / 2
    live: Dict[str, float] = {}
    created: Dict[str, float] = {}
    team_of: Dict[str, str] = {}
    seq = 0
    samples: List[Dict[str, Any]] = []
    waits_b: List[float] = []
    seen_bound: set = set()

    def arrivals(load: float) -> List[str]:
        lam = load * gpus / (mean_frac * mean_life)
        n, p, L = 0, 1.0, math.exp(-lam)
        while True:
            p *= rng.random()
            if p <= L:
                break
            n += 1
        out = []
        for _ in range(n):
            r, acc, prof = rng.random(), 0.0, MIX[-1][0]
            for name, w in MIX:
                acc += w
                if r < acc:
                    prof = name
                    break
            out.append(prof)
        return out

    for e in range(epochs):
        now = c.clock()
        for name in [n for n, left in live.items() if left <= 0]:
            del live[name]
            try:
                c.complete(name, team_of[name])
                c.delete_pod(name, team_of[name])
            except Exception:  # noqa: BLE001 - preempted meanwhile
                pass
        batches = [("team-a", load_a)] + ([("team-b", load_b)] if e >= b_start else [])
        for team, load in batches:
            for prof in arrivals(load):
                name = f"{team[-1]}{seq}"
                seq += 1
                c.submit({f"amd.com/{prof}": 1}, name=name, namespace=team, scheduler_name="nos-scheduler")
                created[name], team_of[name] = now, team
        c.run(cluster_s)
        c.clock.set(now + cluster_s)
        running = {ko.name(p): p for p in c.running_pods()}
        for n in list(live):
            if n not in running:
                del live[n]  # preempted: its controller would recreate it later; the churn moves on
        for n in running:
            if n not in live:
                live[n] = float(rng.randint(*lifetime))
        for n in live:
            live[n] -= 1.0
        for t, name, _ in c.binds:
            if name in seen_bound or name not in created:
                continue
            seen_bound.add(name)
            if team_of.get(name) == "team-b":
                waits_b.append(t - created[name])
        used = {}
        for team in ("team-a", "team-b"):
            q = c.api.get(api.KIND_ELASTIC_QUOTA, f"q-{team}", team)
            used[team] = int((q.get("status", {}).get("used") or {}).get(api.RESOURCE_GPU_MEMORY, "0"))
        samples.append({"epoch": e, "util_pct": round(c.utilization(), 1), "used_gb": used,
                        "pending": len(c.pending_pods())})
    s = c.nos_scheduler
    after = [x for x in samples if x["epoch"] >= b_start + 2 * int(mean_life)]
    return {"gpus": gpus, "epochs": epochs, "b_start": b_start, "min_gb_per_team": share,
            "preemptions": s.preempted, "reclaim_latency_s": _stats(s.reclaim_latency_s),
            "team_b_wait_s": _stats(waits_b),
            "util_pct_mean": round(sum(x["util_pct"] for x in samples) / len(samples), 1),
            "team_a_borrowed_gb_before_b": max(x["used_gb"]["team-a"] for x in samples[:b_start]) - share,
            "team_b_used_over_min_after_reclaim": round(
                sum(x["used_gb"]["team-b"] for x in after) / max(1, len(after)) / share, 2),
            "samples": samples}
