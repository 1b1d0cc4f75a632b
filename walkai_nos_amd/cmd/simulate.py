"""Run the whole nos control plane on the in-process cluster and print utilisation / density per
step (the ``kind``-cluster scenario of BASELINE.json config 1, no GPU needed).

``--scenario churn`` (default) uses the bench's model: one step = ``--cluster-s`` seconds of
cluster time; every compute-partition flip darkens its GPU for ``--flip-cost`` seconds (default:
the measured components), during which it counts as unallocated and its pods neither serve nor
age; ``util_pct`` is that effective allocation; per-profile time-to-schedule is reported.

``--scenario erq``: Elastic Resource Quota on an xcp node under churn (``sim/erq.py``): team A
borrows team B's idle share, team B reclaims it through nos-scheduler preemption; reports the
reclaim latency and each team's ``used`` against its ``min``."""
from __future__ import annotations

import argparse
import json
import logging
import sys
import time

from ..bench_core import BenchConfig, NodeBench


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="nos control-plane simulation")
    ap.add_argument("--gpus", type=int, default=8, help="GPUs per node")
    ap.add_argument("--nodes", type=int, default=1, help="cluster nodes (the planner plans across all of them)")
    ap.add_argument("--epochs", type=int, default=50)
    ap.add_argument("--load", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--policy", default="pack", choices=("pack", "fifo", "batch", "simulate"))
    ap.add_argument("--flip-cost", type=float, default=-1.0, help="seconds per flip (default: measured components)")
    ap.add_argument("--cluster-s", type=float, default=60.0, help="cluster seconds per step")
    ap.add_argument("--preroll", type=int, default=60)
    ap.add_argument("--scenario", default="churn", choices=("churn", "erq"))
    ap.add_argument("--layout", default="partitions", choices=("partitions", "slices", "auto"),
                    help="xcp-layout label of the nodes (churn scenario): hardware modes, sliced GPUs or auto")
    ap.add_argument("--quiet", action="store_true", help="print only the summary line")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.WARNING)
    if args.scenario == "erq":
        from ..sim.erq import run_erq_churn
        r = run_erq_churn(gpus=args.gpus, epochs=args.epochs, seed=args.seed, cluster_s=args.cluster_s,
                          layout=args.layout)
        samples = r.pop("samples")
        if not args.quiet:
            for x in samples:
                print(json.dumps(x))
        print(json.dumps(r))
        return 0
    nb = NodeBench(BenchConfig(gpus=args.gpus, nodes=args.nodes, offered_load=args.load, seed=args.seed,
                               policy=args.policy, flip_cost_s=args.flip_cost, cluster_s=args.cluster_s,
                               layout=args.layout),
                   gpu_data_plane=False)
    for _ in range(args.preroll):
        nb.control_step()
        nb.end_step()
    nb.reset_stats()
    t0 = time.perf_counter()
    for e in range(args.epochs):
        nb.control_step()
        nb.end_step()
        if not args.quiet:
            print(json.dumps({"epoch": e, "util_pct": round(nb.util_samples[-1], 2), "pods": nb.pods_samples[-1],
                              "pending": nb.pending_samples[-1]}))
    dt = time.perf_counter() - t0
    print(json.dumps({"policy": args.policy, "layout": args.layout, "nodes": args.nodes, "gpus_per_node": args.gpus, "load": args.load,
                      "mean_util_pct": round(sum(nb.util_samples) / len(nb.util_samples), 2),
                      "mean_pods_per_node": round(sum(nb.pods_samples) / len(nb.pods_samples) / args.nodes, 2),
                      "pending_mean": round(sum(nb.pending_samples) / len(nb.pending_samples), 2),
                      "pending_max": max(nb.pending_samples), "flips": nb.flips, "flip_cost_s": nb.cfg.flip_cost_s,
                      "time_in_flip_pct": round(100.0 * nb.outage_gpu_quanta / max(1, nb.gpu_quanta), 2),
                      "per_profile": nb.profile_report(args.epochs * nb.cfg.quantum_s),
                      "control_plane_ms_per_epoch": round(1000 * dt / args.epochs, 2)}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
