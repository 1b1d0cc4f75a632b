"""Run the whole nos control plane on the in-process cluster and print utilisation / density per
step (the ``kind``-cluster scenario of BASELINE.json config 1, no GPU needed).

Uses the bench's outage model: every compute-partition flip darkens its GPU for ``--flip-cost``
seconds (``--quantum`` seconds per step), during which it counts as unallocated and its pods
neither serve nor age; ``util_pct`` is that effective allocation."""
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
    ap.add_argument("--flip-cost", type=float, default=2.0)
    ap.add_argument("--quantum", type=float, default=0.5)
    ap.add_argument("--preroll", type=int, default=60)
    ap.add_argument("--quiet", action="store_true", help="print only the summary line")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.WARNING)
    nb = NodeBench(BenchConfig(gpus=args.gpus, nodes=args.nodes, offered_load=args.load, seed=args.seed,
                               policy=args.policy, flip_cost_s=args.flip_cost, quantum_s=args.quantum),
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
    print(json.dumps({"policy": args.policy, "nodes": args.nodes, "gpus_per_node": args.gpus, "load": args.load,
                      "mean_util_pct": round(sum(nb.util_samples) / len(nb.util_samples), 2),
                      "mean_pods_per_node": round(sum(nb.pods_samples) / len(nb.pods_samples) / args.nodes, 2),
                      "pending_mean": round(sum(nb.pending_samples) / len(nb.pending_samples), 2),
                      "pending_max": max(nb.pending_samples), "flips": nb.flips, "flip_cost_s": args.flip_cost,
                      "time_in_flip_pct": round(100.0 * nb.outage_gpu_steps / max(1, nb.gpu_steps), 2),
                      "control_plane_ms_per_epoch": round(1000 * dt / args.epochs, 2)}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
