"""Run the whole nos control plane on the in-process cluster and print utilisation / density per
epoch (the ``kind``-cluster scenario of BASELINE.json config 1, no GPU needed)."""
from __future__ import annotations

import argparse
import json
import logging
import sys
import time

from ..bench_core import BenchConfig, NodeBench


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description="nos control-plane simulation")
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--epochs", type=int, default=50)
    ap.add_argument("--load", type=float, default=1.0)
    ap.add_argument("--seed", type=int, default=1234)
    ap.add_argument("--policy", default="fifo", choices=("fifo", "batch", "simulate"))
    ap.add_argument("--quiet", action="store_true", help="print only the summary line")
    args = ap.parse_args(argv)
    logging.basicConfig(level=logging.WARNING)
    nb = NodeBench(BenchConfig(gpus=args.gpus, offered_load=args.load, seed=args.seed, policy=args.policy),
                   gpu_data_plane=False)
    t0 = time.perf_counter()
    for e in range(args.epochs):
        nb.control_step()
        if not args.quiet:
            print(json.dumps({"epoch": e, "util_pct": round(nb.util_samples[-1], 2), "pods": nb.pods_samples[-1],
                              "pending": nb.pending_samples[-1]}))
    dt = time.perf_counter() - t0
    print(json.dumps({"policy": args.policy, "gpus": args.gpus, "mean_util_pct": round(sum(nb.util_samples) / len(nb.util_samples), 2),
                      "mean_pods_per_node": round(sum(nb.pods_samples) / len(nb.pods_samples), 2),
                      "control_plane_ms_per_epoch": round(1000 * dt / args.epochs, 2)}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
