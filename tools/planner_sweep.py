"""Planner sweep without a GPU: the bench's control plane and outage model (bench_core.NodeBench with
no data plane) for each policy x GPUs x offered load, 200 quanta after the preroll.

    python tools/planner_sweep.py [--gpus 1,2,4,8] [--loads 0.7,0.85,1.0] [--policies pack,fifo]
        [--steps 200] [--out profiles/planner_sweep_r2.json]
"""
from __future__ import annotations

import argparse
import itertools
import json
import multiprocessing as mp
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(job):
    gpus, load, policy, steps = job
    import logging
    logging.disable(logging.CRITICAL)
    from walkai_nos_amd.bench_core import BenchConfig, NodeBench
    cfg = BenchConfig(gpus=gpus, offered_load=load, policy=policy)
    nb = NodeBench(cfg, gpu_data_plane=False)
    for _ in range(cfg.preroll):
        nb.control_step()
        nb.end_step()
    nb.reset_stats()
    for _ in range(steps):
        nb.control_step()
        nb.end_step()
    n = len(nb.util_samples)
    half = nb.pending_samples[n // 2:]
    return {"policy": policy, "gpus": gpus, "offered_load": load, "steps": steps,
            "util_pct": round(sum(nb.util_samples) / n, 2),
            "util_incl_outage_pct": round(sum(nb.raw_util_samples) / n, 2),
            "flips": nb.flips, "time_in_flip_pct": round(100.0 * nb.outage_gpu_steps / max(1, nb.gpu_steps), 2),
            "pending_mean": round(sum(nb.pending_samples) / n, 2), "pending_max": max(nb.pending_samples),
            "pending_first_half_mean": round(sum(nb.pending_samples[:n // 2]) / (n // 2), 2),
            "pending_second_half_mean": round(sum(half) / len(half), 2),
            "pods_per_gpu": round(sum(nb.pods_samples) / n / gpus, 2)}


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--loads", default="0.7,0.85,1.0")
    ap.add_argument("--policies", default="pack,fifo")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--workers", type=int, default=6)
    ap.add_argument("--out", default="profiles/planner_sweep_r2.json")
    a = ap.parse_args()
    jobs = list(itertools.product([int(g) for g in a.gpus.split(",")], [float(x) for x in a.loads.split(",")],
                                  a.policies.split(","), [a.steps]))
    res = []
    with mp.Pool(a.workers) as pool:
        for r in pool.imap(run, jobs):
            print(json.dumps(r), flush=True)
            res.append(r)
    with open(a.out, "w") as f:
        json.dump(res, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
